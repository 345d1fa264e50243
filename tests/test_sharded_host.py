"""CPU tests of the sharded path's host logic (no GPU, no process group).

* kth_sharded_sample_split (include/kth.h): the per-shard sample sizes of the
  single-process sharded select, against a restatement -- rounding, the 64-key
  minimum, the shard cap, totals, bad input.
* kselect.dist.lockstep at P = 8 (the Python mirror of kth_sharded's local
  transport: P shards in one process, all-gather = concatenation, all-reduce =
  sum) with the CPU restatement of the per-rank steps (tests/dist_cpu_backend.py):
  exact k-th of the union for balanced and ragged shards.  The same driver runs
  P = 8 HIP backends on one GPU in tests/test_gpu_config3.py.
"""
import ctypes

import numpy as np
import pytest

import gen as G

FAMS = ["uniform_full", "few_distinct", "sorted_desc", "all_equal"]


def _split(sizes):
    from kselect import LIB
    arr = (ctypes.c_int64 * len(sizes))(*sizes)
    out = (ctypes.c_int64 * len(sizes))()
    total = LIB.kth_sharded_sample_split(arr, len(sizes), out)
    return total, list(out)


def _split_ref(sizes):
    """Restatement of kth_sharded_sample_split (kth_sharded.cpp)."""
    from kselect import LIB
    n = sum(sizes)
    want = int(LIB.kth_dist_sample_size(n))
    s = [min(max(64, int(want * x / n) & ~63), x & ~63) for x in sizes]
    return sum(s), s


@pytest.mark.parametrize("sizes", [
    [1 << 30] * 8,                                  # BASELINE config 3: 8 x 2^30
    [(1 << 30) + 1] * 3 + [(1 << 30)] * 5,          # the reference's block partition of 2^33 + 3
    [1000] * 7 + [(1 << 23) - 7000],                # one big shard, the others small
    [10, (1 << 23) - 10],                           # a shard under 64 keys (0: the gathered path)
    [64, 65, 127, 128, 1 << 20],                    # rounding at the 64-key grain
    [(1 << 20) + 3],                                # one shard
    [3, 5],                                         # tiny union
])
def test_sample_split(sizes):
    total, s = _split(sizes)
    rt, rs = _split_ref(sizes)
    assert (total, s) == (rt, rs), (sizes, total, s, rt, rs)
    for x, si in zip(sizes, s):
        assert si % 64 == 0 and si <= x and (si >= 64 or x < 64)
    if sizes == [1 << 30] * 8:
        assert s == [1 << 17] * 8 and total == 1 << 20  # the single-GPU sample size, split evenly


def test_sample_split_bad_input():
    from kselect import KTH_EINVAL, LIB
    out = (ctypes.c_int64 * 2)()
    assert LIB.kth_sharded_sample_split((ctypes.c_int64 * 2)(5, -1), 2, out) == KTH_EINVAL
    assert LIB.kth_sharded_sample_split((ctypes.c_int64 * 2)(0, 0), 2, out) == KTH_EINVAL
    assert LIB.kth_sharded_sample_split(None, 2, out) == KTH_EINVAL
    assert LIB.kth_sharded_sample_split((ctypes.c_int64 * 1)(5), 0, out) == KTH_EINVAL


def _lockstep_cpu(a, sizes, k, cap=None):
    import torch
    from dist_cpu_backend import CpuBackend
    from kselect.dist import DistSelector, lockstep
    P = len(sizes)
    offs = np.concatenate([[0], np.cumsum(sizes)])
    shards = [torch.from_numpy(np.ascontiguousarray(a[offs[i]:offs[i + 1]])) for i in range(P)]
    sels = [DistSelector(CpuBackend(cap=cap), world=P) for _ in range(P)]
    outs = lockstep(sels, shards, sizes, k)
    got = {int(o[0]) for o in outs}
    assert len(got) == 1, got  # every rank holds the same answer
    return got.pop(), sels[0].b.path


@pytest.mark.parametrize("fam", FAMS)
def test_lockstep_cpu_p8(fam):
    """P = 8 in one process: balanced (the reference's block partition) and
    ragged shards, k at the edges and the middle."""
    from kselect.dist import shard_bounds
    n = (1 << 21) + 13
    a = G.gen(n, G.BY_NAME[fam], 0x5EED0001, 7)
    srt = np.sort(a)
    balanced = [shard_bounds(n, r, 8)[1] for r in range(8)]
    ragged = [70000, 70000, 71000, 70000, 70000, 70000, 72000]  # each at least the per-rank sample
    ragged = [n - sum(ragged)] + ragged
    for sizes in (balanced, ragged):
        assert sum(sizes) == n
        for k in (1, n // 3, n // 2, n):
            got, path = _lockstep_cpu(a, sizes, k)
            assert got == srt[k - 1], (fam, sizes, k, got, srt[k - 1])


def test_lockstep_cpu_p8_fallback():
    """A candidate capacity of 8 keys per rank overflows: the exact fallback levels."""
    n = (1 << 20) + 5
    a = G.gen(n, G.BY_NAME["uniform_full"], 0x5EED0001, 7)
    from kselect.dist import shard_bounds
    sizes = [shard_bounds(n, r, 8)[1] for r in range(8)]
    got, path = _lockstep_cpu(a, sizes, n // 2, cap=8)
    assert got == np.sort(a)[n // 2 - 1] and path == "fallback"


def test_lockstep_refuses_bad_arguments():
    import torch
    from dist_cpu_backend import CpuBackend
    from kselect.dist import DistSelector, lockstep
    sels = [DistSelector(CpuBackend(), world=2) for _ in range(2)]
    sh = [torch.zeros(100000, dtype=torch.int32)] * 2
    with pytest.raises(ValueError):
        lockstep(sels, sh, [100000, 100000], 0)
    with pytest.raises(ValueError):
        lockstep(sels, sh[:1], [100000], 5)
    with pytest.raises(ValueError):  # a shard smaller than the per-rank sample
        lockstep(sels, sh, [100000, 10], 5)
