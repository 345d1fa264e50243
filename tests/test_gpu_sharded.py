"""GPU tests of the sharded paths on the one-GPU box.

* kth_select_i32_sharded / kth_sharded_* (single process, RCCL communicators from
  ncclCommInitAll; include/kth.h) at ngpu = 1: golden reference fixtures and
  synthetic families against the oracle's order statistic.
* The gloo tests' CPU restatement of the per-rank steps (tests/dist_cpu_backend.py)
  against the device steps (kth_dist_* through kselect.dist.HipBackend) at world
  1: identical samples and identical stats slots after the scan and every level,
  so the multi-rank gloo runs exercise the arithmetic a GPU run performs.
"""
import numpy as np
import pytest

from conftest import load_input

pytestmark = pytest.mark.gpu

FAMS = ["uniform_full", "uniform_half", "few_distinct", "all_equal", "sorted_desc", "mod_1000"]


def _dev_keys(gpu, n, fam, param=7):
    import torch
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu.fill(keys, n, fam, param=param)
    gpu.sync()
    return keys


@pytest.fixture(scope="module")
def sharded():
    import kselect
    s = kselect.ShardedSelector([0])
    yield s
    s.close()


def test_sharded_golden(sharded, golden):
    """Reference-generated fixtures (seq and mpirun CGM outputs): n <= 16384 --
    shards under 64 keys take the gather-to-device-0 path, the rest the protocol."""
    import torch
    for c in golden["cases"]:
        a = torch.from_numpy(load_input(c["input"])).cuda()
        got = sharded.select([a], c["k"])
        assert got == c["true"], c
        for p, v in c["cgm_ref"].items():
            if v != "livelock":
                assert got == v, (c, p)


@pytest.mark.parametrize("n", [(1 << 20) + 3, (1 << 24) + 5])
def test_sharded_families(gpu, sharded, n):
    import kselect
    for fam in FAMS:
        keys = _dev_keys(gpu, n, fam)
        srt = np.sort(keys.cpu().numpy())
        for k in (1, n // 3, n // 2, n):
            assert sharded.select([keys], k) == srt[k - 1], (fam, n, k)
            assert kselect.select_sharded([keys], k) == srt[k - 1], (fam, n, k)


def test_sharded_errors(gpu, sharded):
    import kselect
    import torch
    keys = torch.zeros(1000, dtype=torch.int32, device="cuda")
    for k in (0, 1001):
        with pytest.raises(kselect.KthError) as e:
            sharded.select([keys], k)
        assert e.value.code == kselect.KTH_EINVAL
    with pytest.raises(kselect.KthError) as e:  # host memory is not a shard
        kselect.select_sharded([np.zeros(1000, dtype=np.int32)], 5)
    assert e.value.code == kselect.KTH_EINVAL
    with pytest.raises(kselect.KthError) as e:  # the local transport holds at most 64 shards
        kselect.ShardedSelector([0] * 65)
    assert e.value.code == kselect.KTH_EINVAL
    if _ndev() >= 2:  # a device repeated among others: neither RCCL (one rank per device) nor local
        with pytest.raises(kselect.KthError) as e:
            kselect.ShardedSelector([0, 1, 0])
        assert e.value.code == kselect.KTH_EINVAL


@pytest.mark.parametrize("fam", FAMS)
def test_dist_backend_slots_match(gpu, fam):
    """HipBackend (device) and CpuBackend (the gloo tests' restatement) step by
    step on the same shard at world 1: same sample, same slots, same answer."""
    import torch
    from dist_cpu_backend import CpuBackend
    from kselect import KTH_DIST_DONE, KTH_DIST_MAX_LEVELS
    from kselect.dist import HipBackend
    n = (1 << 23) + 77
    keys = _dev_keys(gpu, n, fam)
    host = keys.cpu()
    hb, cb = HipBackend(0, gpu), CpuBackend()
    s = max(64, (hb.sample_size(n) // 1) & ~63)
    assert s == max(64, (cb.sample_size(n) // 1) & ~63)
    for k in (1, n // 2, n):
        sg, sc = hb.alloc_slots(), cb.alloc_slots()
        hb.begin(sg, n, k)
        cb.begin(sc, n, k)
        smp_g, smp_c = hb.alloc_sample(s), cb.alloc_sample(s)
        hb.sample(keys, n, smp_g, s)
        cb.sample(host, n, smp_c, s)
        torch.cuda.synchronize()
        assert torch.equal(smp_g.cpu(), smp_c), (fam, k, "sample")
        hb.window(smp_g, s)
        cb.window(smp_c, s)
        i, j = hb.scan(keys, n), cb.scan(host, n)
        torch.cuda.synchronize()
        assert i == j and torch.equal(sg[i].cpu(), sc[j]), (fam, k, "scan", sg[i][:5].tolist(), sc[j][:5].tolist())
        for level in range(KTH_DIST_MAX_LEVELS + 1):  # until KTH_DIST_DONE (the same call on both)
            i, j = hb.level(keys, n, level), cb.level(host, n, level)
            torch.cuda.synchronize()
            assert i == j, (fam, k, "level", level, i, j)
            if i == KTH_DIST_DONE:
                break
            assert torch.equal(sg[i].cpu(), sc[j]), (fam, k, "level", level)
        else:
            raise AssertionError("no KTH_DIST_DONE")
        og, oc = hb.alloc_out(), cb.alloc_out()
        hb.result(og)
        cb.result(oc)
        torch.cuda.synchronize()
        assert int(og.item()) == int(oc.item()) == int(np.sort(host.numpy())[k - 1]), (fam, k)


# --------------------------------------------- more than one device (skip on 1)
def _ndev():
    import torch
    return torch.cuda.device_count()


needs2 = pytest.mark.skipif("_ndev() < 2", reason="needs >= 2 GPUs (runs on the driver's multi-GPU node)")


def _split(a, devs, sizes=None):
    """Block partition of TODO-kth-problem-cgm.c:81-100 (or explicit sizes),
    shard i copied to device devs[i]."""
    import torch
    from kselect.dist import shard_bounds
    P = len(devs)
    if sizes is None:
        sizes = [shard_bounds(a.size, i, P)[1] for i in range(P)]
    offs = np.concatenate([[0], np.cumsum(sizes)])
    return [torch.from_numpy(np.ascontiguousarray(a[offs[i]:offs[i + 1]])).to(f"cuda:{d}")
            for i, d in enumerate(devs)], sizes


@needs2
def test_sharded_multi_device_golden(golden):
    """ShardedSelector over every visible device: reference fixtures split by
    the reference's block partition (shards under 64 keys: the peer-copy gather
    to device 0, select_gathered), against seq-ref / CGM-ref / true values."""
    import kselect
    devs = list(range(_ndev()))
    sh = kselect.ShardedSelector(devs)
    try:
        for c in golden["cases"]:
            a = load_input(c["input"])
            shards, sizes = _split(a, devs)
            got = sh.select(shards, c["k"], sizes)
            assert got == c["true"], c
            for p, v in c["cgm_ref"].items():
                if v != "livelock":
                    assert got == v, (c, p)
    finally:
        sh.close()


@needs2
@pytest.mark.parametrize("fam", ["uniform_full", "few_distinct", "sorted_asc", "all_equal"])
def test_sharded_multi_device_families(gpu, fam):
    """2^24 + 5 keys over every device, balanced; k in {1, n/3, n/2, n}."""
    import torch
    import kselect
    devs = list(range(_ndev()))
    n = (1 << 24) + 5
    t = torch.empty(n, dtype=torch.int32, device="cuda:0")
    gpu.fill(t, n, fam, param=7)
    gpu.sync()
    a = t.cpu().numpy()
    srt = np.sort(a)
    shards, sizes = _split(a, devs)
    sh = kselect.ShardedSelector(devs)
    try:
        for k in (1, n // 3, n // 2, n):
            assert sh.select(shards, k, sizes) == srt[k - 1], (fam, k)
            assert kselect.select_sharded(shards, k, sizes) == srt[k - 1], (fam, k)
    finally:
        sh.close()


@needs2
def test_sharded_multi_device_ragged():
    """Unbalanced shards: the per-device sample is weighted by shard size (a
    gatherv of broadcasts), and one shard under 64 keys takes the peer-copy
    gather to device 0."""
    import kselect
    devs = list(range(_ndev()))
    P = len(devs)
    rng = np.random.default_rng(17)
    n = 1 << 23
    a = rng.integers(-2 ** 31, 2 ** 31, size=n, dtype=np.int64).astype(np.int32)
    srt = np.sort(a)
    sh = kselect.ShardedSelector(devs)
    try:
        # one big shard, the others 1000 keys
        sizes = [1000] * (P - 1) + [n - 1000 * (P - 1)]
        shards, sizes = _split(a, devs, sizes)
        for k in (1, n // 2, n):
            assert sh.select(shards, k, sizes) == srt[k - 1], ("ragged", k)
        # one shard of 10 keys: select_gathered
        sizes = [10] + [0] * (P - 2) + [n - 10] if P > 2 else [10, n - 10]
        shards, sizes = _split(a, devs, sizes)
        for k in (1, n // 2, n):
            assert sh.select(shards, k, sizes) == srt[k - 1], ("tiny shard", k)
    finally:
        sh.close()


@needs2
def test_bench_two_gpus():
    """bench.py --gpus 2 launches two ranks over RCCL and verifies the answer."""
    import json
    import subprocess
    import sys
    from conftest import REPO
    p = subprocess.run([sys.executable, "bench.py", "--gpus", "2", "--log2n", "24", "--steps", "3", "--warmup", "1",
                        "--no-cpu-baseline"], cwd=REPO, capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["verified"] is True and line["n_gpus"] == 2 and line["config"]["rccl_world"] == 2, line


# ------------------------------------------------------- full size, one device
def test_sharded_full_size_rank_certificate(gpu):
    """kth_select_i32_sharded at 2^30 keys on one device (BASELINE config 2's
    size through the sharded entry): the answer v satisfies the exact rank
    certificate #(< v) < k <= #(<= v), counted on the device."""
    import torch
    import kselect
    n = 1 << 30
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu.fill(keys, n, "uniform_half")
    gpu.sync()
    for k in (1, n // 2, n):
        v = kselect.select_sharded([keys], k)
        lt = int((keys < v).sum().item())
        le = int((keys <= v).sum().item())
        assert lt < k <= le, (k, v, lt, le)
    del keys
    torch.cuda.empty_cache()
