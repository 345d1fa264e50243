"""BASELINE config 3 (2^33 int32, k = n/2, sharded 8 ways) on the one GPU the
pool gives: every int64 and P = 8 code path of the sharded protocol, on the
device, except the RCCL transport ("P shards on one device ... a
host-side sum standing in for the allreduce").

* One array: kth_select_i32 over 2^33 keys (32 GiB) -- n and k past 2^32, the
  candidates past one workgroup grid's LDS (the streamed finish levels).
* Eight shards x 2^30 on the same device through the product's kth_dist_*
  steps: kth_sharded_* with the device id repeated (the local transport:
  samples gathered in place, each all-reduce a device-side sum of the shards'
  slots), and kselect.dist.lockstep with eight HipBackends (all-gather =
  concatenation, all-reduce = sum; the Python mirror).  Balanced and ragged
  shards; both must equal the one-array answer on the same keys.
* Slot by slot at P = 8 on a small n: the eight device backends in lockstep
  against the eight CPU restatements (tests/dist_cpu_backend.py).

Every 2^33 answer is checked by the exact rank certificate #(<v) < k <= #(<=v),
counted on the device (TODO-kth-problem-cgm.c:45,81-103,135-190 are the int
sizes the reference cannot exceed).
"""
import numpy as np
import pytest

from conftest import load_input

pytestmark = pytest.mark.gpu

N33 = 1 << 33


def _certificate(keys, v):
    import torch
    lt = le = 0
    for c in torch.split(keys, 1 << 30):
        lt += int((c < v).sum())
        le += int((c <= v).sum())
    return lt, le


def _free():
    import torch
    torch.cuda.synchronize()
    torch.cuda.empty_cache()


@pytest.fixture(scope="module")
def keys33(gpu):
    """2^33 uniform_half keys on cuda:0 (32 GiB), the one-array answers of k in
    {1, 2^32, n} (checked by the certificate) -- shared by the shard tests."""
    import torch
    keys = torch.empty(N33, dtype=torch.int32, device="cuda")
    gpu.fill(keys, N33, "uniform_half")
    gpu.sync()
    answers = {}
    for k in (1, N33 // 2, N33):
        v = gpu.select(keys, k)
        lt, le = _certificate(keys, v)
        assert lt < k <= le, (k, v, lt, le, gpu.stats())
        st = gpu.stats()
        assert st["path"] == 3 and st["n"] == N33 and st["k"] == k, st
        answers[k] = v
    yield keys, answers
    del keys
    _free()


def test_one_array_2e33(keys33):
    """kth_select_i32 over 2^33 keys in one array (the fixture checked the
    answers); the k = 2^32 candidates (~0.5 % of n) exceed the LDS-resident finish."""
    keys, answers = keys33
    assert len(answers) == 3


def test_one_array_2e33_adversarial(gpu, keys33):
    """sorted_desc over 2^33 keys (each value twice: the generator wraps at
    2^32) and few_distinct (four values), in the same buffer."""
    keys, answers = keys33
    try:
        for fam in ("sorted_desc", "few_distinct"):
            gpu.fill(keys, N33, fam, param=7)
            gpu.sync()
            for k in (1, N33 // 2, N33):
                v = gpu.select(keys, k)
                lt, le = _certificate(keys, v)
                assert lt < k <= le, (fam, k, v, lt, le, gpu.stats())
                assert gpu.stats()["path"] == 3, (fam, k, gpu.stats())
    finally:  # restore the fixture's keys for the shard tests
        gpu.fill(keys, N33, "uniform_half")
        gpu.sync()


def _views(keys, sizes):
    offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
    return [keys[int(offs[i]):int(offs[i + 1])] for i in range(len(sizes))]


RAGGED_33 = [(1 << 30) + (1 << 29), 1 << 29, (1 << 30) - 12345, (1 << 30) + 12345, 1 << 28,
             (1 << 30) + (1 << 28) - 1000, 1 << 30, 0]
RAGGED_33[-1] = N33 - sum(RAGGED_33[:-1])


@pytest.mark.parametrize("split", ["balanced", "ragged"])
def test_local_shards_2e33(keys33, split):
    """kth_sharded_* with device 0 repeated 8 times: 8 shards of the 2^33 keys,
    n_total = 2^33, k up to 2^33 -- the same answer as the one-array select."""
    import kselect
    keys, answers = keys33
    sizes = [1 << 30] * 8 if split == "balanced" else RAGGED_33
    assert sum(sizes) == N33
    shards = _views(keys, sizes)
    sh = kselect.ShardedSelector([0] * 8)
    try:
        for k, want in answers.items():
            assert sh.select(shards, k, sizes) == want, (split, k)
        assert kselect.select_sharded(shards, N33 // 2, sizes) == answers[N33 // 2]
    finally:
        sh.close()


def test_lockstep_hip_2e33(gpu, keys33):
    """kselect.dist.lockstep with 8 HipBackends (8 ctxs) on one device: the
    DistSelector protocol at P = 8, n_total = 2^33."""
    from kselect import Selector
    from kselect.dist import DistSelector, HipBackend, lockstep
    keys, answers = keys33
    sizes = [1 << 30] * 8
    shards = _views(keys, sizes)
    sels = [Selector(0) for _ in range(8)]
    try:
        ds = [DistSelector(HipBackend(0, s), world=8) for s in sels]
        for k, want in answers.items():
            outs = lockstep(ds, shards, sizes, k)
            got = {int(o.item()) for o in outs}
            assert got == {want}, (k, got, want)
            assert all(d.error() == 0 for d in ds)
    finally:
        for s in sels:
            s.close()


def test_local_shards_small(gpu, oracle):
    """Local transport at P in {2, 3, 8} on 2^24 + 5 keys: families, balanced and
    ragged shards, and a shard under 64 keys (the gather-to-one-buffer path)."""
    import torch
    import kselect
    from kselect.dist import shard_bounds
    n = (1 << 24) + 5
    for fam in ("uniform_full", "few_distinct", "sorted_asc", "all_equal"):
        t = torch.empty(n, dtype=torch.int32, device="cuda")
        gpu.fill(t, n, fam, param=7)
        gpu.sync()
        srt = np.sort(t.cpu().numpy())
        for P in (2, 3, 8):
            sh = kselect.ShardedSelector([0] * P)
            try:
                layouts = [[shard_bounds(n, r, P)[1] for r in range(P)],
                           [n - 200000 * (P - 1)] + [200000] * (P - 1),
                           [10] + [(n - 10) // (P - 1)] * (P - 2) + [(n - 10) - (n - 10) // (P - 1) * (P - 2)]]
                for sizes in layouts:
                    assert sum(sizes) == n
                    shards = _views(t, sizes)
                    for k in (1, n // 3, n // 2, n):
                        assert sh.select(shards, k, sizes) == srt[k - 1], (fam, P, sizes, k)
            finally:
                sh.close()
        del t
    _free()


def test_local_shards_golden(golden):
    """Reference fixtures split by the reference's block partition
    (TODO-kth-problem-cgm.c:81-100) into P = 8 shards on one device: equal to
    the true value and to every terminating mpirun CGM-ref run (P = 8 included)."""
    import torch
    import kselect
    from kselect.dist import shard_bounds
    sh = kselect.ShardedSelector([0] * 8)
    try:
        for c in golden["cases"]:
            a = torch.from_numpy(load_input(c["input"])).cuda()
            sizes = [shard_bounds(a.numel(), r, 8)[1] for r in range(8)]
            got = sh.select(_views(a, sizes), c["k"], sizes)
            assert got == c["true"], c
            for p, v in c["cgm_ref"].items():
                if v != "livelock":
                    assert got == v, (c, p)
    finally:
        sh.close()


@pytest.mark.parametrize("fam", ["uniform_full", "few_distinct", "sorted_desc"])
def test_lockstep_slots_match_cpu_p8(gpu, fam):
    """P = 8: the eight device backends (kth_dist_* on one GPU) and the eight
    CPU restatements, both in lockstep on the same shards (ragged included),
    give the same gathered sample and the same reduced slot after every
    collective, and the same answer."""
    import torch
    from dist_cpu_backend import CpuBackend
    from kselect import Selector
    from kselect.dist import DistSelector, HipBackend, lockstep
    n = (1 << 23) + 77
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu.fill(t, n, fam, param=7)
    gpu.sync()
    host = t.cpu()
    srt = np.sort(host.numpy())
    sels = [Selector(0) for _ in range(8)]
    try:
        for sizes in ([n // 8] * 7 + [n - 7 * (n // 8)], [n - 7 * 300000] + [300000] * 7):
            offs = np.concatenate([[0], np.cumsum(sizes)])
            dsh = [t[int(offs[i]):int(offs[i + 1])] for i in range(8)]
            csh = [host[int(offs[i]):int(offs[i + 1])] for i in range(8)]
            for k in (1, n // 2, n):
                seen_g, seen_c = [], []
                hd = [DistSelector(HipBackend(0, s), world=8) for s in sels]
                cd = [DistSelector(CpuBackend(), world=8) for _ in range(8)]
                og = lockstep(hd, dsh, sizes, k, observe=lambda kind, x: seen_g.append((kind, x.cpu().clone())))
                oc = lockstep(cd, csh, sizes, k, observe=lambda kind, x: seen_c.append((kind, x.clone())))
                torch.cuda.synchronize()
                # one all-gather, then 2 all-reduces (window <= 2^24 wide, or
                # decided by the counts), 3 (wider) or 4 (the exact fallback)
                assert len(seen_g) == len(seen_c) and 3 <= len(seen_g) <= 5, (len(seen_g), len(seen_c))
                for (kg, xg), (kc, xc) in zip(seen_g, seen_c):
                    assert kg == kc and torch.equal(xg, xc), (fam, sizes, k, kg)
                assert {int(o.item()) for o in og} == {int(o[0]) for o in oc} == {int(srt[k - 1])}, (fam, k)
    finally:
        for s in sels:
            s.close()


@pytest.mark.parametrize("fam", ["uniform_half", "few_distinct"])
def test_lockstep_two_allreduces_p8(gpu, fam):
    """The protocol's common case: P = 8 shards of a 2^26-key input whose window
    is at most 2^24 values wide (uniform half-range keys, the bench's family)
    or decided by its counts (few distinct values) -- one all-gather and TWO
    all-reduces, device and CPU restatement slot for slot."""
    import torch
    from dist_cpu_backend import CpuBackend
    from kselect import Selector
    from kselect.dist import DistSelector, HipBackend, lockstep
    n = 1 << 26
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu.fill(t, n, fam, param=7)
    gpu.sync()
    host = t.cpu()
    sizes = [n // 8] * 8
    dsh = [t[i * (n // 8):(i + 1) * (n // 8)] for i in range(8)]
    csh = [host[i * (n // 8):(i + 1) * (n // 8)] for i in range(8)]
    k = n // 2
    want = int(torch.kthvalue(host, k).values)
    sels = [Selector(0) for _ in range(8)]
    try:
        seen_g, seen_c = [], []
        og = lockstep([DistSelector(HipBackend(0, s), world=8) for s in sels], dsh, sizes, k,
                      observe=lambda kind, x: seen_g.append((kind, x.cpu().clone())))
        oc = lockstep([DistSelector(CpuBackend(), world=8) for _ in range(8)], csh, sizes, k,
                      observe=lambda kind, x: seen_c.append((kind, x.clone())))
        torch.cuda.synchronize()
        assert [kd for kd, _ in seen_g] == [kd for kd, _ in seen_c] == ["all_gather", "all_reduce", "all_reduce"]
        for (kg, xg), (kc, xc) in zip(seen_g, seen_c):
            assert torch.equal(xg, xc), (fam, kg)
        assert {int(o.item()) for o in og} == {int(o[0]) for o in oc} == {want}
    finally:
        for s in sels:
            s.close()


def test_dist_error_surfaces(gpu):
    """A grid-barrier timeout in the sharded window (KTH_HOOK_FAULT_BARRIER) leaves
    the answer tensor unwritten, and DistSelector.error() reports it (the
    reused answer buffer must not pass for a fresh answer)."""
    import torch
    import kselect
    from kselect.dist import DistSelector, HipBackend, lockstep
    n = (1 << 23) + 5
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu.fill(t, n, "uniform_full")
    gpu.sync()
    faulty = kselect.Selector(0)
    faulty.test_hook(kselect.KTH_HOOK_FAULT_BARRIER, 1)
    try:
        ds = DistSelector(HipBackend(0, faulty), world=1)
        out = torch.full((1,), 12345, dtype=torch.int32, device="cuda")
        lockstep([ds], [t], [n], n // 2, outs=[out])
        assert ds.error() == 64  # ERR_BARRIER
        assert int(out.item()) == 12345
    finally:
        faulty.close()


@pytest.mark.parametrize("early", ["1", "0"])
def test_dist_level0_pick_error_surfaces(gpu, monkeypatch, early):
    """Level 0's pick fails (the scan's all-reduced slot is tampered with: its
    first-digit histogram zeroed, so no bin holds k) and level 0 was the last
    level: with the early result on (KTH_DIST_EARLY=1, the default) its k_dresult
    must write the error itself -- kth_dist_result does not relaunch after one
    level -- so error() is nonzero and the answer tensor stays untouched; the
    next select on the same ctx is exact again."""
    import torch
    from kselect import KTH_STATS_WORDS
    from kselect.dist import DistSelector, HipBackend, lockstep
    monkeypatch.setenv("KTH_DIST_EARLY", early)
    n = (1 << 23) + 5
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu.fill(t, n, "uniform_full")
    gpu.sync()
    k = n // 2
    want = int(torch.kthvalue(t.cpu(), k).values)
    ds = DistSelector(HipBackend(0, gpu), world=1)
    out = torch.full((1,), 12345, dtype=torch.int32, device="cuda")
    ops = []
    for op in ds.steps(t, n, n, k, out):  # world 1: the collectives are identities
        ops.append(op[0])
        if op[0] == "all_gather":
            op[1].copy_(op[2])
        elif ops.count("all_reduce") == 1:  # the scan's slot: counts kept, digit histogram zeroed
            op[1][8:KTH_STATS_WORDS] = 0
    assert ops == ["all_gather", "all_reduce", "all_reduce"], ops  # the error ends the protocol after level 0
    assert ds.error() != 0
    assert int(out.item()) == 12345
    assert int(lockstep([ds], [t], [n], k, outs=[out])[0].item()) == want
    assert ds.error() == 0
