"""GPU tests of the library's ordering and residency guarantees.

* One process runs the single-process sharded entry (kth_sharded_*, its own
  non-blocking streams and an ncclCommInitAll communicator on device 0) and then
  world-1 DistSelectors (direct RCCL and torch.distributed collectives, on
  torch's default stream and on a private stream), and the same in the reverse
  order.  Round 2 saw a stale answer here: the answer tensor was read by torch
  before the select that writes it had run, because libkth.so had been loaded
  with /opt/rocm's HIP runtime next to torch's own (two null streams).  kselect
  now loads one runtime (tests/test_abi.py pins that on the CPU) and these tests
  pin the GPU behaviour in both orders.
* A cooperative window select followed by a sharded select on the SAME ctx: the
  window select leaves its count slot and candidate count for its next k_head
  to clear, so the sharded steps must clear them (kth_dist_begin).
* Grid-barrier timeouts (the test-only KTH_HOOK_FAULT_BARRIER): reported in the state, d_out left
  untouched by the asynchronous entry, and the synchronous entry redoes the
  select on the per-level path.
"""
import contextlib

import numpy as np
import pytest

from conftest import load_input

pytestmark = pytest.mark.gpu


@contextlib.contextmanager
def _world1():
    """A one-rank RCCL group over an in-process HashStore: no TCP rendezvous, so
    no port to race for (round 4's driver run lost a probed port to EADDRINUSE)."""
    import torch
    import torch.distributed as dist
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0),
                            store=dist.HashStore())
    try:
        yield
    finally:
        dist.destroy_process_group()


def _keys(gpu, n, fam):
    import torch
    t = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu.fill(t, n, fam, param=7)
    gpu.sync()
    return t, np.sort(t.cpu().numpy())


def _dist_checks(gpu, fams=("uniform_full", "few_distinct", "sorted_desc"), n=1 << 23):
    """World-1 DistSelector: RCCL and torch comms on the default stream, then
    RCCL on a private stream; every answer read with .item() right after."""
    import torch
    from kselect.dist import DistSelector, HipBackend
    from kselect.rccl import RcclComm, TorchComm
    data = {f: _keys(gpu, n, f) for f in fams}
    b = HipBackend(0)
    for comm in (None, TorchComm()):
        ds = DistSelector(b, comm=comm)
        assert isinstance(ds.comm, RcclComm if comm is None else TorchComm)
        for fam, (keys, srt) in data.items():
            for k in (1, n // 2, n):
                got = int(ds.select(keys, n, n, k).item())
                assert got == srt[k - 1], (fam, k, type(ds.comm).__name__, b.sel.stats())
        ds.close()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        bp = HipBackend(0)
        ds = DistSelector(bp)
        for fam, (keys, srt) in data.items():
            for k in (1, n // 2, n):
                got = int(ds.select(keys, n, n, k).item())
                assert got == srt[k - 1], (fam, k, "private stream", bp.sel.stats())
        ds.close()
    torch.cuda.current_stream().wait_stream(s)


def _sharded_checks(golden, gpu):
    import torch
    import kselect
    sh = kselect.ShardedSelector([0])
    try:
        for c in golden["cases"][::7]:
            a = torch.from_numpy(load_input(c["input"])).cuda()
            assert sh.select([a], c["k"]) == c["true"], c
        keys, srt = _keys(gpu, (1 << 23) + 5, "uniform_half")
        for k in (1, keys.numel() // 2, keys.numel()):
            assert sh.select([keys], k) == srt[k - 1]
            assert kselect.select_sharded([keys], k) == srt[k - 1]
    finally:
        sh.close()


def test_sharded_then_dist_world1(gpu, golden):
    """The order that failed in round 2: the sharded handle first."""
    import kselect
    assert len(kselect.hip_runtimes()) == 1, kselect.hip_runtimes()
    _sharded_checks(golden, gpu)
    with _world1():
        _dist_checks(gpu)


def test_dist_world1_then_sharded(gpu, golden):
    with _world1():
        _dist_checks(gpu, fams=("uniform_half", "mod_1000"))
    _sharded_checks(golden, gpu)


def test_window_select_then_dist_on_same_ctx(gpu):
    """A cooperative window select leaves islot(1) and the candidate count for
    its next k_head; a sharded select on the same ctx must not append after the
    stale count (the candidate levels would see the previous select's keys)."""
    import kselect
    from kselect.dist import DistSelector, HipBackend
    sel = kselect.Selector(0)
    n = (1 << 23) + 13
    a, srt_a = _keys(gpu, n, "uniform_full")
    b, srt_b = _keys(gpu, n, "uniform_half")
    with _world1():
        hb = HipBackend(0, sel)
        ds = DistSelector(hb)
        for k in (n // 2, n // 3, 1, n):
            assert sel.select(a, k) == srt_a[k - 1]  # window path: k_head + k_main + k_finish
            got = int(ds.select(b, n, n, k).item())
            assert got == srt_b[k - 1], (k, sel.stats())
            assert sel.select(a, k) == srt_a[k - 1]
        ds.close()
    sel.close()


@pytest.fixture
def faulty():
    import kselect
    f = kselect.Selector(0)
    f.test_hook(kselect.KTH_HOOK_FAULT_BARRIER, 1)
    yield f
    f.close()


def test_coop_backoff_counts_every_entry_point(gpu):
    """One grid-barrier timeout (KTH_HOOK_FAULT_BARRIER, value 2: once) turns the cooperative
    kernels off for COOP_BACKOFF = 64 selections; asynchronous selects count
    down too, so a ctx used only asynchronously afterwards gets them back."""
    import torch
    import kselect
    sel = kselect.Selector(0)
    sel.test_hook(kselect.KTH_HOOK_FAULT_BARRIER, 2)
    try:
        n = (1 << 24) + 3
        keys, srt = _keys(gpu, n, "uniform_full")
        assert sel.coop()
        assert sel.select(keys, n // 2) == srt[n // 2 - 1]  # times out once, redone per level
        assert not sel.coop()
        out = torch.zeros(1, dtype=torch.int32, device="cuda")
        for i in range(63):
            sel.select_async(keys, n, n // 3, out)
            assert not sel.coop(), i
        sel.select_async(keys, n, n // 3, out)  # the 64th: cooperative again
        assert sel.coop()
        sel.sync()
        assert int(out.item()) == srt[n // 3 - 1] and sel.stats()["error"] == 0
    finally:
        sel.close()


@pytest.mark.parametrize("n", [(1 << 20) + 7, (1 << 24) + 3])  # radix path (k_finish only), window path
def test_barrier_timeout_reported_and_out_untouched(gpu, faulty, n):
    import torch
    keys, srt = _keys(gpu, n, "uniform_full")
    out = torch.full((1,), 12345, dtype=torch.int32, device="cuda")
    faulty.select_async(keys, n, n // 2, out)
    faulty.sync()
    st = faulty.stats()
    assert st["error"] == 64, st  # ERR_BARRIER
    assert int(out.item()) == 12345  # the unverified answer never reaches d_out
    # the synchronous entry redoes the select on the per-level path
    for k in (1, n // 2, n):
        assert faulty.select(keys, k) == srt[k - 1]
    # a healthy ctx is unaffected
    assert gpu.select(keys, n // 2) == srt[n // 2 - 1]
