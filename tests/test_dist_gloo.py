"""Multi-process CPU tests of the sharded path (one process per 'GPU').

The product's orchestration, kselect.dist.DistSelector, runs unchanged on the
gloo backend with world_size 2 and 3; the per-rank device steps are replaced by
their CPU restatement (tests/dist_cpu_backend.py).  Checks: every rank returns
the exact k-th smallest of the union of the shards (block partition of
TODO-kth-problem-cgm.c:81-100), across families, edge ranks, ragged shards and
the window-fallback path.
"""
import os
import sys
import tempfile

import numpy as np
import pytest
import torch.multiprocessing as mp

HERE = os.path.dirname(os.path.abspath(__file__))


def _rdv():
    """A fresh file:// rendezvous: the ranks meet through a FileStore, so no TCP
    port is probed and then raced for (round 4's EADDRINUSE)."""
    return "file://" + os.path.join(tempfile.mkdtemp(prefix="kth_rdv_"), "store")


def _worker(rank, world, rdv, cases, q, host_comm=False):
    sys.path.insert(0, HERE)
    from conftest import PKG  # noqa: F401 -- sets sys.path for kselect and gen
    import torch
    import torch.distributed as dist

    import gen as G
    from dist_cpu_backend import CpuBackend
    from kselect.dist import DistSelector, shard_bounds
    from kselect.rccl import HostComm

    dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
    try:
        out = []
        for fam, param, n, ks, cap in cases:
            # host_comm: the shared-GPU transport (KTH_SHARE_GPU=1) -- its host
            # staging is a copy here, its collectives the same gloo ops
            ds = DistSelector(CpuBackend(cap=cap), comm=HostComm() if host_comm else None)
            start, cnt = shard_bounds(n, rank, world)
            shard = torch.from_numpy(G.gen(cnt, G.BY_NAME[fam], 0x5EED0001, param, offset=start, n_total=n))
            for k in ks:
                got = int(ds.select(shard, cnt, n, k)[0])
                out.append((fam, n, k, got, getattr(ds.b, "path", "small")))
                ds.b.path = "small"  # reset: the next select sets it again unless it takes the small path
        q.put((rank, out))
    finally:
        dist.destroy_process_group()


def _run(world, cases, host_comm=False):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    rdv = _rdv()
    procs = [ctx.Process(target=_worker, args=(r, world, rdv, cases, q, host_comm)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return res


def _expected(fam, param, n):
    import gen as G
    return np.sort(G.gen(n, G.BY_NAME[fam], 0x5EED0001, param, n_total=n).astype(np.int64))


CASES = [
    ("uniform_full", 0, 7, None, None),      # fewer keys than ranks on some ranks: all-gather path
    ("few_distinct", 0, 100, None, None),
    ("uniform_full", 0, 600_001, None, None),
    ("uniform_half", 0, 400_000, None, None),
    ("few_distinct", 0, 300_000, None, None),
    ("all_equal", 7, 300_000, None, None),
    ("sorted_desc", 0, 500_000, None, None),
    ("mod_1000", 0, 300_000, None, None),
]


@pytest.mark.parametrize("world", [2, 3])
def test_dist_selector_gloo(world):
    cases = []
    for fam, param, n, _, cap in CASES:
        ks = sorted({k for k in (1, 2, n // 3, n // 2, n - 1, n) if 1 <= k <= n})
        cases.append((fam, param, n, ks, cap))
    res = _run(world, cases)
    by_rank = [res[r] for r in range(world)]
    assert all(len(b) == len(by_rank[0]) for b in by_rank)
    i = 0
    for fam, param, n, ks, _ in cases:
        srt = _expected(fam, param, n)
        for k in ks:
            answers = {by_rank[r][i][3] for r in range(world)}
            assert answers == {int(srt[k - 1])}, (fam, n, k, answers, int(srt[k - 1]))
            i += 1


def test_dist_selector_host_comm():
    """DistSelector over kselect.rccl.HostComm (the transport of ranks sharing
    one GPU, bench.py KTH_SHARE_GPU=1) at world 2: the same exact answers, the
    small-input gather path included."""
    cases = [(fam, param, n, sorted({1, n // 2, n}), cap) for fam, param, n, _, cap in
             (CASES[0], CASES[2], CASES[4], CASES[6])]
    res = _run(2, cases, host_comm=True)
    i = 0
    for fam, param, n, ks, _ in cases:
        srt = _expected(fam, param, n)
        for k in ks:
            assert {res[r][i][3] for r in range(2)} == {int(srt[k - 1])}, (fam, n, k)
            i += 1


def test_dist_selector_gloo_fallback():
    """Candidate capacity forced tiny: the window overflows on every rank and the
    selection finishes through the full-shard radix levels, still exact."""
    n = 500_000
    cases = [("uniform_full", 0, n, [1, n // 2, n], 16)]
    res = _run(2, cases)
    srt = _expected("uniform_full", 0, n)
    for r in range(2):
        for (fam, nn, k, got, mode), kk in zip(res[r], [1, n // 2, n]):
            assert got == int(srt[kk - 1]), (k, got)
    paths = {m for r in range(2) for *_, m in res[r]}
    assert paths == {"fallback"}


def _bad_worker(rank, world, rdv, q):
    sys.path.insert(0, HERE)
    from conftest import PKG  # noqa: F401
    import torch
    import torch.distributed as dist

    from dist_cpu_backend import CpuBackend
    from kselect.dist import DistSelector

    dist.init_process_group("gloo", init_method=rdv, rank=rank, world_size=world)
    try:
        ds = DistSelector(CpuBackend())
        errs = []
        n = 400_000
        # rank 1 holds a shard smaller than its sample share: every rank must
        # raise together (no rank left waiting in a collective)
        sizes = [n - 100, 100]
        shard = torch.arange(sizes[rank], dtype=torch.int32)
        for args in ((shard, sizes[rank], n, n // 2),                        # unbalanced
                     (shard, sizes[rank], n + rank, n // 2),                 # n_total disagrees
                     (torch.arange(n // 2, dtype=torch.int32), n // 2, n + 5, 7)):  # sizes do not sum
            try:
                ds.select(*args)
                errs.append(None)
            except ValueError as e:
                errs.append(str(e)[:40])
        q.put((rank, errs))
    finally:
        dist.destroy_process_group()


def test_dist_selector_bad_arguments_raise_on_every_rank():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    rdv = _rdv()
    procs = [ctx.Process(target=_bad_worker, args=(r, 2, rdv, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(2))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in range(2):
        assert all(e is not None for e in res[r]), res
    assert res[0] == res[1]
