"""GPU parity for the single-array top-k (kth_topk_i32).

Contract (include/kth.h): the k smallest (largest) int32 keys with their int64
indices, in index order; of the keys equal to the k-th, the first ones by
index.  The reference implies this as sort(a)[:k] after its select block
(kth-problem-seq.c:32-33); the restatement here is numpy's stable argsort
(ties by index) re-sorted into index order.  Integer work: bit-exact.
Large sizes are checked through size-independent properties (index order,
vals == keys[idx], everything kept <= the k-th <= everything dropped, the tie
quota taken first-by-index)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _ref_idx(a, k, largest):
    order = -a.astype(np.int64) if largest else a.astype(np.int64)
    return np.sort(np.argsort(order, kind="stable")[:k])


def _run(gpu, d, n, k, largest, with_vals=True, with_idx=True):
    import torch
    vals = torch.empty(k, dtype=torch.int32, device=d.device) if with_vals else None
    idx = torch.empty(k, dtype=torch.int64, device=d.device) if with_idx else None
    gpu.topk(d, n, k, vals, idx, largest=largest)
    gpu.sync()
    return vals, idx


def _inputs(n, seed):
    rng = np.random.default_rng(seed)
    yield "uniform_full", rng.integers(-2 ** 31, 2 ** 31, size=n, dtype=np.int64).astype(np.int32)
    yield "few_distinct", rng.integers(-3, 3, size=n).astype(np.int32)
    yield "all_equal", np.full(n, 7, dtype=np.int32)
    a = np.arange(n, dtype=np.int64)
    yield "sorted_desc", (n - a).astype(np.int32)
    b = rng.integers(-1000, 1000, size=n).astype(np.int32)
    b[:: 3] = 2 ** 31 - 1
    b[1:: 5] = -2 ** 31
    yield "extremes", b


@pytest.mark.parametrize("n", [1, 7, 4096, 5000, 100003, (1 << 22) + 5])
@pytest.mark.parametrize("largest", [False, True])
def test_topk_vs_stable_sort(gpu, n, largest):
    import torch
    for fam, a in _inputs(n, n):
        d = torch.from_numpy(a).cuda()
        for k in sorted({k for k in (1, 2, 64, n // 2, n - 1, n) if 1 <= k <= n}):
            vals, idx = _run(gpu, d, n, k, largest)
            want = _ref_idx(a, k, largest)
            np.testing.assert_array_equal(idx.cpu().numpy(), want, err_msg=f"{fam} k={k}")
            np.testing.assert_array_equal(vals.cpu().numpy(), a[want], err_msg=f"{fam} k={k}")


def test_topk_unaligned_and_single_output(gpu):
    import torch
    n = 300001
    rng = np.random.default_rng(3)
    a = rng.integers(-50, 50, size=n + 3).astype(np.int32)
    base = torch.from_numpy(a).cuda()
    for off in (1, 2, 3):
        d = base[off:off + n]
        for largest in (False, True):
            for k in (1, 777, n // 3):
                want = _ref_idx(a[off:off + n], k, largest)
                vals, _ = _run(gpu, d, n, k, largest, with_idx=False)
                np.testing.assert_array_equal(vals.cpu().numpy(), a[off:off + n][want])
                _, idx = _run(gpu, d, n, k, largest, with_vals=False)
                np.testing.assert_array_equal(idx.cpu().numpy(), want)


def test_topk_errors(gpu):
    import kselect
    import torch
    d = torch.zeros(10, dtype=torch.int32, device="cuda")
    out = torch.empty(10, dtype=torch.int32, device="cuda")
    for n, k in ((10, 0), (10, 11), (0, 1)):
        with pytest.raises(kselect.KthError):
            gpu.topk(d, n, k, out, None)
    with pytest.raises(kselect.KthError):
        gpu.topk(d, 10, 1, None, None)


@pytest.mark.parametrize("fam,k,largest", [("uniform_half", 64, False), ("uniform_full", 1 << 20, True),
                                           ("few_distinct", (1 << 27) + 3, False), ("sorted_desc", 1000, True)])
def test_topk_full_size_properties(gpu, fam, k, largest):
    """2^28 keys (BASELINE-scale chunking, 1 GiB): properties that pin the exact top-k."""
    import torch
    n = 1 << 28
    d = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu.fill(d, n, fam, param=7)
    gpu.sync()
    vals, idx = _run(gpu, d, n, k, largest)
    idx_c = idx.cpu().numpy()
    assert np.all(np.diff(idx_c) > 0) and idx_c[0] >= 0 and idx_c[-1] < n
    assert torch.equal(vals, d[idx])
    kth = gpu.select(d, n - k + 1 if largest else k)
    sgn = -1 if largest else 1
    dd = d.to(torch.int64) * sgn
    v = kth * sgn
    vv = vals.to(torch.int64) * sgn
    assert int(vv.max()) == v  # the k-th is kept, nothing beyond it
    n_better = int((dd < v).sum())
    assert int((vv < v).sum()) == n_better  # every strictly better key is kept
    # the ties kept are the first (k - n_better) ties by index
    ties = torch.nonzero(dd == v).flatten()[: k - n_better].cpu().numpy()
    np.testing.assert_array_equal(idx_c[(vv == v).cpu().numpy()], ties)


def test_topk_window_path_unaligned_small_k(gpu):
    """n > 4 Mi takes the window path, whose streaming pass flags the tiles that
    can hold output (k * 1024 <= n): unaligned heads, a ragged tail, clustered keys."""
    import torch
    n = (1 << 23) + 3
    rng = np.random.default_rng(11)
    a = rng.integers(-2 ** 31, 2 ** 31, size=n + 3, dtype=np.int64).astype(np.int32)
    a[5_000_000:5_000_100] = -2 ** 31  # a cluster of minima inside one tile
    a[-40:] = 2 ** 31 - 1              # maxima in the ragged tail
    base = torch.from_numpy(a).cuda()
    for off in (0, 1, 3):
        d = base[off:off + n]
        h = a[off:off + n]
        for largest in (False, True):
            for k in (1, 37, 100, 4096, 8191):
                vals, idx = _run(gpu, d, n, k, largest)
                want = _ref_idx(h, k, largest)
                np.testing.assert_array_equal(idx.cpu().numpy(), want, err_msg=f"off={off} k={k} {largest}")
                np.testing.assert_array_equal(vals.cpu().numpy(), h[want])


@pytest.mark.parametrize("largest", [False, True])
def test_topk_tile_flag_cutoff_and_window_miss(gpu, largest):
    """k = n // 1024 (streaming-pass tile flags on) and n // 1024 + 1 (off), and
    inputs whose sample window misses the k-th (a spike of one value at the
    median and a narrow band: the flags are not trusted, skip_ok false) or
    whose candidates overflow (fallback levels)."""
    import torch
    n = (1 << 23) + 1029
    rng = np.random.default_rng(23 + largest)
    spike = rng.integers(-2 ** 31, 2 ** 31, size=n, dtype=np.int64).astype(np.int32)
    spike[rng.random(n) < 0.3] = 12345
    narrow = rng.integers(-2048, 2048, size=n).astype(np.int32)
    uni = rng.integers(-2 ** 31, 2 ** 31, size=n, dtype=np.int64).astype(np.int32)
    for name, a in (("uniform", uni), ("spike", spike), ("narrow", narrow)):
        d = torch.from_numpy(a).cuda()
        for k in (n // 1024, n // 1024 + 1, 1, n // 2):
            vals, idx = _run(gpu, d, n, k, largest)
            want = _ref_idx(a, k, largest)
            np.testing.assert_array_equal(idx.cpu().numpy(), want, err_msg=f"{name} k={k}")
            np.testing.assert_array_equal(vals.cpu().numpy(), a[want], err_msg=f"{name} k={k}")
            assert gpu.stats()["error"] == 0


def test_topk_bracket_failure_is_reported(gpu):
    """A k-th that does not bracket k in the count pass (forced here with the
    test-only KTH_HOOK_FAULT_TOPK_RANK hook, which selects a neighbouring rank) must
    surface as kth_ctx_last_stats().error and leave the outputs unwritten."""
    import torch
    import kselect
    faulty = kselect.Selector(0)
    faulty.test_hook(kselect.KTH_HOOK_FAULT_TOPK_RANK, 1)
    n, k = (1 << 22) + 7, 1000
    a = np.random.default_rng(5).permutation(n).astype(np.int32)  # distinct keys
    d = torch.from_numpy(a).cuda()
    for largest in (False, True):
        vals = torch.full((k,), -77, dtype=torch.int32, device="cuda")
        idx = torch.full((k,), -77, dtype=torch.int64, device="cuda")
        faulty.topk(d, n, k, vals, idx, largest=largest)
        faulty.sync()
        assert faulty.stats()["error"] == 32
        assert bool((vals == -77).all()) and bool((idx == -77).all())
    faulty.close()
    vals, idx = _run(gpu, d, n, k, False)  # a normal ctx: no error
    assert gpu.stats()["error"] == 0
    np.testing.assert_array_equal(idx.cpu().numpy(), _ref_idx(a, k, False))


@pytest.mark.parametrize("largest", [False, True])
def test_topk_large_k_from_stream_counts(gpu, largest):
    """k > n / 1024 on the window path with 16-byte aligned keys: the tile counts
    come from the streaming pass's per-row words (#beyond the window, #on each
    edge) plus the candidates' rows (k_main<3/4>, k_topk_cands), not from a
    second read of the input.  Families put the k-th on a window edge (narrow,
    few distinct: heavy ties at lo / hi), strictly inside it (uniform), or
    outside it (spike at the median: window miss, counted from the input); the
    ragged tail past k_main's full tiles is counted from the input."""
    import torch
    n = (1 << 23) + 4099
    rng = np.random.default_rng(31 + largest)
    uni = rng.integers(-2 ** 31, 2 ** 31, size=n, dtype=np.int64).astype(np.int32)
    narrow = rng.integers(-300, 300, size=n).astype(np.int32)
    few = rng.integers(-3, 4, size=n).astype(np.int32)
    spike = uni.copy()
    spike[rng.random(n) < 0.4] = -99
    for name, a in (("uniform", uni), ("narrow", narrow), ("few", few), ("spike", spike)):
        d = torch.from_numpy(a).cuda()
        for k in (n // 1024 + 1, n // 3, n // 2, n - 5):
            vals, idx = _run(gpu, d, n, k, largest)
            want = _ref_idx(a, k, largest)
            np.testing.assert_array_equal(idx.cpu().numpy(), want, err_msg=f"{name} k={k}")
            np.testing.assert_array_equal(vals.cpu().numpy(), a[want], err_msg=f"{name} k={k}")
            assert gpu.stats()["error"] == 0


def _staged_cases(n, rng):
    uni = rng.integers(-2 ** 31, 2 ** 31, size=n, dtype=np.int64).astype(np.int32)
    yield "uniform", uni
    yield "narrow", rng.integers(-300, 300, size=n).astype(np.int32)     # heavy ties on the window edges
    yield "few", rng.integers(-3, 4, size=n).astype(np.int32)
    spike = uni.copy()
    spike[rng.random(n) < 0.4] = -99                                       # window miss at the median
    yield "spike", spike
    a = np.arange(n, dtype=np.int64)
    yield "sorted_asc", (a - n // 2).astype(np.int32)                      # the kept side in a few segments
    yield "sorted_desc", (n // 2 - a).astype(np.int32)


@pytest.mark.parametrize("largest", [False, True])
def test_topk_staged_index_order(gpu, largest):
    """n / 65536 < k <= n / 16 on the window path, 16-byte aligned keys: the
    streaming pass stages every key on the kept side of the window's far edge in
    index order per wave-row, with its position, in per-wave segments
    (k_main<5/6>), and the count and write passes read those entries, not the
    input (k_tk5_count, k_tk5_write); the ragged tail past the full tiles is
    counted and written from the input.  k > n / 32 takes the larger LDS stage
    of k_tk5_write; windows whose output exceeds the stage (sorted inputs: every
    key of a window kept) are written directly.  Against a stable argsort."""
    import torch
    n = (1 << 23) + 4099
    rng = np.random.default_rng(41 + largest)
    for name, a in _staged_cases(n, rng):
        d = torch.from_numpy(a).cuda()
        for k in (n // 65536 + 1, n // 1024, n // 256, n // 64, n // 32, n // 24, n // 16):
            vals, idx = _run(gpu, d, n, k, largest)
            want = _ref_idx(a, k, largest)
            np.testing.assert_array_equal(idx.cpu().numpy(), want, err_msg=f"{name} k={k}")
            np.testing.assert_array_equal(vals.cpu().numpy(), a[want], err_msg=f"{name} k={k}")
            assert gpu.stats()["error"] == 0


def test_topk_staged_segment_overflow_falls_back(gpu):
    """Staging segments too small for the kept side (KTH_HOOK_TOPK_SEG_CAP, a
    test-only hook): the overflow flag sends the count and write passes back to
    the input, and the result is the same."""
    import torch
    import kselect
    small = kselect.Selector(0)
    small.test_hook(kselect.KTH_HOOK_TOPK_SEG_CAP, 300)
    n = (1 << 23) + 4099
    rng = np.random.default_rng(53)
    for name, a in _staged_cases(n, rng):
        d = torch.from_numpy(a).cuda()
        for largest in (False, True):
            for k in (n // 1024, n // 64):
                vals, idx = _run(small, d, n, k, largest)
                want = _ref_idx(a, k, largest)
                np.testing.assert_array_equal(idx.cpu().numpy(), want, err_msg=f"{name} k={k} {largest}")
                np.testing.assert_array_equal(vals.cpu().numpy(), a[want], err_msg=f"{name} k={k} {largest}")
    small.close()


@pytest.mark.parametrize("k", [1 << 20, 1 << 24])
def test_topk_staged_full_size(gpu, k):
    """2^28 keys, k in the staged range: the exact top-k properties."""
    test_topk_full_size_properties(gpu, "uniform_full", k, False)
