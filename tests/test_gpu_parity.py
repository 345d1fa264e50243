"""GPU parity: the HIP path (through the C-ABI) against the oracle and the
reference's own golden vectors.  Integer work -> every comparison is bit-exact.

Sizes: golden fixtures (reference outputs, n <= 16384); synthetic families up to
2^24 against the oracle; BASELINE sizes (2^30) through the exact rank
certificate #(<v) < k <= #(<=v), which holds iff v is the k-th smallest.
"""
import ctypes

import numpy as np
import pytest

from conftest import load_input, true_kth

pytestmark = pytest.mark.gpu

FAMS = ["uniform_full", "uniform_half", "uniform_ref", "all_equal", "few_distinct", "sorted_asc", "sorted_desc",
        "mod_1000"]


def _dev_keys(gpu, n, fam, seed=0x5EED0001, param=7):
    import torch
    keys = torch.empty(n, dtype=torch.int32, device="cuda")
    gpu.fill(keys, n, fam, seed=seed, param=param)
    gpu.sync()
    return keys


def _ks(n):
    return sorted({k for k in (1, 2, n // 2, n - 1, n) if 1 <= k <= n})


# ------------------------------------------------------------ golden vectors
def test_golden_fixtures(gpu, golden):
    """Every reference-generated case: GPU == true order statistic, == the
    reference seq answer where it is not defective, == every terminating CGM run."""
    import torch
    cache = {}
    for c in golden["cases"]:
        a = cache.setdefault(c["input"], load_input(c["input"]))
        got_host = gpu.select(a, c["k"])
        got_dev = gpu.select(torch.from_numpy(a).cuda(), c["k"])
        assert got_host == got_dev == c["true"], c
        if not c["seq_ref_defect"]:
            assert got_host == c["seq_ref"], c
        for p, v in c["cgm_ref"].items():
            if v != "livelock":
                assert got_host == v, (c, p)


def test_shipped_pins(gpu, golden, oracle):
    """The unmodified shipped programs (n = 1e8) -- regenerate their inputs with the
    pinned restated generators and select on the GPU."""
    shipped = golden.get("shipped")
    if not shipped:
        pytest.skip("no shipped pins in expected.json")
    gens = {"kth-problem-seq.c:26-28": oracle.ko_gen_shipped_seq, "TODO-kth-problem-cgm.c:10-17": oracle.ko_gen_shipped_cgm}
    done = 0
    for rec in shipped:
        if "generator" not in rec:
            continue
        a = np.empty(rec["n"], dtype=np.int32)
        gens[rec["generator"]](a.ctypes.data, rec["n"], rec["time_seed"])
        got = gpu.select(a, rec["k"])
        assert got == rec["true"], rec
        if rec["printed"] != "livelock" and rec["printed"] != rec["true"]:
            assert rec["program"].startswith("seq"), rec  # only the seq comparator defect may differ
        done += 1
    assert done


# --------------------------------------------------------- oracle, all paths
def test_device_generator_matches_numpy(gpu):
    import gen as G
    for fam in FAMS:
        d = _dev_keys(gpu, 1 << 16, fam).cpu().numpy()
        h = G.gen(1 << 16, G.BY_NAME[fam], 0x5EED0001, 7)
        np.testing.assert_array_equal(d, h, err_msg=fam)


@pytest.mark.parametrize("n", [1, 2, 3, 100, 16384, 16385, 100003, (1 << 22), (1 << 22) + 1, (1 << 24) + 5])
def test_paths_vs_oracle(gpu, oracle, n):
    """LDS (n <= 16384), radix (<= 4M) and window (> 4M) paths, every family, k at the edges."""
    for fam in FAMS:
        keys = _dev_keys(gpu, n, fam)
        host = keys.cpu().numpy()
        srt = np.sort(host)
        assert true_kth(oracle, host, (n + 1) // 2) == srt[(n + 1) // 2 - 1]
        for k in _ks(n):
            got = gpu.select(keys, k)
            assert got == srt[k - 1], (fam, n, k, got, srt[k - 1], gpu.stats())


def _fuzz_keys(rng, n, kind):
    """Distributions the synthetic families do not cover: they move the window
    and the candidate set around (not uniform, clustered, spiky, narrow)."""
    if kind == "normal":
        a = rng.normal(0, 2e8, n)
    elif kind == "exponential":
        a = rng.exponential(1e6, n) - 5e5
    elif kind == "narrow":  # heavy duplicates: 4096 distinct values
        a = rng.integers(-2048, 2048, n)
    elif kind == "spike_median":  # 30 % of the keys on one value near the median
        a = rng.integers(-2 ** 31, 2 ** 31, n)
        a[rng.random(n) < 0.3] = 12345
    elif kind == "clusters":  # 5 tight clusters
        c = rng.integers(-2 ** 30, 2 ** 30, 5)
        a = c[rng.integers(0, 5, n)] + rng.integers(-1000, 1000, n)
    elif kind == "two_values":
        a = np.where(rng.random(n) < 0.5, -7, 2 ** 31 - 1)
    else:  # "blocks": sorted runs, each run from its own range
        a = np.sort(rng.integers(-2 ** 31, 2 ** 31, n).reshape(-1, n // 8), axis=1).reshape(-1)
    return np.clip(a, -2 ** 31, 2 ** 31 - 1).astype(np.int32)


@pytest.mark.parametrize("kind", ["normal", "exponential", "narrow", "spike_median", "clusters", "two_values",
                                  "blocks"])
def test_window_path_fuzz(gpu, kind):
    """Window path (n > 4 Mi, including sample sizes that end in a partial chunk)
    on non-uniform inputs, random k: GPU == np.partition."""
    import torch
    rng = np.random.default_rng(sum(map(ord, kind)))  # stable across processes
    for n in (5_000_008, (1 << 23) + 4096):
        a = _fuzz_keys(rng, n, kind)
        d = torch.from_numpy(a).cuda()
        for k in sorted({1, n, n // 2, int(rng.integers(1, n + 1)), int(rng.integers(1, n + 1))}):
            want = np.partition(a, k - 1)[k - 1]
            assert gpu.select(d, k) == want, (kind, n, k, gpu.stats())


@pytest.mark.parametrize("copies,spread", [(6000, 1), (20000, 1), (9000, 40), (40000, 3)])
def test_finish_tail_clustered_block(gpu, copies, spread):
    """k_finish's tail at 2^28 keys (~1.3 M candidates, ~5 K per workgroup
    slice): a contiguous block of near-duplicate keys at the median lands in a
    few slices, so a slice can hold more of the picked bin's keys than its LDS
    stage (the second append scan), or the bin more than one workgroup's LDS
    (40000: no tail, grid levels); spread > 1 leaves several values in the last
    bin (the one-wave list rank).  Checked by the exact rank certificate
    #(< v) < k <= #(<= v) on the device."""
    import torch
    n = 1 << 28
    d = _dev_keys(gpu, n, "uniform_full")
    med = gpu.select(d, n // 2)
    g = torch.Generator(device="cuda")
    g.manual_seed(copies + spread)
    start = (n // 3 + copies * 7919) % (n - copies)
    d[start:start + copies] = med + torch.randint(0, spread, (copies,), device="cuda", dtype=torch.int32,
                                                  generator=g)
    torch.cuda.synchronize()
    for k in (n // 2 - copies // 3, n // 2, n // 2 + 1, n // 2 + copies // 2):
        v = gpu.select(d, k)
        lt, le = int((d < v).sum()), int((d <= v).sum())
        assert lt < k <= le, (copies, spread, k, v, lt, le, gpu.stats())


def test_unaligned_device_pointer(gpu):
    """Shards start anywhere: 4-byte but not 16-byte aligned inputs."""
    import torch
    n = (1 << 22) + 123
    keys = _dev_keys(gpu, n + 3, "uniform_full")
    for off in (1, 2, 3):
        sub = keys[off:off + n]
        srt = np.sort(sub.cpu().numpy())
        for k in (1, n // 3, n):
            assert gpu.select(sub, k) == srt[k - 1]
    torch.cuda.synchronize()


@pytest.mark.parametrize("fam,param", [("uniform_half", 0), ("uniform_full", 0), ("uniform_ref", 0),
                                       ("all_equal", 7), ("all_equal", -2 ** 31), ("all_equal", 2 ** 31 - 1),
                                       ("few_distinct", 0), ("sorted_asc", 0), ("sorted_desc", 0),
                                       ("mod_1000", 0)])
def test_full_size_rank_certificate(gpu, fam, param):
    """BASELINE configs 2 and 4 at n = 2^30: exact rank certificate for k in {1, n/2, n}."""
    import torch
    n = 1 << 30
    keys = _dev_keys(gpu, n, fam, param=param)
    for k in (1, n // 2, n):
        v = gpu.select(keys, k)
        lt = int((keys < v).sum())
        le = int((keys <= v).sum())
        assert lt < k <= le, (fam, param, k, v, lt, le)
        st = gpu.stats()
        assert st["path"] == 3, (fam, k, st)  # resolved by the one-pass window, no fallback
    del keys
    torch.cuda.empty_cache()


def test_window_fallback_is_exact(gpu):
    """An input that defeats the sample (its sampled chunks are all one value,
    everything else differs) must still be exact via the fallback passes."""
    import torch
    import kselect
    n = 1 << 24
    keys = _dev_keys(gpu, n, "uniform_full")
    fresh = kselect.Selector(0)  # candidate capacity sized for this n (the shared ctx grew for 2^30)
    # k_gather samples ceil(s/C) chunks of C keys at stride n / ceil(s/C)
    # (include/kth.h kth_sample_chunk); overwrite those chunks
    from kselect._lib import load
    lib = load()
    s = int(lib.kth_dist_sample_size(n))
    c = int(lib.kth_sample_chunk())
    nch = -(-s // c)
    stride = n // nch
    idx = (torch.arange(nch, device="cuda") * stride).repeat_interleave(c) + torch.arange(c, device="cuda").repeat(nch)
    keys[idx] = 5
    srt = np.sort(keys.cpu().numpy())
    for k in (1, n // 2, n):
        assert fresh.select(keys, k) == srt[k - 1]
    assert fresh.stats()["path"] == 4
    fresh.close()


# ---------------------------------------------------------------- async API
def test_async_and_stats(gpu):
    import torch
    n = 1 << 24
    keys = _dev_keys(gpu, n, "uniform_half")
    out = torch.zeros(4, dtype=torch.int32, device="cuda")
    for i, k in enumerate((1, 1000, n // 2, n)):
        gpu.select_async(keys, n, k, out[i:i + 1])
    gpu.sync()
    srt = np.sort(keys.cpu().numpy())
    assert out.cpu().tolist() == [srt[0], srt[999], srt[n // 2 - 1], srt[n - 1]]
    st = gpu.stats()
    assert st["path"] == 3 and st["error"] == 0 and st["n"] == n and st["k"] == n


def test_errors(gpu):
    import kselect
    import torch
    keys = torch.zeros(10, dtype=torch.int32, device="cuda")
    for k in (0, 11, -1):
        with pytest.raises(kselect.KthError) as e:
            gpu.select(keys, k)
        assert e.value.code == kselect.KTH_EINVAL


# --------------------------------------------------------------- IntVector
def test_vec_kth_select_dropin(gpu):
    """VecKthSelect == VecQuickSort + VecGet(k-1) (kth-problem-seq.c:32-33), sentinels kept."""
    import kselect
    rng = np.random.default_rng(3)
    a = rng.integers(-2 ** 30, 2 ** 30, size=100_000, dtype=np.int64).astype(np.int32)
    v = kselect.IntVec.from_array(a)
    w = kselect.IntVec.from_array(a)
    w.quicksort()
    for k in (1, 17, 50_000, 100_000):
        assert v.kth_select(k) == w.get(k - 1)
    assert v.kth_select(0) == -2 and v.kth_select(100_001) == -2
    np.testing.assert_array_equal(v.array(), a)  # input not modified


# ------------------------------------------------------------ batched rows
def _row_ref(m, k):
    return np.sort(m, axis=1, kind="stable")[:, k - 1]


@pytest.mark.parametrize("cols", [1, 7, 1000, 1024, 1500, 2048, 4093, 4096, 5000, 16384])
def test_rows_i32(gpu, cols):
    import torch
    rows = 257
    rng = np.random.default_rng(cols)
    m = rng.integers(-2 ** 31, 2 ** 31, size=(rows, cols), dtype=np.int64).astype(np.int32)
    m[::3] = rng.integers(-3, 3, size=(len(m[::3]), cols))  # duplicate-heavy rows
    d = torch.from_numpy(m).cuda()
    out = torch.empty(rows, dtype=torch.int32, device="cuda")
    for k in sorted({1, min(64, cols), (cols + 1) // 2, cols}):
        gpu.rows(d, rows, cols, k, out)
        gpu.sync()
        np.testing.assert_array_equal(out.cpu().numpy(), _row_ref(m, k), err_msg=f"k={k}")


def test_rows_unaligned_and_adversarial(gpu):
    """Wave-per-row kernel: a base pointer 4 bytes off 16-byte alignment (scalar
    load path), all-equal rows at INT_MIN / INT_MAX, and rows of two values."""
    import torch
    rows, cols = 300, 4096
    rng = np.random.default_rng(11)
    m = rng.integers(-2 ** 31, 2 ** 31, size=(rows, cols + 1), dtype=np.int64).astype(np.int32)
    m[0] = -2 ** 31
    m[1] = 2 ** 31 - 1
    m[2] = rng.choice(np.array([5, -5], dtype=np.int32), size=cols + 1)
    flat = torch.from_numpy(m.reshape(-1)).cuda()
    sub = flat[1:1 + rows * cols]  # 4-byte aligned, not 16
    host = sub.cpu().numpy().reshape(rows, cols)
    out = torch.empty(rows, dtype=torch.int32, device="cuda")
    for k in (1, 2, 64, cols // 2, cols - 1, cols):
        gpu.rows(sub, rows, cols, k, out)
        gpu.sync()
        np.testing.assert_array_equal(out.cpu().numpy(), _row_ref(host, k), err_msg=f"k={k}")


def _f32_order_key(x):
    b = x.view(np.uint32).astype(np.uint64)
    nan = np.isnan(x)
    key = np.where(b & 0x80000000, (~b) & 0xFFFFFFFF, b | 0x80000000)
    return np.where(nan, 0xFFFFFFFF, key)


@pytest.mark.parametrize("cols", [4096, 2048, 333, 6000])
def test_rows_f32(gpu, cols):
    import torch
    rows = 129
    rng = np.random.default_rng(7)
    m = rng.uniform(-1, 1, size=(rows, cols)).astype(np.float32)
    m[1] = np.round(m[1] * 4) / 4  # duplicate-heavy
    m[2, :5] = [np.nan, -0.0, 0.0, np.inf, -np.inf]
    m[3, :] = -0.0
    m[3, ::2] = 0.0
    d = torch.from_numpy(m).cuda()
    out = torch.empty(rows, dtype=torch.float32, device="cuda")
    keys = _f32_order_key(m)
    for k in (1, 64, cols // 2, cols):
        gpu.rows(d, rows, cols, k, out, f32=True)
        gpu.sync()
        got = out.cpu().numpy()
        idx = np.argsort(keys, axis=1, kind="stable")[:, k - 1]
        want = m[np.arange(rows), idx]
        np.testing.assert_array_equal(_f32_order_key(got), _f32_order_key(want), err_msg=f"k={k}")


def _f32_adversarial_rows(rng, rows, cols):
    """Rows that stress the value-linear first pass of the row kernel: huge and
    tiny value ranges, subnormals, infinities, NaN, signed zeros, a few
    distinct values, clusters a few ulps wide, and one outlier per row."""
    m = rng.uniform(-1, 1, size=(rows, cols)).astype(np.float32)
    fams = [
        lambda: rng.uniform(-3e38, 3e38, cols),                       # range overflows float
        lambda: rng.uniform(-1e-38, 1e-38, cols),                     # subnormals / tiny
        lambda: np.float32(1.0) + rng.integers(0, 8, cols) * np.float32(2 ** -23),  # ulp cluster
        lambda: np.where(rng.random(cols) < 0.5, np.inf, -np.inf),
        lambda: np.where(rng.random(cols) < 0.1, np.nan, rng.uniform(-1, 1, cols)),
        lambda: np.where(rng.random(cols) < 0.5, -0.0, 0.0),
        lambda: rng.choice(np.array([-2.5, 0.0, 7.0, 1e30], dtype=np.float32), cols),
        lambda: np.concatenate([rng.normal(0, 1, cols - 1), [1e35]]),  # one outlier
        lambda: np.concatenate([rng.normal(0, 1, cols - 1), [np.inf]]),
        lambda: np.exp(rng.normal(0, 10, cols)),                      # log-normal, wide
        lambda: rng.uniform(-1, 1, cols) * np.float32(1e-30),
        lambda: np.full(cols, 3.0),
    ]
    for i in range(rows):
        if i % 2 == 0:
            m[i] = np.asarray(fams[(i // 2) % len(fams)](), dtype=np.float64).astype(np.float32)
    return m


@pytest.mark.parametrize("cols", [4096, 2048, 1000, 333])
def test_rows_f32_adversarial(gpu, cols):
    import torch
    rows = 96
    rng = np.random.default_rng(cols + 99)
    with np.errstate(over="ignore", invalid="ignore"):
        m = _f32_adversarial_rows(rng, rows, cols)
    d = torch.from_numpy(m).cuda()
    out = torch.empty(rows, dtype=torch.float32, device="cuda")
    keys = _f32_order_key(m)
    for k in sorted({1, 2, 64, cols // 3, cols // 2, cols - 1, cols}):
        gpu.rows(d, rows, cols, k, out, f32=True)
        gpu.sync()
        got = out.cpu().numpy()
        idx = np.argsort(keys, axis=1, kind="stable")[:, k - 1]
        want = m[np.arange(rows), idx]
        np.testing.assert_array_equal(_f32_order_key(got), _f32_order_key(want), err_msg=f"k={k}")


@pytest.mark.parametrize("cols", [4096, 1000])
def test_rows_i32_ranges(gpu, cols):
    """Row key ranges of every width (the row kernel normalises each row to its
    own [min, max]): narrow, wide, one outlier, INT_MIN/INT_MAX mixes."""
    import torch
    rows = 64
    rng = np.random.default_rng(cols + 5)
    m = np.empty((rows, cols), dtype=np.int64)
    for i in range(rows):
        w = 1 << (i % 33)
        lo = int(rng.integers(-2 ** 31, 2 ** 31 - min(w, 2 ** 31 - 1)))
        m[i] = rng.integers(lo, min(lo + w, 2 ** 31), size=cols) if w > 1 else lo
        if i % 5 == 0:
            m[i, int(rng.integers(cols))] = 2 ** 31 - 1 if i % 2 else -2 ** 31
    m = m.astype(np.int32)
    d = torch.from_numpy(m).cuda()
    out = torch.empty(rows, dtype=torch.int32, device="cuda")
    for k in sorted({1, 2, 64, cols // 2, cols - 1, cols}):
        gpu.rows(d, rows, cols, k, out)
        gpu.sync()
        np.testing.assert_array_equal(out.cpu().numpy(), _row_ref(m, k), err_msg=f"k={k}")


def _dense_bin_rows(rng, rows, cols, f32):
    """Rows whose picked first-pass bin holds more than 64 keys (the fast path's
    row_select_dense_bin): one value per bin (span 0), at most 8 values in the
    bin (per-lane register counts), and wider clusters (the radix sweeps) --
    BASELINE config 5's duplicate-heavy variant and its neighbours."""
    m = np.empty((rows, cols), dtype=np.float32 if f32 else np.int32)
    for i in range(rows):
        f = i % 6
        if f32:
            if f == 0:
                m[i] = np.round(rng.uniform(-1, 1, cols) * 8) / 8          # 17 values, one per bin
            elif f == 1:
                m[i] = np.float32(1.0) + rng.integers(0, 8, cols) * np.float32(2 ** -23)  # 8 adjacent keys
            elif f == 2:
                m[i] = rng.choice(np.array([-1.5, 0.25, 3.0], dtype=np.float32), cols)
            elif f == 3:
                m[i] = np.where(rng.random(cols) < 0.5, rng.uniform(-1, 1, cols),
                                np.float32(0.5) + rng.integers(0, 300, cols) * np.float32(2 ** -22))
            elif f == 4:
                m[i] = np.round(rng.normal(0, 1, cols) * 4) / 4
            else:
                m[i] = rng.uniform(-1, 1, cols)
        else:
            if f == 0:
                m[i] = rng.integers(-3, 4, cols)                                # 7 values around 0
            elif f == 1:
                m[i] = (rng.integers(0, 16, cols) << 24) - 2 ** 31              # one value per top byte
            elif f == 2:
                m[i] = rng.integers(100, 108, cols)                             # 8 adjacent values
            elif f == 3:
                m[i] = rng.integers(0, 1000, cols)                              # a wide cluster (radix)
            elif f == 4:
                m[i] = np.where(rng.random(cols) < 0.3, 77, rng.integers(-2 ** 31, 2 ** 31, cols))
            else:
                m[i] = rng.integers(-2 ** 31, 2 ** 31, cols)
    return m


@pytest.mark.parametrize("f32", [False, True])
def test_rows_dense_bins(gpu, f32):
    import torch
    rows, cols = 240, 4096
    rng = np.random.default_rng(1234 + f32)
    m = _dense_bin_rows(rng, rows, cols, f32)
    d = torch.from_numpy(m).cuda()
    out = torch.empty(rows, dtype=torch.float32 if f32 else torch.int32, device="cuda")
    keys = _f32_order_key(m).astype(np.int64) if f32 else m.astype(np.int64)
    for k in (1, 2, 64, 1000, 2048, 4095, 4096):
        gpu.rows(d, rows, cols, k, out, f32=f32)
        gpu.sync()
        idx = np.argsort(keys, axis=1, kind="stable")[:, k - 1]
        want = m[np.arange(rows), idx]
        got = out.cpu().numpy()
        if f32:
            np.testing.assert_array_equal(_f32_order_key(got), _f32_order_key(want), err_msg=f"k={k}")
        else:
            np.testing.assert_array_equal(got, want, err_msg=f"k={k}")
    for k in (1, 64, 2048, 4096):
        for largest in (False, True):
            vals = torch.empty((rows, k), dtype=out.dtype, device="cuda")
            idx = torch.empty((rows, k), dtype=torch.int32, device="cuda")
            gpu.topk_rows(d, rows, cols, k, vals, idx, largest=largest, f32=f32)
            gpu.sync()
            want_idx = _topk_ref(keys, k, largest)
            np.testing.assert_array_equal(idx.cpu().numpy(), want_idx, err_msg=f"topk k={k} largest={largest}")
            np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32),
                                          np.take_along_axis(m, want_idx, axis=1).view(np.uint32))


# ------------------------------------------------------------- top-k rows
def _topk_ref(keys, k, largest):
    """Column-order top-k with ties by column: numpy restatement of the contract
    (include/kth.h kth_topk_rows_*), on order keys (u64 view of the total order)."""
    order = -keys.astype(np.int64) if largest else keys.astype(np.int64)
    rows, cols = keys.shape
    idx = np.argsort(order, axis=1, kind="stable")[:, :k]  # stable: ties by column
    return np.sort(idx, axis=1)  # column order


def _i32_order_key(m):
    return m.astype(np.int64)


@pytest.mark.parametrize("cols,k", [(4096, 64), (4096, 1), (4096, 4096), (1500, 8), (7, 3), (2048, 2047)])
@pytest.mark.parametrize("largest", [False, True])
def test_topk_rows_i32(gpu, cols, k, largest):
    import torch
    rows = 193
    rng = np.random.default_rng(cols * 7 + k)
    m = rng.integers(-2 ** 31, 2 ** 31, size=(rows, cols), dtype=np.int64).astype(np.int32)
    m[::4] = rng.integers(-3, 3, size=(len(m[::4]), cols))  # heavy ties
    m[1] = 2 ** 31 - 1
    d = torch.from_numpy(m).cuda()
    vals = torch.empty((rows, k), dtype=torch.int32, device="cuda")
    idx = torch.empty((rows, k), dtype=torch.int32, device="cuda")
    gpu.topk_rows(d, rows, cols, k, vals, idx, largest=largest)
    gpu.sync()
    want_idx = _topk_ref(_i32_order_key(m), k, largest)
    np.testing.assert_array_equal(idx.cpu().numpy(), want_idx)
    np.testing.assert_array_equal(vals.cpu().numpy(), np.take_along_axis(m, want_idx, axis=1))


@pytest.mark.parametrize("largest", [False, True])
def test_topk_rows_f32(gpu, largest):
    import torch
    rows, cols, k = 129, 4096, 64
    rng = np.random.default_rng(5)
    m = rng.uniform(-1, 1, size=(rows, cols)).astype(np.float32)
    m[1] = np.round(m[1] * 4) / 4
    m[2, :6] = [np.nan, -0.0, 0.0, np.inf, -np.inf, np.nan]
    d = torch.from_numpy(m).cuda()
    vals = torch.empty((rows, k), dtype=torch.float32, device="cuda")
    idx = torch.empty((rows, k), dtype=torch.int32, device="cuda")
    gpu.topk_rows(d, rows, cols, k, vals, idx, largest=largest, f32=True)
    gpu.sync()
    want_idx = _topk_ref(_f32_order_key(m).astype(np.int64), k, largest)
    np.testing.assert_array_equal(idx.cpu().numpy(), want_idx)
    got = vals.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, np.take_along_axis(m, want_idx, axis=1).view(np.uint32))


@pytest.mark.parametrize("largest", [False, True])
def test_topk_rows_f32_adversarial(gpu, largest):
    import torch
    rows, cols, k = 96, 4096, 64
    rng = np.random.default_rng(17)
    with np.errstate(over="ignore", invalid="ignore"):
        m = _f32_adversarial_rows(rng, rows, cols)
    d = torch.from_numpy(m).cuda()
    vals = torch.empty((rows, k), dtype=torch.float32, device="cuda")
    idx = torch.empty((rows, k), dtype=torch.int32, device="cuda")
    gpu.topk_rows(d, rows, cols, k, vals, idx, largest=largest, f32=True)
    gpu.sync()
    want_idx = _topk_ref(_f32_order_key(m).astype(np.int64), k, largest)
    np.testing.assert_array_equal(idx.cpu().numpy(), want_idx)
    got = vals.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, np.take_along_axis(m, want_idx, axis=1).view(np.uint32))


def test_topk_rows_errors(gpu):
    import kselect
    import torch
    d = torch.zeros((2, 5000), dtype=torch.int32, device="cuda")
    out = torch.empty((2, 4), dtype=torch.int32, device="cuda")
    for cols, k in ((5000, 4), (10, 0), (10, 11)):
        with pytest.raises(kselect.KthError):
            gpu.topk_rows(d, 2, cols, k, out, None)


# ----------------------------------------------------- sharded, one rank
@pytest.mark.parametrize("path", ["c", "py"])
def test_dist_world1_nccl(gpu, monkeypatch, path):
    """The sharded protocol (kth_dist_* + RCCL collectives) with one rank: over
    RCCL in one library call (kth_dist_select_rccl, the default) or as the
    scripted steps (KTH_DIST_PY=1), and over torch.distributed's collectives."""
    import torch
    import torch.distributed as dist
    from kselect.dist import DistSelector, HipBackend
    if path == "py":
        monkeypatch.setenv("KTH_DIST_PY", "1")
    # one rank over an in-process HashStore: no TCP port to race for
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0),
                            store=dist.HashStore())
    try:
        from kselect.rccl import RcclComm, TorchComm
        b = HipBackend(0)
        for comm in (None, TorchComm()):  # direct RCCL on the selector's stream (default), torch's
            ds = DistSelector(b, comm=comm)
            assert isinstance(ds.comm, RcclComm if comm is None else TorchComm)
            for fam in ("uniform_full", "few_distinct", "sorted_desc"):
                n = 1 << 23
                keys = _dev_keys(gpu, n, fam)
                srt = np.sort(keys.cpu().numpy())
                for k in (1, n // 2, n):
                    got = int(ds.select(keys, n, n, k).item())
                    assert got == srt[k - 1], (fam, k, type(ds.comm).__name__, b.sel.stats())
                    assert ds.error() == 0
            ds.close()
    finally:
        dist.destroy_process_group()


# ------------------------------------------- reference fixtures, larger sizes
def test_golden_large(gpu, golden):
    """Radix (16385, 2^20 = BASELINE config 1) and window (2^22 + 1) sizes: the
    device generator reproduces the fixture's input (sha256), and the GPU answer
    equals the true order statistic, the reference seq block where it is not
    defective and every terminating reference CGM run (tests/golden/make_golden.py
    --large)."""
    import hashlib
    large = golden.get("large")
    if not large:
        pytest.skip("no large fixtures")
    import torch
    keys = None
    for c in large:
        if keys is None or keys[1] != (c["family"], c["n"]):
            t = torch.empty(c["n"], dtype=torch.int32, device="cuda")
            gpu.fill(t, c["n"], c["dist"], seed=c["seed"], param=c["param"])
            gpu.sync()
            h = hashlib.sha256(t.cpu().numpy().astype("<i4").tobytes()).hexdigest()
            assert h == c["input_sha256"], c
            keys = (t, (c["family"], c["n"]))
        got = gpu.select(keys[0], c["k"])
        assert got == c["true"], c
        if not c["seq_ref_defect"]:
            assert got == c["seq_ref"], c
        for p, v in c["cgm_ref"].items():
            if v != "livelock":
                assert got == v, (c, p)


# -------------------------------------------- batched rows, BASELINE shape
@pytest.mark.parametrize("f32", [False, True])
def test_rows_full_shape(gpu, f32):
    """BASELINE config 5 at its full shape, 65536 x 4096 (every grid-stride round
    of the row loop), k in {1, 64, 2048, 4096}, against torch.sort."""
    import torch
    R, C = 65536, 4096
    g = torch.Generator(device="cuda")
    g.manual_seed(123)
    if f32:
        m = torch.rand((R, C), generator=g, device="cuda") * 2 - 1
        m[::7] = torch.round(m[::7] * 8) / 8  # duplicate-heavy rows
    else:
        m = torch.randint(-2 ** 31, 2 ** 31, (R, C), generator=g, device="cuda", dtype=torch.int64).to(torch.int32)
        m[::7] = torch.randint(-3, 3, (len(range(0, R, 7)), C), generator=g, device="cuda", dtype=torch.int32)
    srt = torch.sort(m, dim=1).values
    out = torch.empty(R, dtype=m.dtype, device="cuda")
    torch.cuda.synchronize()  # m is built on torch's stream; the selector may run on its own
    for k in (1, 64, 2048, 4096):
        gpu.rows(m, R, C, k, out, f32=f32)
        gpu.sync()
        assert torch.equal(out, srt[:, k - 1]), k


@pytest.mark.parametrize("f32", [False, True])
def test_topk_rows_many_rows(gpu, f32):
    """Top-k rows over more rows than the resident waves (several rounds of the
    row loop, the next row's loads in flight during the tail), with staged,
    unstaged (ties) and dense-bin rows interleaved, against a stable sort."""
    import torch
    R, C, k = 16384 + 5, 4096, 64
    g = torch.Generator(device="cuda")
    g.manual_seed(321 + f32)
    if f32:
        m = torch.rand((R, C), generator=g, device="cuda") * 2 - 1
        m[::7] = torch.round(m[::7] * 8) / 8
        m[3::11] = torch.round(m[3::11] * 2000) / 2000
        u = m.view(torch.int32).to(torch.int64)
        key = torch.where(u < 0, -(u & 0x7FFFFFFF) - 1, u)  # the float order (no NaN here)
    else:
        m = torch.randint(-2 ** 31, 2 ** 31, (R, C), generator=g, device="cuda", dtype=torch.int64).to(torch.int32)
        m[::7] = torch.randint(-3, 3, (len(range(0, R, 7)), C), generator=g, device="cuda", dtype=torch.int32)
        m[3::11] = torch.randint(0, 1000, (len(range(3, R, 11)), C), generator=g, device="cuda", dtype=torch.int32)
        key = m.to(torch.int64)
    torch.cuda.synchronize()
    for largest in (False, True):
        order = -key if largest else key
        want = torch.sort(torch.sort(order, dim=1, stable=True).indices[:, :k], dim=1).values.to(torch.int32)
        vals = torch.empty((R, k), dtype=m.dtype, device="cuda")
        idx = torch.empty((R, k), dtype=torch.int32, device="cuda")
        torch.cuda.synchronize()
        gpu.topk_rows(m, R, C, k, vals, idx, largest=largest, f32=f32)
        gpu.sync()
        assert torch.equal(idx, want), largest
        assert torch.equal(vals.view(torch.int32), torch.gather(m, 1, want.to(torch.int64)).view(torch.int32)), largest


def _few_valued_rows(rng, rows, cols, f32):
    """Rows for the few-valued int path (<= 8 values, no histogram) and the
    dense float bin whose ends are zeros: values at INT_MIN / INT_MAX, two
    top bytes in the first key slot with a wide rest, -0.0 / +0.0 mixes."""
    m = np.empty((rows, cols), dtype=np.float32 if f32 else np.int32)
    for i in range(rows):
        f = i % 8
        if f32:
            if f == 0:
                m[i] = np.round(rng.uniform(-1, 1, cols) * 8) / 8                 # 17 values, both zeros
            elif f == 1:
                m[i] = rng.choice(np.array([-0.0, 0.0, 0.5], dtype=np.float32), cols)
            elif f == 2:
                m[i] = rng.choice(np.array([-0.0, 0.0], dtype=np.float32), cols)
                m[i, int(rng.integers(cols))] = -3.0                              # range > 0: value-linear bins
            elif f == 3:
                m[i] = rng.choice(np.array([-2.0, -0.0, 0.0, 1e-30], dtype=np.float32), cols)
            elif f == 4:
                m[i] = np.round(rng.normal(0, 1, cols) * 2) / 2
            elif f == 5:
                m[i] = rng.choice(np.array([-1.0, -0.0], dtype=np.float32), cols)
            elif f == 6:
                m[i] = rng.choice(np.array([0.0, 7.0], dtype=np.float32), cols)
            else:
                m[i] = rng.uniform(-1, 1, cols)
        else:
            if f == 0:
                m[i] = rng.integers(-1, 1, cols)                                  # {-1, 0}: two top bytes
            elif f == 1:
                m[i] = rng.integers(-2 ** 31, -2 ** 31 + 8, cols)                 # 8 values at INT_MIN
            elif f == 2:
                m[i] = rng.integers(2 ** 31 - 8, 2 ** 31, cols)                   # 8 values at INT_MAX
            elif f == 3:
                m[i] = rng.integers(0, 9, cols)                                   # 9 values: one too many
                m[i, :4 * 64] = 0                                                 # (first slot: one top byte)
            elif f == 4:
                m[i] = rng.integers(-2 ** 31, 2 ** 31, cols)
                m[i, :4 * 64] = 5                                                 # few-valued slot, wide row
            elif f == 5:
                m[i] = 42
            elif f == 6:
                m[i] = rng.integers(1000, 1008, cols)
            else:
                m[i] = rng.integers(-2 ** 31, 2 ** 31, cols)
    return m


@pytest.mark.parametrize("f32", [False, True])
def test_rows_few_valued_and_zero_bins(gpu, f32):
    """k-th and top-k per row (smallest and largest) on rows for the
    few-valued int path and the dense float bin with zero ends (round 4)."""
    import torch
    rows, cols = 160, 4096
    rng = np.random.default_rng(4321 + f32)
    m = _few_valued_rows(rng, rows, cols, f32)
    d = torch.from_numpy(m).cuda()
    keys = _f32_order_key(m).astype(np.int64) if f32 else m.astype(np.int64)
    out = torch.empty(rows, dtype=torch.float32 if f32 else torch.int32, device="cuda")
    for k in (1, 2, 64, 1000, 2047, 2048, 2049, 4095, 4096):
        gpu.rows(d, rows, cols, k, out, f32=f32)
        gpu.sync()
        want = m[np.arange(rows), np.argsort(keys, axis=1, kind="stable")[:, k - 1]]
        got = out.cpu().numpy()
        if f32:
            np.testing.assert_array_equal(_f32_order_key(got), _f32_order_key(want), err_msg=f"k={k}")
        else:
            np.testing.assert_array_equal(got, want, err_msg=f"k={k}")
    for k in (1, 64, 2048, 4096):
        for largest in (False, True):
            vals = torch.empty((rows, k), dtype=out.dtype, device="cuda")
            idx = torch.empty((rows, k), dtype=torch.int32, device="cuda")
            gpu.topk_rows(d, rows, cols, k, vals, idx, largest=largest, f32=f32)
            gpu.sync()
            want_idx = _topk_ref(keys, k, largest)
            np.testing.assert_array_equal(idx.cpu().numpy(), want_idx, err_msg=f"topk k={k} largest={largest}")
            np.testing.assert_array_equal(vals.cpu().numpy().view(np.uint32),
                                          np.take_along_axis(m, want_idx, axis=1).view(np.uint32))
