"""kselect -- Python host mirror of the libkth.so C-ABI (include/kth.h).

Mirrors the reference's selection interface (laertispappas/MPI-k-selection):

  * ``IntVec`` wraps the reference's ``IntVector`` (vector.h:7-11) through
    the ABI twin in libkth.so; ``IntVec.kth_select(k)`` is the drop-in for the
    select block ``VecQuickSort(pVec); VecGet(pVec, k - 1)``
    (kth-problem-seq.c:32-33), keeping the VecGet sentinels (-1 NULL, -2 out of
    range, vector.c:209-218).
  * ``kth_select(keys, k)`` / ``Selector`` -- the (data, n, k) -> value contract
    with explicit errors (``KthError``) instead of in-band sentinels.
  * ``kselect.dist`` -- the sharded (one process per GPU) replacement of the CGM
    driver TODO-kth-problem-cgm.c:76-278, with RCCL collectives through
    torch.distributed.

PyTorch is used only as plumbing (device memory, streams, collectives); every
selection runs in the HIP kernels of libkth.so.  There is no CPU fallback:
without the library ``kselect`` fails to import, and without a GPU every
compute call raises ``KthError(KTH_ENODEV)``.
"""
import ctypes

import numpy as np

from ._lib import (  # noqa: F401
    KTH_DIST_DONE,
    KTH_DIST_MAX_LEVELS,
    KTH_ECOMM,
    KTH_EINTERNAL,
    KTH_EINVAL,
    KTH_ENODEV,
    KTH_HOOK_FAULT_BARRIER,
    KTH_HOOK_FAULT_TOPK_RANK,
    KTH_HOOK_TOPK_SEG_CAP,
    KTH_OK,
    KTH_PATH_LDS,
    KTH_PATH_RADIX,
    KTH_PATH_WINDOW,
    KTH_PATH_WINDOW_FALLBACK,
    KTH_ROWS_MAX_COLS,
    KTH_STATS_WORDS,
    KTH_TOPK_MAX_COLS,
    IntVector,
    KthError,
    KthLibraryMissing,
    KthStats,
    check,
    check_single_runtime,
    hip_runtimes,
    load,
    strerror,
)

LIB = load()

# synthetic input families (oracle/kth_oracle.h enum ko_dist)
UNIFORM_FULL, UNIFORM_HALF, UNIFORM_REF, ALL_EQUAL, FEW_DISTINCT, SORTED_ASC, SORTED_DESC, MOD_1000 = range(8)
FAMILIES = {
    "uniform_full": UNIFORM_FULL,
    "uniform_half": UNIFORM_HALF,
    "uniform_ref": UNIFORM_REF,
    "all_equal": ALL_EQUAL,
    "few_distinct": FEW_DISTINCT,
    "sorted_asc": SORTED_ASC,
    "sorted_desc": SORTED_DESC,
    "mod_1000": MOD_1000,
}
DEFAULT_SEED = 0x5EED0001


def device_count():
    return LIB.kth_device_count()


def _ptr(x):
    """Raw address of a torch tensor / numpy array / int."""
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(f"cannot take the address of {type(x)}")


def _numel(x):
    return x.numel() if hasattr(x, "numel") else len(x)


def _stream_handle(stream):
    """hipStream_t of a torch stream (0 / None = the null stream, torch's default)."""
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream or None
    return stream.cuda_stream or None  # torch.cuda.Stream


class Selector:
    """A kth_ctx: scratch, stream and timing for repeated selections on one GPU."""

    def __init__(self, device=0, stream=None):
        self._ctx = ctypes.c_void_p()
        check(LIB.kth_ctx_create(device, ctypes.byref(self._ctx)), "kth_ctx_create")
        self.device = device
        if stream is not None:
            self.set_stream(stream)

    # -- lifecycle ---------------------------------------------------------
    def close(self):
        if self._ctx:
            LIB.kth_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    @property
    def handle(self):
        return self._ctx

    def set_stream(self, stream):
        if stream is not None and not isinstance(stream, int):
            check_single_runtime()  # a torch stream handle is only meaningful to torch's runtime
        check(LIB.kth_ctx_set_stream(self._ctx, _stream_handle(stream)), "kth_ctx_set_stream")

    def sync(self):
        check(LIB.kth_ctx_sync(self._ctx), "kth_ctx_sync")

    def reserve(self, n):
        check(LIB.kth_ctx_reserve(self._ctx, int(n)), "kth_ctx_reserve")

    # -- selection ---------------------------------------------------------
    def select(self, keys, k, n=None):
        """k-th smallest (1-based) of int32 keys (host numpy array or device tensor)."""
        if n is None:
            n = keys.numel() if hasattr(keys, "numel") else len(keys)
        if isinstance(keys, np.ndarray):
            keys = np.ascontiguousarray(keys, dtype=np.int32)
        out = ctypes.c_int32()
        check(LIB.kth_select_i32_ctx(self._ctx, _ptr(keys), int(n), int(k), ctypes.byref(out)),
              "kth_select_i32_ctx")
        return out.value

    def select_async(self, d_keys, n, k, d_out):
        """Enqueue a select of device keys; the answer lands in device int32 *d_out."""
        check(LIB.kth_select_i32_async(self._ctx, _ptr(d_keys), int(n), int(k), _ptr(d_out)),
              "kth_select_i32_async")

    def coop(self):
        """True while the ctx runs the cooperative grid-barrier kernels (kth_ctx_coop)."""
        r = LIB.kth_ctx_coop(self._ctx)
        if r < 0:
            check(r, "kth_ctx_coop")
        return bool(r)

    def test_hook(self, hook, value):
        """TESTS ONLY: turn a fault injector of this ctx on or off
        (kth_ctx_test_hook; KTH_HOOK_* in include/kth.h)."""
        check(LIB.kth_ctx_test_hook(self._ctx, int(hook), int(value)), "kth_ctx_test_hook")

    def stats(self):
        st = KthStats()
        check(LIB.kth_ctx_last_stats(self._ctx, ctypes.byref(st)), "kth_ctx_last_stats")
        return st.as_dict()

    def rows(self, d_keys, rows, cols, k, d_out, f32=False):
        fn = LIB.kth_select_rows_f32 if f32 else LIB.kth_select_rows_i32
        check(fn(self._ctx, _ptr(d_keys), int(rows), int(cols), int(k), _ptr(d_out)), "kth_select_rows")

    def topk_rows(self, d_keys, rows, cols, k, d_vals=None, d_idx=None, largest=False, f32=False):
        """Per row: the k smallest (largest=True: largest) keys and their columns,
        in column order, ties broken by column (kth_topk_rows_*)."""
        fn = LIB.kth_topk_rows_f32 if f32 else LIB.kth_topk_rows_i32
        check(fn(self._ctx, _ptr(d_keys), int(rows), int(cols), int(k), 1 if largest else 0,
                 _ptr(d_vals) if d_vals is not None else None, _ptr(d_idx) if d_idx is not None else None),
              "kth_topk_rows")

    def topk(self, d_keys, n, k, d_vals=None, d_idx=None, largest=False):
        """The k smallest (largest=True: largest) int32 keys of n device keys and
        their int64 indices, in index order, ties broken by index (kth_topk_i32;
        asynchronous on the ctx stream)."""
        check(LIB.kth_topk_i32(self._ctx, _ptr(d_keys), int(n), int(k), 1 if largest else 0,
                               _ptr(d_vals) if d_vals is not None else None,
                               _ptr(d_idx) if d_idx is not None else None), "kth_topk_i32")

    def fill(self, d_out, n, family=UNIFORM_FULL, seed=DEFAULT_SEED, param=0, offset=0, n_total=None):
        if isinstance(family, str):
            family = FAMILIES[family]
        if n_total is None:
            n_total = offset + n
        check(LIB.kth_fill_synthetic(self._ctx, _ptr(d_out), int(n), int(offset), int(n_total), int(family),
                                      ctypes.c_uint64(seed), int(param)), "kth_fill_synthetic")

    # -- timing ------------------------------------------------------------
    def enable_timing(self, on=True):
        check(LIB.kth_ctx_enable_timing(self._ctx, 1 if on else 0), "kth_ctx_enable_timing")

    def take_timing(self):
        """(selects, dominant-kernel ms summed, whole-select ms summed) since the last call."""
        n = ctypes.c_int64()
        m = ctypes.c_double()
        t = ctypes.c_double()
        check(LIB.kth_ctx_take_timing(self._ctx, ctypes.byref(n), ctypes.byref(m), ctypes.byref(t)),
              "kth_ctx_take_timing")
        return n.value, m.value, t.value


def kth_select(keys, k):
    """One-shot (data, n, k) -> value: kth_select_i32 (kth-problem-seq.c:32-33)."""
    if isinstance(keys, np.ndarray):
        keys = np.ascontiguousarray(keys, dtype=np.int32)
        n = keys.size
    else:
        n = keys.numel()
    out = ctypes.c_int32()
    check(LIB.kth_select_i32(_ptr(keys), int(n), int(k), ctypes.byref(out)), "kth_select_i32")
    return out.value


class ShardedSelector:
    """One process, several GPUs (kth_sharded_*): shard i lives on devices[i];
    the union's k-th smallest through grouped RCCL collectives
    (replaces TODO-kth-problem-cgm.c:81-278 without one process per rank)."""

    def __init__(self, devices):
        self.devices = [int(d) for d in devices]
        arr = (ctypes.c_int * len(self.devices))(*self.devices)
        self._h = ctypes.c_void_p()
        check(LIB.kth_sharded_create(arr, len(self.devices), ctypes.byref(self._h)), "kth_sharded_create")

    def select(self, shards, k, sizes=None):
        """shards: one device tensor per device (int32); sizes default to numel()."""
        if len(shards) != len(self.devices):
            raise ValueError(f"{len(shards)} shards for {len(self.devices)} devices")
        sizes = [_numel(s) for s in shards] if sizes is None else [int(x) for x in sizes]
        ptrs = (ctypes.c_void_p * len(shards))(*[_ptr(s) for s in shards])
        ns = (ctypes.c_int64 * len(shards))(*sizes)
        out = ctypes.c_int32()
        check(LIB.kth_sharded_select_i32(self._h, ptrs, ns, int(k), ctypes.byref(out)), "kth_sharded_select_i32")
        return out.value

    def enqueue_us(self):
        """Host microseconds the last select spent enqueueing (kth_sharded_enqueue_us)."""
        return LIB.kth_sharded_enqueue_us(self._h)

    def close(self):
        if self._h:
            LIB.kth_sharded_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass


def select_sharded(shards, k, sizes=None):
    """One-shot kth_select_i32_sharded: each shard's device from its pointer."""
    sizes = [_numel(s) for s in shards] if sizes is None else [int(x) for x in sizes]
    ptrs = (ctypes.c_void_p * len(shards))(*[_ptr(s) for s in shards])
    ns = (ctypes.c_int64 * len(shards))(*sizes)
    out = ctypes.c_int32()
    check(LIB.kth_select_i32_sharded(ptrs, ns, len(shards), int(k), ctypes.byref(out)), "kth_select_i32_sharded")
    return out.value


class IntVec:
    """The reference's IntVector (vector.h:7-11) owned through libkth.so's twin."""

    def __init__(self, capacity):
        self.p = LIB.VecNew(int(capacity))
        if not self.p:
            raise MemoryError("VecNew")

    @classmethod
    def from_array(cls, a):
        a = np.ascontiguousarray(a, dtype=np.int32)
        v = cls(max(1, a.size))
        ctypes.memmove(v.p.contents.data, a.ctypes.data, a.size * 4)
        v.p.contents.size = a.size
        return v

    def add(self, x):
        return LIB.VecAdd(self.p, int(x))

    def get(self, i):
        return LIB.VecGet(self.p, int(i))

    def size(self):
        return LIB.VecGetSize(self.p)

    def array(self):
        n = self.p.contents.size
        return np.ctypeslib.as_array(self.p.contents.data, shape=(n,)).copy() if n else np.empty(0, np.int32)

    def quicksort(self):
        LIB.VecQuickSort(self.p)

    def kth_select(self, k):
        """VecKthSelect: GPU drop-in for VecQuickSort + VecGet(k-1), VecGet sentinels kept."""
        return LIB.VecKthSelect(self.p, int(k))

    def kth_select_ex(self, k):
        out = ctypes.c_int()
        check(LIB.VecKthSelectEx(self.p, int(k), ctypes.byref(out)), "VecKthSelectEx")
        return out.value

    def close(self):
        if self.p:
            LIB.VecDelete(self.p)
            self.p = None

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001
            pass
