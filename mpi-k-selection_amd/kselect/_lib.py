"""ctypes binding of libkth.so (include/kth.h, include/vector.h).

The library is built in-tree by ``make -C mpi-k-selection_amd`` (or
``__graft_entry__.build()``) into ``mpi-k-selection_amd/lib/libkth.so``.  There
is no fallback: if the shared library is missing, importing this module raises.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(HERE)
LIB_PATH = os.environ.get("KTH_LIB") or os.path.join(PKG_ROOT, "lib", "libkth.so")

KTH_OK = 0
KTH_EINVAL = -1
KTH_ENOMEM = -2
KTH_EHIP = -3
KTH_ENODEV = -4
KTH_EINTERNAL = -5
KTH_ECOMM = -6

KTH_PATH_LDS, KTH_PATH_RADIX, KTH_PATH_WINDOW, KTH_PATH_WINDOW_FALLBACK = 1, 2, 3, 4
KTH_STATS_WORDS = 8 + 2 * 2048
KTH_DIST_DONE = 3  # kth_dist_level: no collective left, call kth_dist_result
KTH_DIST_MAX_LEVELS = 3
KTH_ROWS_MAX_COLS = 16384
KTH_TOPK_MAX_COLS = 4096
# kth_ctx_test_hook (tests only): fault injectors, off in every new ctx
KTH_HOOK_FAULT_TOPK_RANK, KTH_HOOK_FAULT_BARRIER, KTH_HOOK_TOPK_SEG_CAP = 1, 2, 3

c_i32p = ctypes.POINTER(ctypes.c_int32)
c_u32p = ctypes.POINTER(ctypes.c_uint32)
c_u64p = ctypes.POINTER(ctypes.c_uint64)
c_vp = ctypes.c_void_p


class KthStats(ctypes.Structure):  # include/kth.h kth_stats
    _fields_ = [
        ("path", ctypes.c_int32),
        ("mode", ctypes.c_int32),
        ("lo_key", ctypes.c_uint32),
        ("hi_key", ctypes.c_uint32),
        ("n", ctypes.c_uint64),
        ("k", ctypes.c_uint64),
        ("cnt_lt", ctypes.c_uint64),
        ("cnt_eq_lo", ctypes.c_uint64),
        ("cnt_eq_hi", ctypes.c_uint64),
        ("candidates", ctypes.c_uint64),
        ("capacity", ctypes.c_uint64),
        ("answer", ctypes.c_int32),
        ("error", ctypes.c_int32),
    ]

    def as_dict(self):
        return {f: getattr(self, f) for f, _ in self._fields_}


class IntVector(ctypes.Structure):  # include/vector.h (reference vector.h:7-11)
    _fields_ = [("size", ctypes.c_int), ("capacity", ctypes.c_int), ("data", ctypes.POINTER(ctypes.c_int))]


IntVectorPtr = ctypes.POINTER(IntVector)


class KthError(RuntimeError):
    def __init__(self, code, what=""):
        self.code = code
        super().__init__(f"{what}: {code} ({strerror(code)})" if what else f"{code} ({strerror(code)})")


class KthLibraryMissing(ImportError):
    pass


# name -> (restype, argtypes); every entry point of include/kth.h and include/vector.h
PROTOS = {
    # kth.h
    "kth_strerror": (ctypes.c_char_p, [ctypes.c_int]),
    "kth_version": (ctypes.c_int, []),
    "kth_build_id": (ctypes.c_char_p, []),
    "kth_device_count": (ctypes.c_int, []),
    "kth_select_i32": (ctypes.c_int, [c_vp, ctypes.c_int64, ctypes.c_int64, c_i32p]),
    "kth_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(c_vp)]),
    "kth_ctx_destroy": (ctypes.c_int, [c_vp]),
    "kth_ctx_set_stream": (ctypes.c_int, [c_vp, c_vp]),
    "kth_ctx_sync": (ctypes.c_int, [c_vp]),
    "kth_ctx_reserve": (ctypes.c_int, [c_vp, ctypes.c_int64]),
    "kth_select_i32_ctx": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int64, c_i32p]),
    "kth_select_i32_async": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int64, c_vp]),
    "kth_ctx_last_stats": (ctypes.c_int, [c_vp, ctypes.POINTER(KthStats)]),
    "kth_ctx_coop": (ctypes.c_int, [c_vp]),
    "kth_ctx_test_hook": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.c_int64]),
    "kth_ctx_enable_timing": (ctypes.c_int, [c_vp, ctypes.c_int]),
    "kth_ctx_take_timing": (ctypes.c_int, [c_vp, ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double),
                                           ctypes.POINTER(ctypes.c_double)]),
    "kth_select_rows_i32": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, c_vp]),
    "kth_select_rows_f32": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, c_vp]),
    "kth_topk_rows_i32": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int,
                                         c_vp, c_vp]),
    "kth_topk_rows_f32": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int32, ctypes.c_int,
                                         c_vp, c_vp]),
    "kth_topk_i32": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, c_vp, c_vp]),
    "kth_fill_synthetic": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                                          ctypes.c_uint64, ctypes.c_int32]),
    "kth_dist_begin": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int64]),
    "kth_dist_sample": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, c_vp, ctypes.c_int64]),
    "kth_dist_window": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64]),
    "kth_dist_scan": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64]),
    "kth_dist_level": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int64, ctypes.c_int]),
    "kth_dist_result": (ctypes.c_int, [c_vp, c_vp]),
    "kth_dist_result_early": (ctypes.c_int, [c_vp, c_vp]),
    "kth_dist_select_rccl": (ctypes.c_int, [c_vp, c_vp, c_vp, c_vp, ctypes.c_int, c_vp, ctypes.c_int64, ctypes.c_int64,
                                            ctypes.c_int64, c_vp, c_vp, c_vp, ctypes.c_int64, c_vp, ctypes.c_int]),
    "kth_dist_sample_size": (ctypes.c_int64, [ctypes.c_int64]),
    "kth_sample_chunk": (ctypes.c_int, []),
    "kth_window_z": (ctypes.c_double, []),
    "kth_dist_cand_capacity": (ctypes.c_int64, [ctypes.c_int64]),
    "kth_window_slack64": (ctypes.c_int, []),
    "kth_sharded_create": (ctypes.c_int, [c_vp, ctypes.c_int, ctypes.POINTER(c_vp)]),
    "kth_sharded_destroy": (ctypes.c_int, [c_vp]),
    "kth_sharded_select_i32": (ctypes.c_int, [c_vp, c_vp, c_vp, ctypes.c_int64, c_i32p]),
    "kth_select_i32_sharded": (ctypes.c_int, [c_vp, c_vp, ctypes.c_int, ctypes.c_int64, c_i32p]),
    "kth_sharded_enqueue_us": (ctypes.c_double, [c_vp]),
    "kth_sharded_sample_split": (ctypes.c_int64, [c_vp, ctypes.c_int, c_vp]),
    # vector.h
    "VecNew": (IntVectorPtr, [ctypes.c_int]),
    "VecAdd": (ctypes.c_int, [IntVectorPtr, ctypes.c_int]),
    "VecDelete": (None, [IntVectorPtr]),
    "VecErase": (ctypes.c_int, [IntVectorPtr, ctypes.c_int]),
    "MinFind": (ctypes.c_int, [IntVectorPtr]),
    "MaxFind": (ctypes.c_int, [IntVectorPtr]),
    "AverageFind": (ctypes.c_double, [IntVectorPtr]),
    "VecGetCapacity": (ctypes.c_int, [IntVectorPtr]),
    "VecGetSize": (ctypes.c_int, [IntVectorPtr]),
    "VecIsFull": (ctypes.c_int, [IntVectorPtr]),
    "VecSet": (ctypes.c_int, [IntVectorPtr, ctypes.c_int, ctypes.c_int]),
    "VecGet": (ctypes.c_int, [IntVectorPtr, ctypes.c_int]),
    "VecSearch": (ctypes.c_int, [IntVectorPtr, ctypes.c_int, ctypes.c_int]),
    "VecQuickSort": (None, [IntVectorPtr]),
    "VecQuickSort2": (None, [IntVectorPtr]),
    "VecBinarySearch": (ctypes.c_int, [IntVectorPtr, ctypes.c_int]),
    "VecBinarySearch2": (ctypes.c_int, [IntVectorPtr, ctypes.c_int]),
    "VecKthSelect": (ctypes.c_int, [IntVectorPtr, ctypes.c_int]),
    "VecKthSelectEx": (ctypes.c_int, [IntVectorPtr, ctypes.c_int, ctypes.POINTER(ctypes.c_int)]),
}

_lib = None


def hip_runtimes():
    """Distinct HIP runtime files (libamdhip64) mapped into this process."""
    found = set()
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                path = line.rsplit(None, 1)[-1] if "/" in line else ""
                if "libamdhip64" in os.path.basename(path):
                    found.add(os.path.realpath(path))
    except OSError:
        pass
    return sorted(found)


def check_single_runtime():
    """Raise if two HIP runtimes are loaded.  Streams, events and the null
    stream of one runtime mean nothing to the other: work libkth.so enqueues
    would not be ordered against torch's streams (a .item() could read an
    answer buffer before the select that writes it), and a torch stream handle
    passed to libkth.so would be an invalid handle."""
    rts = hip_runtimes()
    if len(rts) > 1:
        raise RuntimeError(
            "two HIP runtimes are loaded in this process (" + ", ".join(rts) + "); "
            "import torch before libkth.so is loaded (kselect does this itself when torch is importable)")


def load():
    """Load libkth.so once; raise KthLibraryMissing if it is not built.

    torch (when importable) is imported first: libkth.so needs the HIP runtime
    by its soname (libamdhip64.so.7), which then binds to the copy torch has
    already loaded, so the process holds ONE HIP runtime and libkth.so's
    streams and torch's are the same objects.  Loaded the other way round, torch
    would add its bundled runtime next to /opt/rocm's (check_single_runtime)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise KthLibraryMissing(
            f"libkth.so not found at {LIB_PATH}; build it with `make -C {PKG_ROOT}` "
            "(there is no CPU fallback)")
    try:
        import torch  # noqa: F401 -- see the docstring: one HIP runtime per process
    except ImportError:
        pass
    lib = ctypes.CDLL(LIB_PATH)
    check_single_runtime()
    for name, (res, args) in PROTOS.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def strerror(code):
    try:
        return load().kth_strerror(code).decode()
    except Exception:  # noqa: BLE001 -- only used for messages
        return "?"


def check(code, what=""):
    if code != KTH_OK:
        raise KthError(code, what)
    return code
