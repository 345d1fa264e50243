"""CPU checks of the drop-in boundary: libkth.so loads, exports every entry
point declared in include/*.h, keeps the reference IntVector ABI and host
semantics, and has no CPU fallback (compute calls fail loudly without a GPU)."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from conftest import PKG, REPO

LIB = os.environ.get("KTH_LIB") or os.path.join(PKG, "lib", "libkth.so")
REF_VEC = os.path.join(REPO, "oracle", "_ref", "libvector_ref.so")


def declared_functions(header):
    text = open(os.path.join(REPO, "include", header)).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    text = re.sub(r"#define[^\n]*", "", text)
    names = re.findall(r"\b([A-Za-z_]\w*)\s*\([^;{]*\)\s*;", text)
    return sorted({n for n in names if n not in ("sizeof",)})


@pytest.fixture(scope="module")
def lib():
    import kselect
    return kselect.LIB


def test_headers_declare_expected_api():
    k = declared_functions("kth.h")
    v = declared_functions("vector.h")
    for name in ("kth_select_i32", "kth_select_i32_async", "kth_ctx_create", "kth_select_rows_f32",
                 "kth_dist_scan", "kth_dist_level", "kth_dist_result", "kth_dist_result_early"):
        assert name in k
    # the reference's 18 prototypes (vector.h:13-33) + the drop-in select
    ref18 = ["VecNew", "VecAdd", "VecDelete", "VecErase", "MinFind", "MaxFind", "AverageFind", "VecGetCapacity",
             "VecGetSize", "VecIsFull", "VecSet", "VecGet", "VecSearch", "VecQuickSort", "VecQuickSort2",
             "VecBinarySearch", "VecBinarySearch2"]
    assert len(ref18) == 17  # the reference header has 17 functions + the struct
    for name in ref18 + ["VecKthSelect", "VecKthSelectEx"]:
        assert name in v, name


def test_library_exports_every_declared_symbol(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True, check=True).stdout
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for h in ("kth.h", "vector.h"):
        for name in declared_functions(h):
            assert name in exported, f"{name} declared in include/{h} but not exported by libkth.so"


def test_python_binding_covers_every_symbol():
    from kselect._lib import PROTOS
    for h in ("kth.h", "vector.h"):
        for name in declared_functions(h):
            assert name in PROTOS, name


def test_intvector_layout():
    from kselect import IntVector
    assert ctypes.sizeof(IntVector) == 16
    assert IntVector.size.offset == 0 and IntVector.capacity.offset == 4 and IntVector.data.offset == 8


def test_no_cpu_fallback(lib):
    """Without a GPU every compute entry point fails loudly (KTH_ENODEV)."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import kselect
    a = np.arange(100, dtype=np.int32)
    out = ctypes.c_int32(12345)
    assert lib.kth_select_i32(a.ctypes.data, 100, 50, ctypes.byref(out)) == kselect.KTH_ENODEV
    assert out.value == 12345
    with pytest.raises(kselect.KthError):
        kselect.Selector(0)
    v = kselect.IntVec.from_array(a)
    assert v.kth_select(5) == -3  # VecKthSelect's device-error sentinel


def test_topk_argument_checks(lib):
    """kth_topk_i32 validates before touching a device (include/kth.h contract)."""
    import kselect
    a = np.arange(16, dtype=np.int32)
    out = np.zeros(16, dtype=np.int32)
    for n, k in ((16, 0), (16, 17), (0, 1)):
        assert lib.kth_topk_i32(None, a.ctypes.data, n, k, 0, out.ctypes.data, None) == kselect.KTH_EINVAL
    assert lib.kth_topk_i32(None, a.ctypes.data, 16, 1, 0, None, None) == kselect.KTH_EINVAL


def test_missing_library_is_loud():
    code = ("import sys; sys.path.insert(0, %r); import kselect" % PKG)
    p = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, KTH_LIB="/nonexistent/libkth.so"),
                       capture_output=True, text=True)
    assert p.returncode != 0 and "KthLibraryMissing" in p.stderr


def _vec_ops(L, seed):
    """Random IntVector op sequence (no sort); returns the observable trace."""
    L.VecNew.restype = ctypes.c_void_p
    for name in ("VecAdd", "VecErase", "MinFind", "VecGetCapacity", "VecGetSize", "VecIsFull", "VecSet",
                 "VecGet", "VecSearch"):
        getattr(L, name).restype = ctypes.c_int
    L.AverageFind.restype = ctypes.c_double
    rng = np.random.default_rng(seed)
    v = ctypes.c_void_p(L.VecNew(4))
    trace = []
    for _ in range(400):
        op = rng.integers(0, 8)
        x = int(rng.integers(-1000, 1000))
        i = int(rng.integers(-2, 40))
        if op <= 2:
            trace.append(("add", L.VecAdd(v, x)))
        elif op == 3:
            trace.append(("erase", L.VecErase(v, i)))
        elif op == 4:
            trace.append(("set", L.VecSet(v, i, x)))
        elif op == 5:
            trace.append(("get", L.VecGet(v, i)))
        elif op == 6:
            trace.append(("search", L.VecSearch(v, i, x)))
        else:
            n = L.VecGetSize(v)
            # MinFind of an empty vector reads uninitialised data[0] in the reference
            trace.append(("stat", n, L.VecIsFull(v), L.MinFind(v) if n else None, L.AverageFind(v)))
    n = L.VecGetSize(v)
    trace.append(("final", [L.VecGet(v, j) for j in range(n)]))
    L.VecDelete(v)
    return trace


def test_intvector_semantics_match_reference():
    """Same observable behaviour as the reference vector.c on random op
    sequences (compiled from /root/reference into oracle/_ref)."""
    if not os.path.exists(REF_VEC):
        pytest.skip("oracle/_ref not built")
    ours = ctypes.CDLL(LIB)
    ref = ctypes.CDLL(REF_VEC)
    for seed in range(5):
        assert _vec_ops(ours, seed) == _vec_ops(ref, seed)


def test_quicksort_fixes_reference_comparator():
    """VecQuickSort sorts full-range keys; the reference's `*a - *b` does not."""
    import kselect
    rng = np.random.default_rng(1)
    a = rng.integers(-2 ** 31, 2 ** 31, size=4096, dtype=np.int64).astype(np.int32)
    v = kselect.IntVec.from_array(a)
    v.quicksort()
    np.testing.assert_array_equal(v.array(), np.sort(a))
    if os.path.exists(REF_VEC):
        ref = ctypes.CDLL(REF_VEC)
        from kselect import IntVector
        b = a.copy()
        iv = IntVector(b.size, b.size, b.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
        ref.VecQuickSort(ctypes.byref(iv))
        assert not np.array_equal(b, np.sort(a))  # the documented reference defect


def test_reference_driver_links_against_twin(tmp_path):
    """The reference's unmodified kth-problem-seq.c compiles and links against
    include/vector.h + libkth.so (ABI drop-in)."""
    src = "/root/reference/kth-problem-seq.c"
    if not os.path.exists(src):
        pytest.skip("reference not present")
    exe = tmp_path / "seq_on_twin"
    subprocess.run(["gcc", "-O2", "-w", "-I", os.path.join(REPO, "include"), src, "-L", os.path.dirname(LIB),
                    "-lkth", "-o", str(exe)], check=True)
    assert exe.exists()


def test_sharded_argument_checks(lib):
    """kth_select_i32_sharded / kth_sharded_*: bad arguments are EINVAL before
    any device work; without a GPU the compute entry points are ENODEV."""
    import torch
    import kselect
    a = np.arange(1000, dtype=np.int32)
    ptrs = (ctypes.c_void_p * 1)(a.ctypes.data)
    ns = (ctypes.c_int64 * 1)(1000)
    out = ctypes.c_int32(99)
    assert lib.kth_select_i32_sharded(None, ns, 1, 5, ctypes.byref(out)) == kselect.KTH_EINVAL
    assert lib.kth_select_i32_sharded(ptrs, None, 1, 5, ctypes.byref(out)) == kselect.KTH_EINVAL
    assert lib.kth_select_i32_sharded(ptrs, ns, 0, 5, ctypes.byref(out)) == kselect.KTH_EINVAL
    assert lib.kth_select_i32_sharded(ptrs, ns, 1, 5, None) == kselect.KTH_EINVAL
    h = ctypes.c_void_p()
    assert lib.kth_sharded_create(None, 1, ctypes.byref(h)) == kselect.KTH_EINVAL
    devs = (ctypes.c_int * 2)(0, 0)
    assert lib.kth_sharded_create(devs, 0, ctypes.byref(h)) == kselect.KTH_EINVAL
    assert lib.kth_sharded_select_i32(None, ptrs, ns, 5, ctypes.byref(out)) == kselect.KTH_EINVAL
    assert lib.kth_sharded_destroy(None) == kselect.KTH_EINVAL
    if not torch.cuda.is_available():
        assert lib.kth_select_i32_sharded(ptrs, ns, 1, 5, ctypes.byref(out)) == kselect.KTH_ENODEV
        assert lib.kth_sharded_create(devs, 1, ctypes.byref(h)) == kselect.KTH_ENODEV
        assert out.value == 99
    assert lib.kth_strerror(kselect.KTH_ECOMM).decode().startswith("RCCL")


def test_protocol_constants_exported(lib):
    """The tunables the gloo CPU backend mirrors are read from the library
    (tests/dist_cpu_backend.py), not restated: window z, sample chunk and
    size rule, candidate capacity."""
    import dist_cpu_backend as cb
    assert lib.kth_window_z() == 5.0 == cb.WINDOW_Z
    assert lib.kth_sample_chunk() == 1024 == cb.SAMPLE_CHUNK
    assert lib.kth_dist_sample_size(1 << 30) == 1 << 20
    assert lib.kth_dist_sample_size(100) == 64
    assert lib.kth_dist_cand_capacity(1 << 30) == (1 << 30) // 32
    assert lib.kth_dist_cand_capacity(1000) == 1 << 20
    idx = cb.sample_indices(1 << 24, (1 << 18) + 64)  # 257 chunks, the last one partial
    assert idx.size == (1 << 18) + 64 and idx[1024] == (1 << 24) // 257 and idx[-1] == 256 * ((1 << 24) // 257) + 63


def test_dist_one_call_and_test_hook_argument_checks(lib):
    """kth_dist_select_rccl and kth_ctx_test_hook refuse a missing ctx / null
    pointers / bad values with KTH_EINVAL before touching a device."""
    import kselect
    one = ctypes.c_void_p(1)
    args = [one, one, one, 2, one, 1 << 20, 1 << 21, 5, one, one, one, 1024, one, 1]
    assert lib.kth_dist_select_rccl(None, *args) == kselect.KTH_EINVAL
    for i in (0, 1, 2, 4, 8, 9, 10, 12):  # each pointer NULL in turn
        bad = list(args)
        bad[i] = None
        assert lib.kth_dist_select_rccl(one, *bad) == kselect.KTH_EINVAL, i
    bad = list(args)
    bad[11] = 32  # a per-rank sample under 64 keys
    assert lib.kth_dist_select_rccl(one, *bad) == kselect.KTH_EINVAL
    bad = list(args)
    bad[3] = 0  # world
    assert lib.kth_dist_select_rccl(one, *bad) == kselect.KTH_EINVAL
    assert lib.kth_ctx_test_hook(None, kselect.KTH_HOOK_FAULT_BARRIER, 1) == kselect.KTH_EINVAL


@pytest.mark.parametrize("first", ["kselect", "torch"])
def test_one_hip_runtime_whatever_the_import_order(first):
    """libkth.so and torch share ONE HIP runtime in a process, whichever is
    imported first.  libkth.so needs libamdhip64.so.7 by soname; torch bundles
    its own copy under that soname.  Loaded before torch, libkth.so used to pull
    /opt/rocm's runtime and torch then added its own: two null streams, so a
    torch .item() was not ordered after libkth's kernels (a world-1
    DistSelector read the previous select's answer) and torch stream handles
    were invalid in libkth (kth_dist_sample: HIP runtime error).  kselect now
    imports torch before loading the library and refuses a second runtime."""
    second = "torch" if first == "kselect" else "kselect"
    code = (f"import sys; sys.path.insert(0, {PKG!r}); import {first}; import {second}; import kselect; "
            "print(len(kselect.hip_runtimes())); kselect.check_single_runtime()")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    assert p.returncode == 0, p.stderr
    assert p.stdout.split()[-1] == "1", p.stdout


def test_second_hip_runtime_is_refused():
    """A process that loaded /opt/rocm's runtime through libkth.so before torch
    (bypassing kselect) holds two runtimes; kselect's check names them."""
    rocm = "/opt/rocm/lib/libamdhip64.so.7"
    if not os.path.exists(rocm):
        pytest.skip("no /opt/rocm runtime")
    code = (f"import ctypes, sys; ctypes.CDLL({LIB!r}); import torch; sys.path.insert(0, {PKG!r}); "
            "import kselect")
    p = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    assert p.returncode != 0 and "two HIP runtimes" in p.stderr, p.stderr[-2000:]
