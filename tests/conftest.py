"""Shared test setup.  `-m gpu` tests need a real MI355X and call libkth.so
through its C-ABI; everything else runs on CPU (oracle vs golden vectors, host
logic, ABI/export checks, gloo multi-process orchestration)."""
import ctypes
import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "mpi-k-selection_amd")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, GOLDEN):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an AMD GPU (MI355X); run with -m gpu")
    config.addinivalue_line("markers", "slow: long CPU test (reference-sized inputs)")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "expected.json")) as f:
        return json.load(f)


def load_input(name):
    return np.fromfile(os.path.join(GOLDEN, "inputs", name), dtype="<i4")


@pytest.fixture(scope="session")
def oracle():
    """oracle/liboracle.so -- the CPU restatement (test infrastructure only)."""
    path = os.environ.get("KTH_ORACLE_LIB") or os.path.join(REPO, "oracle", "liboracle.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "liboracle.so"], check=True)
    lib = ctypes.CDLL(path)
    i32p = ctypes.POINTER(ctypes.c_int32)
    lib.ko_hash.restype = ctypes.c_uint64
    lib.ko_hash.argtypes = [ctypes.c_uint64, ctypes.c_uint64]
    lib.ko_gen.restype = None
    lib.ko_gen.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int64, ctypes.c_int,
                           ctypes.c_uint64, ctypes.c_int32]
    lib.ko_true_kth.restype = ctypes.c_int
    lib.ko_true_kth.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, i32p]
    lib.ko_rank_check.restype = ctypes.c_int
    lib.ko_rank_check.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64, ctypes.c_int32]
    lib.ko_seq_ref.restype = ctypes.c_int32
    lib.ko_seq_ref.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_int64]
    lib.ko_cgm_ref.restype = ctypes.c_int
    lib.ko_cgm_ref.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, i32p,
                               ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]
    lib.ko_gen_shipped_seq.restype = None
    lib.ko_gen_shipped_seq.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint]
    lib.ko_gen_shipped_cgm.restype = None
    lib.ko_gen_shipped_cgm.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_uint]
    return lib


def true_kth(oracle, a, k):
    a = np.ascontiguousarray(a, dtype=np.int32)
    out = ctypes.c_int32()
    assert oracle.ko_true_kth(a.ctypes.data, a.size, k, ctypes.byref(out)) == 0
    return out.value


@pytest.fixture(scope="session")
def gpu():
    """The product library on cuda:0 (skips when no GPU is visible)."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import kselect
    sel = kselect.Selector(0)
    yield sel
    sel.close()
