"""Pins the CPU oracle (oracle/liboracle.so) to the reference's own outputs.

tests/golden/expected.json was produced by tests/golden/make_golden.py from the
reference compiled out of /root/reference (oracle/build_ref.sh): the seq select
block of vector.c and `mpirun -n P` of TODO-kth-problem-cgm.c.  These tests do
not need the reference or a GPU.
"""
import ctypes
import hashlib

import numpy as np
import pytest

import gen as G
from conftest import load_input, true_kth


def test_fixture_inventory(golden):
    cases = golden["cases"]
    fams = {c["family"] for c in cases}
    assert {"uniform_full", "uniform_half", "uniform_ref", "all_equal", "few_distinct", "sorted_asc",
            "sorted_desc", "mod_1000"} <= fams
    assert {1, 7, 1000, 4093, 16384} <= {c["n"] for c in cases}
    # the reference's defects are represented
    assert any(c["seq_ref_defect"] for c in cases)
    assert any(v == "livelock" for c in cases for v in c["cgm_ref"].values())


def test_true_kth_matches_fixtures(golden, oracle):
    for c in golden["cases"]:
        a = load_input(c["input"])
        assert true_kth(oracle, a, c["k"]) == c["true"], c
        assert oracle.ko_rank_check(a.ctypes.data, a.size, c["k"], c["true"]) == 1


def test_seq_restatement_matches_reference(golden, oracle):
    """ko_seq_ref restates kth-problem-seq.c:32-33 including the vector.c:6-8
    comparator overflow: it must reproduce the reference's WRONG answers too."""
    for c in golden["cases"]:
        a = load_input(c["input"])
        assert oracle.ko_seq_ref(a.ctypes.data, a.size, c["k"]) == c["seq_ref"], c


def test_cgm_restatement_matches_reference(golden, oracle):
    """ko_cgm_ref restates TODO-kth-problem-cgm.c:76-285: same answers on every
    terminating run, and it reports the livelocks the reference spins in."""
    mismatches = []
    for c in golden["cases"]:
        a = load_input(c["input"])
        for p, ref in c["cgm_ref"].items():
            out = ctypes.c_int32()
            rounds = ctypes.c_int()
            found = ctypes.c_int()
            st = oracle.ko_cgm_ref(a.ctypes.data, a.size, c["k"], int(p), 500, ctypes.byref(out),
                                   ctypes.byref(rounds), ctypes.byref(found))
            if ref == "livelock":
                if st != 1:
                    mismatches.append((c["input"], c["k"], p, "ref livelocks, restatement", st, out.value))
            else:
                if st != 0 or out.value != ref:
                    mismatches.append((c["input"], c["k"], p, ref, st, out.value))
                # the line the reference printed: :289 (found by a pivot's 3-way
                # count, :194-201) or :280 (the final gather + sort)
                if (289 if found.value else 280) != c["cgm_ref_line"][p]:
                    mismatches.append((c["input"], c["k"], p, "line", c["cgm_ref_line"][p], found.value))
    assert not mismatches, mismatches[:10]


def test_generators_agree(oracle):
    """numpy gen.py == ko_gen (C) bit for bit (the device generator is pinned
    to gen.py in the GPU tests)."""
    for fam in range(8):
        for n, off, tot in ((1, 0, 1), (1000, 0, 1000), (4096, 12345, 1 << 20), (1 << 16, 0, 1 << 30)):
            a = G.gen(n, fam, 0x5EED0001, 7, offset=off, n_total=tot)
            b = np.empty(n, dtype=np.int32)
            oracle.ko_gen(b.ctypes.data, n, off, tot, fam, 0x5EED0001, 7)
            np.testing.assert_array_equal(a, b, err_msg=f"family {fam} n {n}")
    assert oracle.ko_hash(1, 2) == int(G.hash64(1, np.array([2], dtype=np.uint64))[0])


def test_rank_certificate_semantics(oracle):
    a = np.array([5, 1, 5, 3, 5], dtype=np.int32)
    assert oracle.ko_rank_check(a.ctypes.data, 5, 1, 1) == 1
    assert oracle.ko_rank_check(a.ctypes.data, 5, 2, 3) == 1
    for k in (3, 4, 5):
        assert oracle.ko_rank_check(a.ctypes.data, 5, k, 5) == 1
    assert oracle.ko_rank_check(a.ctypes.data, 5, 3, 3) == 0


@pytest.mark.slow
def test_shipped_generators_and_answers(golden, oracle):
    """The unmodified shipped programs (n = 1e8): the restated generators
    reproduce their exact input streams (sha256 of the VecAdd dump) and the
    restated seq/CGM reproduce their printed answers."""
    shipped = [r for r in golden.get("shipped", []) if "generator" in r]
    if not shipped:
        pytest.skip("no shipped pins")
    gens = {"kth-problem-seq.c:26-28": oracle.ko_gen_shipped_seq,
            "TODO-kth-problem-cgm.c:10-17": oracle.ko_gen_shipped_cgm}
    seen = set()
    for rec in shipped:
        key = (rec["generator"], rec["time_seed"])
        a = np.empty(rec["n"], dtype=np.int32)
        gens[rec["generator"]](a.ctypes.data, rec["n"], rec["time_seed"])
        if key not in seen:
            assert hashlib.sha256(a.astype("<i4").tobytes()).hexdigest() == rec["input_sha256"], rec
            seen.add(key)
        assert int(np.partition(a, rec["k"] - 1)[rec["k"] - 1]) == rec["true"]
        if rec["program"].startswith("seq") and rec["k"] == 250:
            assert oracle.ko_seq_ref(a.ctypes.data, a.size, rec["k"]) == rec["printed"], rec
        if rec["program"].startswith("cgm") and rec["printed"] != "livelock":
            out = ctypes.c_int32()
            r = ctypes.c_int()
            f = ctypes.c_int()
            assert oracle.ko_cgm_ref(a.ctypes.data, a.size, rec["k"], rec["P"], 500, ctypes.byref(out),
                                     ctypes.byref(r), ctypes.byref(f)) == 0
            assert out.value == rec["printed"], rec


def test_large_fixtures_pin_the_restatement(golden, oracle):
    """The radix/window-size fixtures (n in {16385, 2^20, 2^22 + 1}): the
    generator reproduces each input (sha256), and the restated seq and CGM
    reproduce the reference's answers, livelocks included."""
    large = golden.get("large")
    if not large:
        pytest.skip("no large fixtures")
    inputs = {}
    mismatches = []
    for c in large:
        key = (c["dist"], c["param"], c["n"])
        if key not in inputs:
            a = G.gen(c["n"], c["dist"], c["seed"], c["param"])
            assert hashlib.sha256(a.astype("<i4").tobytes()).hexdigest() == c["input_sha256"], c
            inputs = {key: a}
        a = inputs[key]
        assert true_kth(oracle, a, c["k"]) == c["true"], c
        if c["n"] <= 1 << 20:  # qsort of 4 Mi keys per case is slow for the CPU suite
            assert oracle.ko_seq_ref(a.ctypes.data, a.size, c["k"]) == c["seq_ref"], c
        for p, ref in c["cgm_ref"].items():
            out, rounds, found = ctypes.c_int32(), ctypes.c_int(), ctypes.c_int()
            st = oracle.ko_cgm_ref(a.ctypes.data, a.size, c["k"], int(p), 500, ctypes.byref(out),
                                   ctypes.byref(rounds), ctypes.byref(found))
            if (ref == "livelock" and st != 1) or (ref != "livelock" and (st != 0 or out.value != ref)):
                mismatches.append((c["family"], c["n"], c["k"], p, ref, st, out.value))
            if ref != "livelock" and (289 if found.value else 280) != c["cgm_ref_line"][p]:  # the printed line
                mismatches.append((c["family"], c["n"], c["k"], p, "line", c["cgm_ref_line"][p], found.value))
    assert not mismatches, mismatches[:10]
    assert any(c["seq_ref_defect"] for c in large) and any(v == "livelock" for c in large
                                                          for v in c["cgm_ref"].values())
