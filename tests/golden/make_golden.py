#!/usr/bin/env python3
"""Generate the golden vectors in tests/golden/ FROM THE REFERENCE ITSELF.

Runs in the build container only (needs /root/reference and the binaries that
oracle/build_ref.sh compiles from it into oracle/_ref/).  Writes:

  tests/golden/inputs/<family>_n<N>.bin   raw little-endian int32 keys
  tests/golden/expected.json              per (input, k):
      true        sorted(a)[k-1] under signed int32 order (numpy)
      seq_ref     what the reference seq select block returns
                  (libvector_ref.so: VecQuickSort + VecGet(k-1), kth-problem-seq.c:32-33)
      cgm_ref     {P: value | "livelock"} from `mpirun -n P cgm_param`
                  (TODO-kth-problem-cgm.c with n, k parameterised; timeout => livelock)
      cgm_ref_line {P: 280 | 289 | "livelock"}: which of rank 0's two output
                  lines the run printed -- "kth element=%d \ntime: %f\n" (:280,
                  the final gather + sort) or "kth element %d\n time: %f\n" (:289,
                  a weighted-median pivot that the 3-way count found, :194-201)
  and a "shipped" section: the unmodified reference programs run as shipped
  (n = 1e8), seeded through the --wrap=time shim, with their printed answers.

  and a "large" section: n in {16385, 2^20, 2^22 + 1} (radix and window paths,
  BASELINE config 1), inputs regenerated from (family, seed, n) and pinned by
  sha256, expected outputs from the reference seq block and mpirun CGM.

Usage: python tests/golden/make_golden.py [--small] [--shipped] [--large] [--lines]
(--lines: re-run the CGM reference on the recorded small and large cases and
record only cgm_ref_line, checking that every value is reproduced)
"""
import argparse
import ctypes
import hashlib
import json
import os
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_DIR = os.path.join(REPO, "oracle", "_ref")
MPIRUN = os.environ.get("MPIRUN", "/opt/conda/bin/mpirun")
sys.path.insert(0, HERE)
import gen as G  # noqa: E402

NS = [1, 7, 1000, 4093, 16384]
PS = [2, 3, 4, 8]
FAMILIES = [
    ("uniform_full", G.UNIFORM_FULL, 0),
    ("uniform_half", G.UNIFORM_HALF, 0),
    ("uniform_ref", G.UNIFORM_REF, 0),
    ("all_equal", G.ALL_EQUAL, 7),
    ("all_equal_min", G.ALL_EQUAL, -(2 ** 31)),
    ("all_equal_max", G.ALL_EQUAL, 2 ** 31 - 1),
    ("few_distinct", G.FEW_DISTINCT, 0),
    ("sorted_asc", G.SORTED_ASC, 0),
    ("sorted_desc", G.SORTED_DESC, 0),
    ("mod_1000", G.MOD_1000, 0),
]
CGM_TIMEOUT = 2.0


class IntVector(ctypes.Structure):  # vector.h:7-11
    _fields_ = [("size", ctypes.c_int), ("capacity", ctypes.c_int), ("data", ctypes.POINTER(ctypes.c_int))]


def seq_ref(lib, a, k):
    buf = np.array(a, dtype=np.int32, copy=True)
    v = IntVector(len(buf), len(buf), buf.ctypes.data_as(ctypes.POINTER(ctypes.c_int)))
    lib.VecQuickSort(ctypes.byref(v))
    return int(lib.VecGet(ctypes.byref(v), ctypes.c_int(k - 1)))


_ANS = re.compile(r"kth element[= ]\s*(-?\d+)")
_LINE_280 = re.compile(r"kth element=(-?\d+) \ntime: [0-9.]+\n")  # TODO-kth-problem-cgm.c:280
_LINE_289 = re.compile(r"kth element (-?\d+)\n time: [0-9.]+\n")  # TODO-kth-problem-cgm.c:289


def cgm_line(stdout):
    """280 or 289: which of the reference's two answer lines rank 0 printed."""
    a, b = _LINE_280.search(stdout), _LINE_289.search(stdout)
    if bool(a) == bool(b):
        raise RuntimeError(f"cgm output has {'both' if a else 'neither'} answer lines: {stdout!r}")
    return 280 if a else 289


def run_cgm(binary, P, env, timeout):
    try:
        p = subprocess.run([MPIRUN, "-n", str(P), binary], env=env, capture_output=True,
                           text=True, timeout=timeout)
    except subprocess.TimeoutExpired:
        return "livelock", None
    m = _ANS.search(p.stdout)
    if not m:
        raise RuntimeError(f"cgm {binary} P={P}: no answer in {p.stdout!r} {p.stderr!r}")
    return int(m.group(1)), p.stdout


def run_cgm_line(binary, P, env, timeout):
    """(value, line) of one run; ("livelock", "livelock") on a timeout."""
    val, out = run_cgm(binary, P, env, timeout)
    return (val, "livelock") if out is None else (val, cgm_line(out))


def ks_for(n):
    return sorted({k for k in (1, 2, n // 2, n - 1, n) if 1 <= k <= n})


def small(lib):
    os.makedirs(os.path.join(HERE, "inputs"), exist_ok=True)
    cases = []
    for name, dist, param in FAMILIES:
        for n in NS:
            if name.startswith("all_equal_") and n not in (7, 4093):
                continue
            a = G.gen(n, dist, G.DEFAULT_SEED, param)
            fname = f"{name}_n{n}.bin"
            a.astype("<i4").tofile(os.path.join(HERE, "inputs", fname))
            srt = np.sort(a.astype(np.int64))
            for k in ks_for(n):
                case = {"input": fname, "family": name, "n": n, "k": k,
                        "true": int(srt[k - 1]), "seq_ref": seq_ref(lib, a, k), "cgm_ref": {}, "cgm_ref_line": {}}
                env = dict(os.environ, KO_N=str(n), KO_K=str(k), KO_TIME="1",
                           KO_INPUT=os.path.join(HERE, "inputs", fname))
                for P in PS:
                    val, line = run_cgm_line(os.path.join(REF_DIR, "cgm_param"), P, env, CGM_TIMEOUT)
                    case["cgm_ref"][str(P)] = val
                    case["cgm_ref_line"][str(P)] = line
                case["seq_ref_defect"] = case["seq_ref"] != case["true"]
                cases.append(case)
                print(name, n, k, case["true"], case["seq_ref"], case["cgm_ref"], flush=True)
    return cases


def livelock_cases(lib):
    """Full-range inputs on which the reference CGM livelocks (SURVEY 8(c) defect 2)."""
    out = []
    n, k = 4096, 2048
    for seed in range(1, 40):
        a = G.gen(n, G.UNIFORM_FULL, seed)
        fname = f"uniform_full_n{n}_seed{seed}.bin"
        path = os.path.join(HERE, "inputs", fname)
        a.astype("<i4").tofile(path)
        env = dict(os.environ, KO_N=str(n), KO_K=str(k), KO_TIME="1", KO_INPUT=path)
        val, _ = run_cgm(os.path.join(REF_DIR, "cgm_param"), 2, env, CGM_TIMEOUT)
        if val == "livelock":
            srt = np.sort(a.astype(np.int64))
            case = {"input": fname, "family": "uniform_full", "seed": seed, "n": n, "k": k,
                    "true": int(srt[k - 1]), "seq_ref": seq_ref(lib, a, k), "cgm_ref": {"2": val}}
            case["cgm_ref_line"] = {"2": "livelock"}
            for P in (3, 4, 8):
                case["cgm_ref"][str(P)], case["cgm_ref_line"][str(P)] = run_cgm_line(
                    os.path.join(REF_DIR, "cgm_param"), P, env, CGM_TIMEOUT)
            case["seq_ref_defect"] = case["seq_ref"] != case["true"]
            out.append(case)
            print("livelock", seed, case, flush=True)
            if len(out) >= 2:
                break
        else:
            os.remove(path)
    return out


LARGE_NS = [16385, 1 << 20, (1 << 22) + 1]  # radix path (n > 16384), BASELINE config 1, window path (n > 4 Mi)
LARGE_PS = [2, 8]


def large(lib):
    """Radix- and window-path sizes.  Inputs are NOT stored: each is the
    counter-based generator's output for (family, seed, param, n) -- gen.py,
    bit-identical to oracle ko_gen and the device's kth_fill_synthetic -- pinned
    by its sha256; the reference seq select block and the reference CGM under
    mpirun (P in LARGE_PS) give the expected outputs."""
    tmp = tempfile.mkdtemp(prefix="ko_large_")
    out = []
    for name, dist, param in FAMILIES:
        if name in ("all_equal_min", "all_equal_max"):
            continue
        for n in LARGE_NS:
            a = G.gen(n, dist, G.DEFAULT_SEED, param)
            path = os.path.join(tmp, "in.bin")
            a.astype("<i4").tofile(path)
            srt = np.sort(a.astype(np.int64))
            for k in sorted({1, n // 2, n}):
                case = {"family": name, "dist": dist, "param": param, "seed": G.DEFAULT_SEED, "n": n, "k": k,
                        "input_sha256": sha256_file(path), "true": int(srt[k - 1]),
                        "seq_ref": seq_ref(lib, a, k), "cgm_ref": {}, "cgm_ref_line": {}}
                env = dict(os.environ, KO_N=str(n), KO_K=str(k), KO_TIME="1", KO_INPUT=path)
                for P in LARGE_PS:
                    case["cgm_ref"][str(P)], case["cgm_ref_line"][str(P)] = run_cgm_line(
                        os.path.join(REF_DIR, "cgm_param"), P, env, 10.0)
                case["seq_ref_defect"] = case["seq_ref"] != case["true"]
                out.append(case)
                print("large", name, n, k, case["true"], case["seq_ref"], case["cgm_ref"], flush=True)
            os.remove(path)
    os.rmdir(tmp)
    return out


def sha256_file(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 24), b""):
            h.update(blk)
    return h.hexdigest()


def shipped():
    """The unmodified reference programs as shipped (n = 1e8), seeded via KO_TIME."""
    n = 100_000_000
    res = []
    tmp = tempfile.mkdtemp(prefix="ko_shipped_")
    _SEQ = re.compile(r"Solution found solution=(-?\d+)")
    for prog, k in (("seq_shipped", 250), ("seq_median_shipped", n // 2)):
        for t in (1, 1444444444):
            dump = os.path.join(tmp, f"{prog}_{t}.bin")
            env = dict(os.environ, KO_TIME=str(t), KO_DUMP=dump)
            p = subprocess.run([os.path.join(REF_DIR, prog)], env=env, capture_output=True, text=True,
                               timeout=600)
            printed = int(_SEQ.search(p.stdout).group(1))
            a = np.fromfile(dump, dtype="<i4")
            assert a.size == n
            true = int(np.partition(a, k - 1)[k - 1])
            rec = {"program": prog, "time_seed": t, "n": n, "k": k, "printed": printed, "true": true,
                   "input_sha256": sha256_file(dump), "generator": "kth-problem-seq.c:26-28"}
            print(rec, flush=True)
            res.append(rec)
            os.remove(dump)
    for prog, k in (("cgm_shipped", 150), ("cgm_median_shipped", n // 2)):
        for P in (2, 4):
            dump = os.path.join(tmp, f"{prog}_{P}.bin")
            env = dict(os.environ, KO_TIME="1", KO_DUMP=dump)
            val, _ = run_cgm(os.path.join(REF_DIR, prog), P, env, 300)
            a = np.fromfile(dump, dtype="<i4")
            assert a.size == n
            true = int(np.partition(a, k - 1)[k - 1])
            rec = {"program": prog, "P": P, "time_seed": 1, "n": n, "k": k, "printed": val, "true": true,
                   "input_sha256": sha256_file(dump), "generator": "TODO-kth-problem-cgm.c:10-17"}
            print(rec, flush=True)
            res.append(rec)
            os.remove(dump)
    # the shipped CGM on the synthetic families of BASELINE config 2 (n fixed at 1e8 by the source)
    for fam in ("uniform_half", "uniform_full"):
        a = G.gen(n, G.BY_NAME[fam], G.DEFAULT_SEED)
        path = os.path.join(tmp, f"{fam}.bin")
        a.astype("<i4").tofile(path)
        for prog, k in (("cgm_shipped", 150), ("cgm_median_shipped", n // 2)):
            true = int(np.partition(a, k - 1)[k - 1])
            for P in (2, 8):
                env = dict(os.environ, KO_TIME="1", KO_INPUT=path)
                val, _ = run_cgm(os.path.join(REF_DIR, prog), P, env, 60)
                rec = {"program": prog, "P": P, "family": fam, "seed": G.DEFAULT_SEED, "n": n, "k": k,
                       "printed": val, "true": true}
                print(rec, flush=True)
                res.append(rec)
        os.remove(path)
    os.rmdir(tmp)
    return res


def lines(doc):
    """cgm_ref_line for every recorded small and large case, from fresh runs of
    the same reference binary on the same inputs (each value must come out as
    recorded: the runs are deterministic under KO_TIME)."""
    tmp = tempfile.mkdtemp(prefix="ko_lines_")
    for c in doc["cases"] + doc["large"]:
        if "input" in c:
            path = os.path.join(HERE, "inputs", c["input"])
        else:
            path = os.path.join(tmp, "in.bin")
            G.gen(c["n"], c["dist"], c["seed"], c["param"]).astype("<i4").tofile(path)
            assert sha256_file(path) == c["input_sha256"], c
        env = dict(os.environ, KO_N=str(c["n"]), KO_K=str(c["k"]), KO_TIME="1", KO_INPUT=path)
        c["cgm_ref_line"] = {}
        for P, want in c["cgm_ref"].items():
            if want == "livelock":  # (recorded as such; not re-run)
                c["cgm_ref_line"][P] = "livelock"
                continue
            val, line = run_cgm_line(os.path.join(REF_DIR, "cgm_param"), int(P), env, 10.0 if "input" not in c else 5.0)
            if val != want:
                raise RuntimeError(f"cgm P={P} gave {val}, recorded {want}: {c}")
            c["cgm_ref_line"][P] = line
        print("lines", c.get("input", c["family"]), c["n"], c["k"], c["cgm_ref_line"], flush=True)
    for f in os.listdir(tmp):
        os.remove(os.path.join(tmp, f))
    os.rmdir(tmp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--shipped", action="store_true")
    ap.add_argument("--large", action="store_true")
    ap.add_argument("--lines", action="store_true")
    args = ap.parse_args()
    if args.lines:
        path = os.path.join(HERE, "expected.json")
        doc = json.load(open(path))
        lines(doc)
        with open(path, "w") as f:
            json.dump(doc, f, indent=1)
        print("wrote", path)
        return
    if not (args.small or args.shipped or args.large):
        args.small = args.shipped = args.large = True
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle")], check=True)
    lib = ctypes.CDLL(os.path.join(REF_DIR, "libvector_ref.so"))
    lib.VecGet.restype = ctypes.c_int
    path = os.path.join(HERE, "expected.json")
    doc = json.load(open(path)) if os.path.exists(path) else {}
    doc["format"] = "tests/golden/make_golden.py v1"
    doc["glibc"] = os.confstr("CS_GNU_LIBC_VERSION")
    if args.small:
        doc["cases"] = small(lib) + livelock_cases(lib)
    if args.shipped:
        doc["shipped"] = shipped()
    if args.large:
        doc["large"] = large(lib)
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()
