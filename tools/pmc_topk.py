"""HBM traffic of one kth_topk_i32 call from two rocprofv3 --pmc passes
(FETCH_SIZE, WRITE_SIZE), per kernel and summed over the call.

Usage: pmc_topk.py FETCH_csv WRITE_csv LOG2N FAMILY K OUT_JSON

Per MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE / WRITE_SIZE are
KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B per lane)
coalesced streaming read, so the read side of the kernels that stream 16-byte
lanes (k_main, k_topk_count, k_topk_write) is doubled.  The other kernels read
4-byte / 1-byte lanes, for which the guide gives no calibration: their counts
are reported as measured (marked uncalibrated), and writes are taken as
measured throughout.  Per kernel the
values are averaged over its dispatches; a call = one dispatch of each.
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-k-selection_amd"))
import kselect  # noqa: E402  (only for the build id of the library the counters were taken on)


def per_kernel(path, counter):
    acc = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            name = r.get("Kernel_Name", "")
            if "kth::" not in name or "k_fill" in name or r.get("Counter_Name") != counter:
                continue
            short = name.split("(")[0].replace("void ", "")
            d = acc.setdefault(short, {})
            d.setdefault(r.get("Dispatch_Id"), 0.0)
            d[r.get("Dispatch_Id")] += float(r["Counter_Value"])
    return {k: (sum(v.values()) / len(v), len(v)) for k, v in acc.items()}


fetch_csv, write_csv, log2n, family, k, out = sys.argv[1:7]
F, W = per_kernel(fetch_csv, "FETCH_SIZE"), per_kernel(write_csv, "WRITE_SIZE")
kernels = {}
total = 0.0
for name in sorted(set(F) | set(W)):
    fk, nf = F.get(name, (0.0, 0))
    wk, nw = W.get(name, (0.0, 0))
    # 16-byte-per-lane streaming reads (the half-count applies): the select's
    # pass, and the count / write passes' aligned tile loads
    wide = name.startswith(("kth::k_main", "kth::k_topk_write", "kth::k_topk_count"))
    rb = (2.0 if wide else 1.0) * fk * 1024
    wb = wk * 1024
    kernels[name] = {"fetch_size_kib": fk, "write_size_kib": wk, "dispatches": [nf, nw], "read_bytes": rb,
                     "write_bytes": wb, "read_calibrated": wide}
    total += rb + wb
n, kk = 1 << int(log2n), int(k)
algo = 4.0 * n + 12.0 * kk
res = {
    "workload": "kth_topk_i32", "log2n": int(log2n), "family": family, "k": kk, "kernels": kernels,
    "hbm_bytes_per_call": total, "algorithmic_bytes_per_call": algo, "traffic_over_algorithmic": total / algo,
    "build_id": kselect.LIB.kth_build_id().decode(),
    "correction": "k_main / k_topk_count / k_topk_write read = 2 x FETCH_SIZE (gfx950 half-count of 16-B/lane "
                  "streaming reads); other reads as measured (4-B / 1-B lanes: uncalibrated); writes = WRITE_SIZE",
    "note": "algorithmic = 4 B per input key + 12 B per output key; the row-word path (k > n / 16) reads the "
            "input twice by design (select pass + write pass): 8 B per key + 12 B per output",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps({"k": kk, "hbm_GB": total / 1e9, "algo_GB": algo / 1e9, "ratio": total / algo,
                  "per_kernel_GB": {k2: round((v["read_bytes"] + v["write_bytes"]) / 1e9, 4) for k2, v in kernels.items()}}))
