"""HBM traffic of the dominant kernel from two rocprofv3 --pmc passes.

Usage: pmc_traffic.py FETCH_csv WRITE_csv KERNEL_SUBSTR LOG2N FAMILY OUT_JSON [OUT_BYTES]

The algorithmic bytes are the 4-byte keys (2^LOG2N of them) read plus
OUT_BYTES written (default 0; e.g. 8 * rows * k for top-k rows).

Per MI355X_MICROARCH.md (HBM / rocprofv3 section): FETCH_SIZE and WRITE_SIZE
are in KiB; on gfx950 FETCH_SIZE reports half the bytes of a wide (16 B per
lane) coalesced streaming read, so the read side is doubled.  Values are
averaged over the kernel's dispatches and reported per launch.
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpi-k-selection_amd"))
import kselect  # noqa: E402  (only for the build id of the library the counters were taken on)


def per_dispatch(path, kernel, counter):
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if kernel in r.get("Kernel_Name", "") and r.get("Counter_Name") == counter:
                vals.setdefault(r.get("Dispatch_Id", len(vals)), 0.0)
                vals[r.get("Dispatch_Id", len(vals))] += float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {counter} rows for {kernel} in {path}")
    return sum(vals.values()) / len(vals), len(vals)


fetch_csv, write_csv, kernel, log2n, family, out = sys.argv[1:7]
out_bytes = float(sys.argv[7]) if len(sys.argv) > 7 else 0.0
fetch_kib, nf = per_dispatch(fetch_csv, kernel, "FETCH_SIZE")
write_kib, nw = per_dispatch(write_csv, kernel, "WRITE_SIZE")
read_bytes = 2.0 * fetch_kib * 1024  # gfx950 FETCH_SIZE = 1/2 of 16-B-per-lane streaming reads
write_bytes = write_kib * 1024
algo = 4.0 * (1 << int(log2n)) + out_bytes
res = {
    "kernel": kernel,
    "log2n": int(log2n),
    "family": family,
    "fetch_size_kib_per_launch": fetch_kib,
    "write_size_kib_per_launch": write_kib,
    "dispatches": [nf, nw],
    "read_bytes_per_launch": read_bytes,
    "write_bytes_per_launch": write_bytes,
    "hbm_bytes_per_launch": read_bytes + write_bytes,
    "algorithmic_bytes_per_launch": algo,
    "traffic_over_algorithmic": (read_bytes + write_bytes) / algo,
    "build_id": kselect.LIB.kth_build_id().decode(),
    "correction": "read = 2 x FETCH_SIZE (gfx950 half-count of 16-B/lane streaming reads), write = WRITE_SIZE",
}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
