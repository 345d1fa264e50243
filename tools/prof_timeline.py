"""The last kernels of a rocprofv3 --kernel-trace CSV as a timeline: start
offset from the first of them, duration, and the idle gap before each (us).
Usage: prof_timeline.py run_kernel_trace.csv [count=40]"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
count = int(sys.argv[2]) if len(sys.argv) > 2 else 40
rows = rows[-count:]
t0 = int(rows[0]["Start_Timestamp"])
prev_end = None
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")[:48]
    gap = "" if prev_end is None else f"{(s - prev_end) / 1000:8.1f}"
    print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f} gap {gap:>8s}  {name}")
    prev_end = e if prev_end is None else max(prev_end, e)
