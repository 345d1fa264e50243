"""Summarise a rocprofv3 --kernel-trace CSV: per-kernel averages and the kernel
timeline of the last selection (or top-k call): prof_summary.py CSV [kernels in the timeline, default 8]."""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
agg = defaultdict(list)
for r in rows:
    agg[r["Kernel_Name"].split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    if "kth::" in k:
        print(f"{k:40s} calls {len(v):4d} avg {sum(v) / len(v):9.1f} us  min {min(v):9.1f}")
ks = [r for r in rows if "kth::" in r["Kernel_Name"]]
starts = [i for i, r in enumerate(ks) if "k_gather" in r["Kernel_Name"] or "k_head" in r["Kernel_Name"]]
ntl = int(sys.argv[2]) if len(sys.argv) > 2 else 8
if starts and ntl > 0:
    seq = ks[starts[-1]:starts[-1] + ntl]
    t0 = int(seq[0]["Start_Timestamp"])
    for r in seq:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        print(f"  {r['Kernel_Name'].split('(')[0]:28s} {(e - s) / 1000:8.1f} us  +{(s - t0) / 1000:8.1f} -> +{(e - t0) / 1000:8.1f}"
              f"  grid {r['Grid_Size_X']} vgpr {r['VGPR_Count']} sgpr {r['SGPR_Count']} lds {r['LDS_Block_Size']}")
