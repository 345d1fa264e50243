"""Per-call durations of the select kernels in a rocprofv3 --kernel-trace CSV,
in call order (the first calls of a process against the rest), and the gaps
between one select's launches: prof_calls.py CSV."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ks = [r for r in rows if "kth::" in r["Kernel_Name"]]
by = {}
for r in ks:
    name = r["Kernel_Name"].split("(")[0].replace("void ", "")
    by.setdefault(name, []).append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000)
for name, v in by.items():
    print(f"{name:24s} n {len(v):3d}: " + " ".join(f"{x:.1f}" for x in v))
# select = k_head, k_main, k_finish: start-to-end and the two launch gaps
sel = []
for i, r in enumerate(ks):
    if "k_head" in r["Kernel_Name"] and i + 2 < len(ks):
        h, m, f = ks[i], ks[i + 1], ks[i + 2]
        t = [int(x[y]) for x in (h, m, f) for y in ("Start_Timestamp", "End_Timestamp")]
        sel.append(((t[5] - t[0]) / 1000, (t[2] - t[1]) / 1000, (t[4] - t[3]) / 1000))
print("select span us: " + " ".join(f"{s:.1f}" for s, _, _ in sel))
print("gap head->main: " + " ".join(f"{g:.1f}" for _, g, _ in sel))
print("gap main->fin : " + " ".join(f"{g:.1f}" for _, _, g in sel))
