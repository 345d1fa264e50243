"""SQ instruction mix of one kernel from a rocprofv3 --pmc counter CSV, per
64-key wave slot (counter per launch / (keys / 64)): sq_mix.py CSV KERNEL_SUBSTR KEYS LABEL."""
import csv
import glob
import sys

path, kern, keys, label = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
f = path if path.endswith(".csv") else glob.glob(path + "/**/*counter_collection.csv", recursive=True)[0]
per = {}
for r in csv.DictReader(open(f)):
    if kern not in r.get("Kernel_Name", ""):
        continue
    per.setdefault(r["Counter_Name"], {}).setdefault(r.get("Dispatch_Id"), 0.0)
    per[r["Counter_Name"]][r.get("Dispatch_Id")] += float(r["Counter_Value"])
slots = keys / 64
print(label, {c: round(sum(v.values()) / len(v) / slots, 3) for c, v in sorted(per.items())})
