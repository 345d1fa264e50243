# SQ instruction mix of the rows kernels (one --pmc pass of 8 SQ counters per
# workload), per 64-key wave slot: counter per launch / (rows * cols / 64)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/sq; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES"
i=0
for args in "--rows-dtype i32" "--rows-dtype f32" "--rows-dtype i32 --topk" "--rows-dtype f32 --topk"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/w$i -o run --output-format csv -- python3 bench.py --workload rows $args --k 64 --steps 3 --warmup 1 > $O/w$i.log 2>&1 || { echo "pmc $args rc=$?"; tail -20 $O/w$i.log; exit 1; }
  python3 - "$O/w$i" "$args" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
per = {}
for r in csv.DictReader(open(f)):
    if "k_rows_reg" not in r.get("Kernel_Name", ""):
        continue
    per.setdefault(r["Counter_Name"], {}).setdefault(r.get("Dispatch_Id"), 0.0)
    per[r["Counter_Name"]][r.get("Dispatch_Id")] += float(r["Counter_Value"])
slots = 65536 * 4096 / 64
out = {c: round(sum(v.values()) / len(v) / slots, 2) for c, v in sorted(per.items())}
print(sys.argv[2], out)
PY
done
