# rows kernel SQ counters: stall breakdown + instruction mix (one --pmc pass per workload)
# WL: comma-joined bench args per workload, space-separated workloads
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
C="${C:-SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM}"
i=0
for args in ${WL:-"--rows-dtype=i32 --rows-dtype=i32,--topk"}; do
  i=$((i+1)); rm -rf gpurun_out/rpmc_$i
  timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/rpmc_$i -o run --output-format csv -- python3 bench.py --workload rows ${args//,/ } --k 64 --steps 3 --warmup 1 > gpurun_out/rpmc.log 2>&1 || { echo pmc rc=$?; tail -20 gpurun_out/rpmc.log; exit 1; }
  F=$(find gpurun_out/rpmc_$i -name "*counter_collection.csv" | head -1)
  python3 - "$F" "$args" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    if "rows_reg" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
slots = (1 << 28) / 64
print(sys.argv[2], {k: f"{sum(v)/len(v):.4g} ({sum(v)/len(v)/slots:.2f}/slot)" for k, v in sorted(acc.items())})
PY
done
