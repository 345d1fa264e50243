# rows kernel SQ counters (one --pmc pass per config): VALU/LDS instruction mix, LDS conflicts, stalls
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU"
for lib in ${LIBS:-default}; do for dt in ${DTS:-i32 f32}; do
  if [ "$lib" = default ]; then L=""; else L="$PWD/mpi-k-selection_amd/lib/variants/libkth_$lib.so"; fi
  rm -rf gpurun_out/rpmc_${lib}_$dt
  KTH_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $C -d gpurun_out/rpmc_${lib}_$dt -o run --output-format csv -- python3 bench.py --workload rows --rows-dtype $dt --k 64 --steps 3 --warmup 1 > gpurun_out/rpmc.log 2>&1 || { echo pmc rc=$?; tail -20 gpurun_out/rpmc.log; exit 1; }
  F=$(find gpurun_out/rpmc_${lib}_$dt -name "*counter_collection.csv" | head -1)
  python3 - "$F" "$lib $dt" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    if "rows_reg" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(sys.argv[2], {k: f"{sum(v)/len(v):.4g}" for k, v in sorted(acc.items())})
PY
done; done
