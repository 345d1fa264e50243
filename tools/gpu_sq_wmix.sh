# CU-side (SQ) counters of k_topk_write against the write-mix probe: waves,
# memory instructions in flight, TA FIFO-full cycles.  Two --pmc passes of 8 SQ
# counters per target; per-launch sums averaged over the target's dispatches.
# Usage: gpurun -- bash tools/gpu_sq_wmix.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-sqwmix}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INST_LEVEL_VMEM SQ_LEVEL_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P2="SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_ANY SQ_WAVES"
summ() {  # dir kernel-substring label
python3 - "$1" "$2" "$3" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
per = {}
for r in csv.DictReader(open(f)):
    if sys.argv[2] not in r.get("Kernel_Name", ""):
        continue
    per.setdefault(r["Counter_Name"], {}).setdefault(r.get("Dispatch_Id"), 0.0)
    per[r["Counter_Name"]][r.get("Dispatch_Id")] += float(r["Counter_Value"])
print(sys.argv[3], {c: round(sum(v.values()) / len(v)) for c, v in sorted(per.items())}, "dispatches", len(next(iter(per.values()), {})))
PY
}
for p in 1 2; do
  eval C=\$P$p
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/probe_$p -o run --output-format csv -- ./tools/wmix_probe 30 > $O/probe_$p.log 2>&1 || { echo "probe pmc $p rc=$?"; tail -5 $O/probe_$p.log; exit 1; }
  summ $O/probe_$p "mix_lane<4>" "probe mix_lane<4> pass $p"
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/tk_$p -o run --output-format csv -- python3 bench.py --workload topk --k 134217728 --steps 3 --warmup 1 > $O/tk_$p.log 2>&1 || { echo "topk pmc $p rc=$?"; tail -5 $O/tk_$p.log; exit 1; }
  summ $O/tk_$p "k_topk_write" "k_topk_write k=2^27 pass $p"
  summ $O/tk_$p "k_main<" "k_main<3> k=2^27 pass $p"
done
