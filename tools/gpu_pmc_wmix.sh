# L2 <-> fabric request counters (TCC_EA0_*) of k_topk_write against the write-
# mix probe's mix_lane kernel (tools/wmix_probe.hip): where the write pass loses
# its ~25 % against a probe of the same byte mix.  Three --pmc passes of 4 TCC
# counters per target; per launch sums, averaged over the target's dispatches.
# Usage: [K="134217728 536870912"] gpurun -- bash tools/gpu_pmc_wmix.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-pmcwmix}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
P1="TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"
P2="TCC_EA0_WRREQ_STALL_sum TCC_TAG_STALL_sum TCC_TOO_MANY_EA_WRREQS_STALL_sum TCC_EA0_WRREQ_DRAM_CREDIT_STALL_sum"
P3="TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TCC_BUSY_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum"
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
for p in 1 2 3; do
  eval C=\$P$p
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/probe_$p -o run --output-format csv -- ./tools/wmix_probe 30 > $O/probe_$p.log 2>&1 || { echo "probe pmc $p rc=$?"; tail -5 $O/probe_$p.log; exit 1; }
  summ $O/probe_$p "mix_lane<4>" "probe mix_lane<4> pass $p"
  summ $O/probe_$p "copy<8>" "probe copy<8> pass $p"
  for k in ${K:-134217728 536870912}; do
    timeout -s KILL 120 rocprofv3 --pmc $C -d $O/tk${k}_$p -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 3 --warmup 1 > $O/tk${k}_$p.log 2>&1 || { echo "topk pmc $k $p rc=$?"; tail -5 $O/tk${k}_$p.log; exit 1; }
    summ $O/tk${k}_$p "k_topk_write" "k_topk_write k=$k pass $p"
    summ $O/tk${k}_$p "k_main<" "k_main k=$k pass $p"
  done
done
