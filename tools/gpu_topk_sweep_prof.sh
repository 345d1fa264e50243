# rocprof kernel averages of one top-k call per k (2^30 int32 keys), the
# final build's per-kernel breakdown.  Usage: gpurun -- bash tools/gpu_topk_sweep_prof.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-tksweep}; O=gpurun_out/$T; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
for k in 1024 1048576 16777216 67108864 134217728 536870912; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/p$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 7 --warmup 2 --no-cpu-baseline > $O/p$k.log 2>&1 || { echo "prof k=$k rc=$?"; tail -5 $O/p$k.log; exit 1; }
  echo "k=$k" >> $O/summary.txt
  python3 tools/prof_summary.py $O/p$k/run_kernel_trace.csv 0 | grep -v k_fill >> $O/summary.txt
done
cat $O/summary.txt
