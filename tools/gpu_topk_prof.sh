# rocprof kernel stats + last-call timeline of the single-array top-k at 2^30
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/tkprof; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
for k in ${TK_KS:-1048576 16777216}; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/k$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 5 --warmup 2 --no-cpu-baseline > $O/k$k.log 2>&1 || { echo prof rc=$?; tail -20 $O/k$k.log; exit 1; }
  echo "== k=$k $(tail -1 $O/k$k.log | cut -c1-0)"
  python3 tools/prof_summary.py $(find $O/k$k -name "*kernel_trace.csv" | head -1) 12
done
