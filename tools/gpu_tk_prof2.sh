# rocprof kernel stats of top-k at 2^30, k = 2^20 and 2^29 (final tree)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 1048576 536870912; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tkf_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 6 --warmup 2 > gpurun_out/tkf_$k.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/tkf_$k.log; exit 1; }
  echo "== k=$k"; python3 tools/prof_summary.py gpurun_out/tkf_$k/run_kernel_trace.csv > gpurun_out/tkf_$k.txt; head -11 gpurun_out/tkf_$k.txt
done
