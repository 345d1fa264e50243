# kernel times of top-k at 2^30 for k = 2^20 (k_main<3>) and k = 1024 (k_main<1>)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for k in 1048576 1024; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tkp_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 8 --warmup 2 > gpurun_out/tkp_$k.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/tkp_$k.log; exit 1; }
  echo "== k=$k"; python3 tools/prof_summary.py gpurun_out/tkp_$k/run_kernel_trace.csv | head -12
done
