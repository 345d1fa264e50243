# top-k of one array: GPU parity tests, bench at 2^30 for several k, rocprof stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/topk_pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error|assert" gpurun_out/topk_pytest.log | tail -40
[ $rc -eq 0 ] || exit $rc
for k in 64 1024 1048576 536870912; do
  timeout -k 10 120 python -u bench.py --workload topk --k $k --steps 10 --warmup 2 > gpurun_out/topk_$k.log 2>&1 || { echo bench k=$k rc=$?; tail -20 gpurun_out/topk_$k.log; exit 1; }
  tail -1 gpurun_out/topk_$k.log | cut -c1-200; grep -o '"avg_launch_ms": [0-9.]*\|"verified": [a-z]*' gpurun_out/topk_$k.log
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_topk -o run --output-format csv -- python3 bench.py --workload topk --k 1024 --steps 10 --warmup 2 > gpurun_out/prof_topk.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/prof_topk.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof_topk/run_kernel_trace.csv | head -20
