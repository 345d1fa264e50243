set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke rc=$?; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
echo "== bench"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench.log 2>&1 || { echo bench rc=$?; tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
if [ -n "$PROF" ]; then
  echo "== rocprof"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/bench_prof.log; exit 1; }
  python3 tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv
fi
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" gpurun_out/pytest.log | tail -60
exit $rc
