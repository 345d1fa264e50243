# round-2 evidence run: smoke, full GPU suite, default bench (with CPU baselines), rocprof, PMC traffic, rows
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke rc=$?; tail -30 gpurun_out/smoke.log; exit 1; }
tail -4 gpurun_out/smoke.log
echo "== pytest"
timeout -k 10 900 python -u -m pytest tests/ -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/pytest.log 2>&1; rc=$?
grep -E "passed|failed" gpurun_out/pytest.log | tail -1; [ $rc -eq 0 ] || exit $rc
echo "== bench (default, with CPU baselines)"
timeout -k 10 600 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { echo bench rc=$?; tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-600
echo "== rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/bench_prof.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv
echo "== pmc"
bash tools/gpu_pmc.sh || exit 1
cat gpurun_out/pmc_traffic.json | head -30
echo "== rows"
bash tools/gpu_rows_bench.sh || exit 1
