set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== smoke" 
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo smoke rc=$?; tail -30 gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
echo "== bench"
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --cpu-log2n 22 > gpurun_out/bench.log 2>&1 || { echo bench rc=$?; tail -30 gpurun_out/bench.log; exit 1; }
cat gpurun_out/bench.log
echo "== pytest"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread -m gpu -k "not golden and not shipped" > gpurun_out/pytest.log 2>&1; rc=$?
tail -40 gpurun_out/pytest.log
exit $rc
