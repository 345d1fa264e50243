# rows parity tests (k-th and top-k per row) + the rows benchmark sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "rows" > gpurun_out/rows_tests.log 2>&1 || { echo tests rc=$?; tail -30 gpurun_out/rows_tests.log; exit 1; }
tail -1 gpurun_out/rows_tests.log
bash tools/gpu_rows_bench.sh
