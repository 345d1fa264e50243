# rows parity + rows benches after the one-row-per-wave / staging change, then select phase stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rows" > gpurun_out/rows_parity.log 2>&1; rc=$?
tail -3 gpurun_out/rows_parity.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_rows_bench.sh || exit 1
bash tools/gpu_stamps.sh || exit 1
