# sharded window as one cooperative launch: sharded / dist / CGM-driver parity, world-1 timing
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_sharded.py tests/test_cgm_driver.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu -k "sharded or dist or cgm or slots" > gpurun_out/dc_parity.log 2>&1; rc=$?
tail -2 gpurun_out/dc_parity.log; [ $rc -eq 0 ] || exit 1
bash tools/gpu_dist1.sh
