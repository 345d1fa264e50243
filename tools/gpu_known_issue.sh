# the sharded-handle -> world-1 DistSelector order that read stale answers, and the default order
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
W=tests/test_gpu_parity.py::test_dist_world1_nccl
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py::test_sharded_golden $W -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/ki.log 2>&1; echo "sharded->world1 rc=$? $(tail -1 gpurun_out/ki.log)"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_sharded.py tests/test_cgm_driver.py -x -q --timeout 200 --timeout-method thread -m gpu -k "sharded or dist or cgm or slots" > gpurun_out/ki2.log 2>&1; echo "subset rc=$? $(tail -1 gpurun_out/ki2.log)"
MASTER_ADDR=127.0.0.1 MASTER_PORT=29536 timeout -k 10 180 python -u bench.py --dist --no-cpu-baseline 2>&1 | tail -1 | cut -c1-200
