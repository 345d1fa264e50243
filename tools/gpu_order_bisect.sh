# which earlier test makes test_dist_world1_nccl read a stale answer (pytest order bisect)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
W=tests/test_gpu_parity.py::test_dist_world1_nccl
for pre in "tests/test_gpu_sharded.py::test_sharded_golden" "tests/test_gpu_sharded.py::test_sharded_errors" "tests/test_cgm_driver.py" "tests/test_gpu_sharded.py::test_dist_backend_slots_match"; do
  timeout -k 10 300 python -u -m pytest $pre $W -x -q --timeout 200 --timeout-method thread -m gpu -p no:randomly > gpurun_out/ob.log 2>&1; rc=$?
  echo "$pre -> rc=$rc $(tail -1 gpurun_out/ob.log)"
  [ $rc -le 1 ] || exit 1
done
