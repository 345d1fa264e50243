# run a subset of the GPU tests (PYTEST_ARGS) in one process, with a time limit
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu $PYTEST_ARGS ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_new.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed|Error" gpurun_out/pytest_new.log | tail -40
exit $rc
