# Round 4: the whole -m gpu suite on the final build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4suite; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
