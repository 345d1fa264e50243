# Round 4: rows parity (incl. the few-valued / zero-bin cases) on the final build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4tests; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "rows" > $O/rows_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error|assert" $O/rows_tests.log | head -40; tail -5 $O/rows_tests.log; exit 1; }
grep -E "few_valued|passed" $O/rows_tests.log
