# Round 4 (i): k_tk5_write's wave-row-parallel placement (OWNER) against the
# per-lane walk, by KTH_TK5_OWNER: top-k parity with both, then the sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4i; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
for o in 1 0; do
  echo "== top-k tests KTH_TK5_OWNER=$o"
  KTH_TK5_OWNER=$o timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_topk.py > $O/topk_tests_$o.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error" $O/topk_tests_$o.log | head -30; tail -5 $O/topk_tests_$o.log; exit 1; }
  tail -1 $O/topk_tests_$o.log
done
for k in 1048576 16777216 67108864; do
  for o in 1 0; do
    KTH_TK5_OWNER=$o timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_${o}_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 5 --warmup 2 --no-cpu-baseline > $O/p_${o}_$k.log 2>&1 || { echo prof rc=$?; tail -20 $O/p_${o}_$k.log; exit 1; }
    echo "k=$k owner=$o"; python3 tools/prof_summary.py $O/p_${o}_$k/run_kernel_trace.csv 0 | grep -E "tk5_write"
  done
done
echo done
