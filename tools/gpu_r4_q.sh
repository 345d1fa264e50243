# Round 4 (q): k_tk5_write's coalesced chunk walk for dense windows
# (KTH_TK5W_CHUNKED=1, default) against the per-lane walk (=0): top-k parity
# with both, then k_tk5_write's time at k = 2^24 / 2^25 / 2^26
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4q; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
for o in 1 0; do
  echo "== top-k tests KTH_TK5W_CHUNKED=$o"
  KTH_TK5W_CHUNKED=$o timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_topk.py > $O/topk_tests_$o.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error" $O/topk_tests_$o.log | head -30; tail -5 $O/topk_tests_$o.log; exit 1; }
  tail -1 $O/topk_tests_$o.log
done
for k in 16777216 33554432 67108864; do
  for o in 1 0; do
    KTH_TK5W_CHUNKED=$o timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_${o}_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 5 --warmup 2 --no-cpu-baseline > $O/p_${o}_$k.log 2>&1 || { echo prof rc=$?; tail -20 $O/p_${o}_$k.log; exit 1; }
    echo "k=$k chunked=$o"; python3 tools/prof_summary.py $O/p_${o}_$k/run_kernel_trace.csv 0 | grep -E "tk5_write"
  done
done
echo done
