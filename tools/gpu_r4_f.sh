# Round 4 (f): staged top-k after the latency-bound flush rewrite: parity, then
# the 2^30 sweep with per-kernel times.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4f; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
echo "== top-k tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_topk.py > $O/topk_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error" $O/topk_tests.log | head -30; tail -5 $O/topk_tests.log; exit 1; }
tail -1 $O/topk_tests.log
echo "== top-k sweep"
for k in 1024 1048576 16777216 67108864 134217728 536870912; do
  timeout -k 10 120 python -u bench.py --workload topk --k $k --steps 10 --warmup 3 --no-cpu-baseline >> $O/topk.jsonl 2>$O/topk.err || { echo topk rc=$?; tail -20 $O/topk.err; exit 1; }
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 5 --warmup 2 --no-cpu-baseline > $O/prof_$k.log 2>&1 || { echo prof rc=$?; tail -20 $O/prof_$k.log; exit 1; }
  echo "k=$k"; python3 tools/prof_summary.py $O/prof_$k/run_kernel_trace.csv 0 | grep -v k_fill | head -8
done
python3 -c "
import json
for l in open('$O/topk.jsonl'):
    d=json.loads(l); print('topk k', d['config']['k'], round(d['ms_per_step'],3), 'ms', round(d['value'],1), 'Gkeys/s', d.get('verified'))"
echo done
