# The whole GPU test suite, smoke(), and the single-array top-k sweep at 2^30
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/suite; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke rc=$?; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
for k in 1024 16385 1048576 16777216 33554432 67108864 536870912; do
  timeout -k 10 120 python -u bench.py --workload topk --k $k --steps 10 --warmup 3 --no-cpu-baseline >> $O/topk.jsonl 2>$O/topk.err || { echo topk rc=$?; tail -20 $O/topk.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/topk.jsonl'):
    d=json.loads(l); print('topk k', d['config']['k'], round(d['ms_per_step'],3), 'ms', round(d['value'],1), 'Gkeys/s', d.get('verified'))"
