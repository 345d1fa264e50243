# Round-3 state on one MI355X: GPU tests (both orders of the sharded / world-1
# dist tests), smoke, default select bench, single-array top-k sweep, rows sweep.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r3; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests rc=$?; tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_sharded.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "sharded or dist" > $O/gpu_tests_rev.log 2>&1 || { echo rev rc=$?; tail -30 $O/gpu_tests_rev.log; exit 1; }
tail -1 $O/gpu_tests_rev.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke rc=$?; tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo bench rc=$?; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-400
for k in 1024 1048576 16777216 536870912; do
  timeout -k 10 120 python -u bench.py --workload topk --k $k --steps 10 --warmup 3 --no-cpu-baseline >> $O/topk.jsonl 2>$O/topk.err || { echo topk rc=$?; tail -20 $O/topk.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/topk.jsonl'):
    d=json.loads(l); print('topk k', d['config']['k'], round(d['ms_per_step'],3), 'ms', d.get('verified'))"
bash tools/gpu_rows_bench.sh
echo done
