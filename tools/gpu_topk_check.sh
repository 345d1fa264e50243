# single-array top-k: GPU parity tests, then the 2^30 bench sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/tk; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_topk.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { echo tests rc=$?; tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for k in ${TK_KS:-1024 1048576 16777216 33554432 536870912}; do
  timeout -k 10 120 python -u bench.py --workload topk --k $k --steps 10 --warmup 3 --no-cpu-baseline >> $O/topk.jsonl 2>$O/topk.err || { echo topk rc=$?; tail -20 $O/topk.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/topk.jsonl'):
    d=json.loads(l); print('topk k', d['config']['k'], round(d['ms_per_step'],3), 'ms', d.get('verified'))"
