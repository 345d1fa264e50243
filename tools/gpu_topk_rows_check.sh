# Top-k and rows after a kernel change: their GPU tests, the top-k whole-call
# times and kernel averages (gpu_topk_ab.sh, base library), and the rows
# lines (uniform and duplicate-heavy, k = 64 and k = n/2).
# Usage: gpurun -- bash tools/gpu_topk_rows_check.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-tkrows}; O=gpurun_out/$T; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_topk.py tests/test_gpu_parity.py -k "topk or rows" -m gpu -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error" $O/tests.log | head -20; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for args in "--rows-dtype i32" "--rows-dtype f32" "--rows-dtype i32 --rows-input dup" "--rows-dtype f32 --rows-input dup" "--rows-dtype f32 --rows-input dup --k 2048" "--rows-dtype i32 --rows-input dup --k 2048"; do
  timeout -k 10 120 python -u bench.py --workload rows --k 64 $args --steps 20 --warmup 3 --no-cpu-baseline >> $O/rows.jsonl 2>$O/rows.err || { echo "rows $args rc=$?"; tail -20 $O/rows.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/rows.jsonl'):
    d=json.loads(l); c=d['config']; r=d['roofline']
    print(c['workload'], round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us', d['verified'])"
KS="67108864 134217728 536870912" bash tools/gpu_topk_ab.sh $T/topk
