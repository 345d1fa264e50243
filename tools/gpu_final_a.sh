# Evidence (a): the whole GPU suite, smoke(), the default bench line
# (the driver's N=1 command, with CPU baselines) and its rocprof kernel stats.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/fa; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
echo "== pytest -m gpu"
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 180 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
echo "== smoke"
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke rc=$?; tail -20 $O/smoke.log; exit 1; }
tail -3 $O/smoke.log
echo "== bench (driver command)"
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1 || { echo bench rc=$?; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log | cut -c1-700
echo "== rocprof (driver command, no CPU baselines)"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof rc=$?; tail -20 $O/prof.log; exit 1; }
python3 tools/prof_summary.py $O/prof/run_kernel_trace.csv > $O/select_summary.txt; head -8 $O/select_summary.txt
python3 tools/prof_calls.py $O/prof/run_kernel_trace.csv > $O/select_calls.txt; tail -3 $O/select_calls.txt | cut -c1-300
echo "== top-k sweep"
for k in 1024 1048576 16777216 67108864 134217728 536870912; do
  timeout -k 10 120 python -u bench.py --workload topk --k $k --steps 10 --warmup 3 --no-cpu-baseline >> $O/topk.jsonl 2>$O/topk.err || { echo topk rc=$?; tail -20 $O/topk.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/topk.jsonl'):
    d=json.loads(l); print('topk k', d['config']['k'], round(d['ms_per_step'],3), 'ms', round(d['value'],1), 'Gkeys/s', d.get('verified'))"
echo "== config 4 (adversarial families at 2^30)"
N=$((1 << 30))
for fam in uniform_half all_equal few_distinct sorted_asc sorted_desc; do
  for k in 1 $((N / 2)) $N; do
    timeout -k 10 120 python -u bench.py --family $fam --k $k --steps 20 --warmup 5 --no-cpu-baseline >> $O/adv.jsonl 2>$O/adv.err || { echo "$fam k=$k rc=$?"; tail -20 $O/adv.err; exit 1; }
  done
done
python3 -c "
import json
for l in open('$O/adv.jsonl'):
    d=json.loads(l); c=d['config']
    print(c.get('family', '?'), 'k', c.get('k'), round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms', 'path', d.get('path'), 'cands', d.get('candidates'), d['verified'])"
echo "== rows (BASELINE config 5: uniform and duplicate-heavy, k-th and top-k)"
for args in "--rows-dtype i32" "--rows-dtype f32" "--rows-dtype i32 --topk" "--rows-dtype f32 --topk" "--rows-dtype i32 --rows-input dup" "--rows-dtype f32 --rows-input dup" "--rows-dtype f32 --rows-input dup --k 2048"; do
  timeout -k 10 120 python -u bench.py --workload rows --k 64 $args --steps 20 --warmup 3 >> $O/rows.jsonl 2>$O/rows.err || { echo "rows $args rc=$?"; tail -20 $O/rows.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/rows.jsonl'):
    d=json.loads(l); c=d['config']; r=d['roofline']
    print(c['workload'], round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us frac', round(r['frac'],3), 'traffic', r['traffic'], d['verified'])"
echo done
