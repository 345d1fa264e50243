# A/B of the select bench over values of one env knob: VAR=name VALS="a b c"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for v in $VALS; do
  env $VAR=$v timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/ab.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$VAR=$v', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms; main', round(r['avg_launch_ms'],4), 'frac', round(r['frac'],4), 'whole', d.get('whole_select_ms_events'), d['verified'])"
done
done
