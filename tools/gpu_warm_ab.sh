# bench steps/warmup A/B (same binary): 20/3 vs 50/10
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for sw in "20 3" "50 10"; do
  set -- $sw
  timeout -k 10 120 python -u bench.py --steps $1 --warmup $2 --no-cpu-baseline > gpurun_out/ab.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$sw', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms; main', round(d['roofline']['avg_launch_ms'],4), 'ne', round(d['ms_per_step_no_events'],4), d['verified'])"
done
done
