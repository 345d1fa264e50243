# bench sweep over env settings: SWEEP="VAR=val,VAR2=val ..." (space-separated configs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in $SWEEP; do
  env $(echo "$cfg" | tr ',' ' ') timeout -k 10 120 python -u bench.py --steps 30 --warmup 3 --no-cpu-baseline > gpurun_out/sw.log 2>&1 || { echo bench $cfg rc=$?; tail -20 gpurun_out/sw.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/sw.log').read().strip().splitlines()[-1]); print('$cfg', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms main', round(d['roofline']['avg_launch_ms'],4), 'total', round(d['whole_select_ms_events'],4), d['verified'], d.get('path'))"
done
