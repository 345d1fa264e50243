# early-window slack A/B (runtime knob KTH_HEAD_SLACK)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for sl in 1.5 1.25 2.0; do
  KTH_HEAD_SLACK=$sl timeout -k 10 120 python -u bench.py --no-cpu-baseline > gpurun_out/ab.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); print('$sl', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms; main', round(d['roofline']['avg_launch_ms'],4), 'ne', round(d['ms_per_step_no_events'],4), 'cand', d.get('candidates'), d['verified'])"
done
done
