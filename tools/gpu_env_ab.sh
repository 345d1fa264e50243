# A/B of environment tunables on the default select bench (one process per
# setting, same box): SETTINGS="KTH_WINDOW_Z=4 KTH_WINDOW_Z=3.5" (base = none)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/envab; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
i=0
for s in base $SETTINGS base; do
  e=""; [ $s = base ] || e=$s
  i=$((i+1)); f=$O/run$i.log
  env $e timeout -k 10 200 python3 -u bench.py --no-cpu-baseline ${ARGS:-} > $f 2>&1 || { echo "$s rc=$?"; tail -20 $f; exit 1; }
  python3 -c "
import json; d=json.loads(open('$f').read().strip().splitlines()[-1])
print('${s##*/}', round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'ev', round(d.get('ms_per_step_events') or 0,4), 'k_main', round(d['roofline']['avg_launch_ms'],4), 'cands', d.get('candidates'), d['verified'])"
done
