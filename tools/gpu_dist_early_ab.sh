# A/B of kth_dist_result_early on the one-rank RCCL protocol (bench.py --dist), interleaved.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r5early; mkdir -p $O; export TMPDIR=/tmp
for i in 1 2 3; do
  for e in 1 0; do
    KTH_DIST_EARLY=$e timeout -k 10 200 python -u bench.py --dist --steps 20 --warmup 5 --no-cpu-baseline >> $O/dist_$e.jsonl 2>>$O/dist_$e.err || { echo "dist $e rc=$?"; tail -20 $O/dist_$e.err; exit 1; }
  done
done
for e in 1 0; do python3 -c "
import json
v=[json.loads(l) for l in open('$O/dist_$e.jsonl') if l.startswith('{')]
print('early=$e', ' '.join('%.4f' % d['ms_per_step'] for d in v), 'ms', ' '.join('%.1f' % d['value'] for d in v), 'verified', all(d['verified'] for d in v))"; done
