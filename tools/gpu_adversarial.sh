# BASELINE config 4: adversarial inputs at 2^30 (all-equal, few-distinct,
# sorted / reverse-sorted; uniform for reference), k in {1, n/2, n}: the
# default select bench per case (verified by the on-device rank certificate)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/adv; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
N=$((1 << 30))
for fam in uniform_half all_equal few_distinct sorted_asc sorted_desc; do
  for k in 1 $((N / 2)) $N; do
    timeout -k 10 120 python -u bench.py --family $fam --k $k --steps 20 --warmup 5 --no-cpu-baseline >> $O/adv.jsonl 2>$O/err.log || { echo "$fam k=$k rc=$?"; tail -20 $O/err.log; exit 1; }
  done
done
python3 -c "
import json
for l in open('$O/adv.jsonl'):
    d=json.loads(l); c=d['config']
    print(c.get('family', '?'), 'k', c.get('k'), round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms', 'path', d.get('path'), 'cands', d.get('candidates'), d['verified'])"
