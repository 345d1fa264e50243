# Round 4 (d): the select's slowdown a few selects after an idle start --
# device (power: random vs constant data, VALU work per key) or ours
# (cooperative kernels, candidates)?
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4d; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 90 ./tools/stream_probe 30 bump > $O/bump.txt 2>&1 || { echo bump rc=$?; tail -5 $O/bump.txt; exit 1; }
cut -c1-330 $O/bump.txt
for fam in uniform_half all_equal; do
  timeout -k 10 120 python -u tools/bump_probe.py $fam >> $O/sel.jsonl 2>> $O/sel.err || { echo sel rc=$?; tail -5 $O/sel.err; exit 1; }
done
KTH_COOP=0 timeout -k 10 120 python -u tools/bump_probe.py uniform_half >> $O/sel.jsonl 2>> $O/sel.err || { echo sel rc=$?; tail -5 $O/sel.err; exit 1; }
python3 -c "
import json
for l in open('$O/sel.jsonl'):
    d=json.loads(l); print(d['phase'], 'first10', d['first10'], 'last20', d['last20'], ' '.join(str(round(x,3)) for x in d['ms'][:20]))"
echo done
