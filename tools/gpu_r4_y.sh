# Round 4 (y): top-k per row on config 5's duplicate-heavy rows (k = 64),
# the workload the few-valued path hands to the general compaction
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4y; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
for dt in i32 f32; do
  timeout -k 10 120 python -u bench.py --workload rows --rows-dtype $dt --rows-input dup --topk --k 64 --steps 20 --warmup 3 --no-cpu-baseline >> $O/rows.jsonl 2>$O/rows.err || { echo "rc=$?"; tail -20 $O/rows.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/rows.jsonl'):
    d=json.loads(l); r=d['roofline']; print(d['config']['workload'], round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us', d['verified'])"
echo done
