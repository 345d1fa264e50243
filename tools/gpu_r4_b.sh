# Round 4 (b): the warmup bump (ours or the device's?), per-kernel times of
# the 2^33 one-array select (k = 1 against k = n/2), and BASELINE config 5's
# duplicate-heavy rows variant.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4b; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
echo "== bump probe"
timeout -k 10 240 python -u tools/bump_probe.py > $O/bump.jsonl 2> $O/bump.err || { echo bump rc=$?; tail -20 $O/bump.err; exit 1; }
python3 -c "
import json
for l in open('$O/bump.jsonl'):
    d=json.loads(l); print(d['phase'], 'first10', d['first10'], 'last20', d['last20'], ' '.join(str(round(x,3)) for x in d['ms'][:16]))"
echo "== 2^33 kernels"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/p33 -o run --output-format csv -- python3 tools/probe_2e33.py 33 uniform_half 3 > $O/p33.log 2>&1 || { echo p33 rc=$?; tail -20 $O/p33.log; exit 1; }
python3 tools/prof_calls.py $O/p33/run_kernel_trace.csv | cut -c1-300
echo "== rows duplicate-heavy"
for dt in i32 f32; do
  for inp in uniform dup; do
    for k in 1 64 2048 4096; do
      timeout -k 10 120 python -u bench.py --workload rows --rows-dtype $dt --rows-input $inp --k $k --steps 20 --warmup 5 >> $O/rows.jsonl 2>>$O/rows.err || { echo rows rc=$?; tail -20 $O/rows.err; exit 1; }
    done
  done
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_rows_dup_$dt -o run --output-format csv -- python3 bench.py --workload rows --rows-dtype $dt --rows-input dup --k 64 --steps 10 --warmup 2 > $O/prof_rows_dup_$dt.log 2>&1 || { echo prof rc=$?; tail -20 $O/prof_rows_dup_$dt.log; exit 1; }
done
python3 -c "
import json
for l in open('$O/rows.jsonl'):
    d=json.loads(l); c=d['config']; print(d['dtype'], c['input'], 'k', c['k'], round(d['value'],1), 'Gkeys/s', round(d['roofline']['avg_launch_ms']*1e3,1), 'us', d['verified'])"
echo done
