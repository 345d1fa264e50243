# Round 4 (e): the warmup bump (device or ours?), the dense-bin rows path
# (parity + config 5's duplicate-heavy variant), staged top-k entry batching A/B.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4e; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
echo "== bump"
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
echo "== rows tests"
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "rows" > $O/rows_tests.log 2>&1 || { echo rows tests rc=$?; grep -E "FAIL|Error|error" $O/rows_tests.log | head -30; tail -5 $O/rows_tests.log; exit 1; }
tail -1 $O/rows_tests.log
echo "== rows bench"
for dt in i32 f32; do
  for inp in uniform dup; do
    for k in 1 64 2048 4096; do
      timeout -k 10 120 python -u bench.py --workload rows --rows-dtype $dt --rows-input $inp --k $k --steps 20 --warmup 5 >> $O/rows.jsonl 2>>$O/rows.err || { echo rows rc=$?; tail -20 $O/rows.err; exit 1; }
    done
  done
  timeout -k 10 120 python -u bench.py --workload rows --rows-dtype $dt --topk --k 64 --steps 20 --warmup 5 >> $O/rows.jsonl 2>>$O/rows.err || { echo rows rc=$?; tail -20 $O/rows.err; exit 1; }
  timeout -k 10 120 python -u bench.py --workload rows --rows-dtype $dt --rows-input dup --topk --k 64 --steps 20 --warmup 5 >> $O/rows.jsonl 2>>$O/rows.err || { echo rows rc=$?; tail -20 $O/rows.err; exit 1; }
done
python3 -c "
import json
for l in open('$O/rows.jsonl'):
    d=json.loads(l); c=d['config']; print(d['dtype'], c['input'], 'topk' if 'top-k' in c['workload'] else 'kth', 'k', c['k'], round(d['value'],1), 'Gkeys/s', round(d['roofline']['avg_launch_ms']*1e3,1), 'us', d['verified'])"
echo "== top-k tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_topk.py > $O/topk_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error" $O/topk_tests.log | head -30; tail -5 $O/topk_tests.log; exit 1; }
tail -1 $O/topk_tests.log
echo "== tk5 A/B"
for k in 1048576 16777216 67108864; do
  for v in base r3flush tk5b4 tk5chunk; do
    lib=mpi-k-selection_amd/lib/variants/libkth_$v.so; [ $v = base ] && lib=mpi-k-selection_amd/lib/libkth.so
    KTH_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/tk_${v}_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 5 --warmup 2 --no-cpu-baseline > $O/tk_${v}_$k.log 2>&1 || { echo "$v rc=$?"; tail -20 $O/tk_${v}_$k.log; exit 1; }
    echo "k=$k $v: $(tail -1 $O/tk_${v}_$k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["ms_per_step"],3), "ms", d["verified"])')"
    python3 tools/prof_summary.py $(find $O/tk_${v}_$k -name "*kernel_trace.csv" | head -1) 0 | grep -E "tk5|k_main"
  done
done
echo "== k_main<5> flush cost (diagnostic variants, k = 2^26; wrong top-k by design)"
for v in nostage nosegstore nocands; do
  lib=mpi-k-selection_amd/lib/variants/libkth_$v.so
  KTH_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/diag_$v -o run --output-format csv -- python3 bench.py --workload topk --k 67108864 --steps 5 --warmup 2 --no-cpu-baseline > $O/diag_$v.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "$v rc=$rc"; tail -20 $O/diag_$v.log; exit 1; }
  echo "$v:"; python3 tools/prof_summary.py $(find $O/diag_$v -name "*kernel_trace.csv" | head -1) 0 | grep -E "k_main"
done
echo done
