# Round 4 (x): config 5's duplicate-heavy rows over k in {1, 64, 2048, 4096}
# (the k = 2048 float bin holds both zeros: its ends from the signed zeros
# present, default, against the order-key loop of the build before, prevrows);
# rows parity first
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4x; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
echo "== rows tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "rows" > $O/rows_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error" $O/rows_tests.log | head -30; tail -5 $O/rows_tests.log; exit 1; }
tail -1 $O/rows_tests.log
L=mpi-k-selection_amd/lib
one() {  # lib args (args carry --k)
  KTH_LIB=$1 timeout -k 10 120 python -u bench.py --workload rows $2 --steps 20 --warmup 3 --no-cpu-baseline > $O/rows.log 2>&1; rc=$?
  [ $rc -le 0 ] || { echo "bench rc=$rc"; tail -20 $O/rows.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/rows.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$(basename $1)', '$2', 'k', d['config']['k'], round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us', d['verified'])"
}
for lib in $L/libkth.so $L/variants/libkth_prevrows.so; do
  for dt in i32 f32; do
    for k in 1 64 2048 4096; do one $lib "--rows-dtype $dt --rows-input dup --k $k" || exit 1; done
  done
done
for dt in i32 f32; do one $L/libkth.so "--rows-dtype $dt --k 64" || exit 1; done
echo done
