# Round 4 (z3): f32 top-k rows compacting from registers (default) against the re-read (nokeyc)
# registers (default) instead of re-reading the row (nokeyc): rows parity,
# then top-k rows on uniform and duplicate-heavy input
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4z3; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
echo "== rows tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "rows" > $O/rows_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error" $O/rows_tests.log | head -30; tail -5 $O/rows_tests.log; exit 1; }
tail -1 $O/rows_tests.log
L=mpi-k-selection_amd/lib
one() {  # lib args
  KTH_LIB=$1 timeout -k 10 120 python -u bench.py --workload rows $2 --steps 20 --warmup 3 --no-cpu-baseline > $O/rows.log 2>&1; rc=$?
  [ $rc -le 0 ] || { echo "bench rc=$rc"; tail -20 $O/rows.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/rows.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$(basename $1)', '$2', round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us', d['verified'])"
}
for rep in 1 2; do
  for lib in $L/libkth.so $L/variants/libkth_nokeyc.so; do
    for args in "--rows-dtype f32 --topk --k 64" "--rows-dtype f32 --topk --rows-input dup --k 64" "--rows-dtype f32 --k 64"; do one $lib "$args" || exit 1; done
  done
done
echo done
