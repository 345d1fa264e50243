# Round 4 (j): k_rows_reg's row loop (the next row's loads in flight during the
# list / rank / copy-out tail): rows parity on the new default build, then the
# rows workloads (config 5, k = 64) on the default build and the variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4j; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
echo "== rows tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "rows" > $O/rows_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error" $O/rows_tests.log | head -30; tail -5 $O/rows_tests.log; exit 1; }
tail -1 $O/rows_tests.log
L=mpi-k-selection_amd/lib
for rep in 1 2; do
for lib in $L/libkth.so $L/variants/libkth_noloop.so $L/variants/libkth_loopw5.so $L/variants/libkth_loopb64.so; do
  for args in "--rows-dtype i32" "--rows-dtype f32" "--rows-dtype i32 --topk" "--rows-dtype f32 --topk"; do
    KTH_LIB=$lib timeout -k 10 120 python -u bench.py --workload rows $args --k 64 --steps 20 --warmup 3 --no-cpu-baseline > $O/rows.log 2>&1 || { echo "bench rc=$?"; tail -20 $O/rows.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/rows.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$(basename $lib)', '$args', round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us', d['verified'])"
  done
done
done
echo done
