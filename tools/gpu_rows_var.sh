# rows: parity tests of the default library, then bench of variants (LIBS) x dtype x k
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu -k "rows" > gpurun_out/pytest_rows.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_rows.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/pytest_rows.log | head -20; exit 1; }
for lib in ${LIBS:-default}; do for dt in i32 f32; do for k in ${KS:-64}; do
  if [ "$lib" = default ]; then L=""; else L="$PWD/mpi-k-selection_amd/lib/variants/libkth_$lib.so"; fi
  KTH_LIB=$L timeout -k 10 120 python -u bench.py --workload rows --rows-dtype $dt --k $k --steps 20 --warmup 3 $BARGS > gpurun_out/rows.log 2>&1 || { echo rows $lib $dt rc=$?; tail -20 gpurun_out/rows.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/rows.log').read().strip().splitlines()[-1]); print('$lib $dt k=$k', round(d['value'],1), 'Gkeys/s kern', round(d['roofline']['avg_launch_ms'],4), 'ms', round(d['roofline']['achieved']), 'GB/s', d['verified'])"
done; done; done
