# rows kernel: histogram-copy variants (LIBS) x dtype, k = 64
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in ${LIBS:-default}; do for dt in i32 f32; do
  if [ "$lib" = default ]; then L=""; else L="$PWD/mpi-k-selection_amd/lib/variants/libkth_$lib.so"; fi
  KTH_LIB=$L timeout -k 10 120 python -u bench.py --workload rows --rows-dtype $dt --k ${K:-64} --steps 10 --warmup 2 > gpurun_out/rows.log 2>&1 || { echo rows $lib $dt rc=$?; tail -20 gpurun_out/rows.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/rows.log').read().strip().splitlines()[-1]); print('$lib $dt', round(d['value'],1), 'Gkeys/s kern', round(d['roofline']['avg_launch_ms'],4), 'ms', round(d['roofline']['achieved']), 'GB/s', d['verified'])"
done; done
