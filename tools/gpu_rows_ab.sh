# A/B of rows benches across library variants (LIBS) and workloads (WL)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
for lib in ${LIBS:-default}; do
  if [ "$lib" = default ]; then L=""; else L="$PWD/mpi-k-selection_amd/lib/variants/libkth_$lib.so"; fi
  for args in ${WL:-"--rows-dtype=i32 --rows-dtype=f32"}; do
    KTH_LIB=$L timeout -k 10 120 python -u bench.py --workload rows ${args//,/ } --k 64 --steps 20 --warmup 3 > gpurun_out/rows.log 2>&1; rc=$?
    [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/rows.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/rows.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$lib $args', round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us frac', round(r['frac'],3), d['verified'])"
  done
done
done
