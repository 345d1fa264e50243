# bench sweep over library variants x streaming-pass grid sizes (design exploration)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for lib in ${LIBS:-default}; do
  for per in ${PERS:-"" 4 8}; do
    if [ "$lib" = default ]; then L=""; else L="$PWD/mpi-k-selection_amd/lib/variants/libkth_$lib.so"; fi
    KTH_LIB=$L KTH_MAIN_WG_PER_CU=$per timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sweep.log 2>&1 || { echo fail $lib $per; tail -5 gpurun_out/sweep.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/sweep.log').read().strip().splitlines()[-1]); print('$lib per=${per:-auto}', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms', 'main', round(d['roofline']['avg_launch_ms'],4), 'ms', round(d['roofline']['achieved']), 'GB/s', d['verified'])"
  done
done
