# bench the default library and variants (LIBS) at several streaming-pass
# occupancies (PERS: workgroups per CU; "auto" = derived from k_main's VGPRs)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in ${LIBS:-default}; do
  if [ "$lib" = default ]; then L=""; else L="$PWD/mpi-k-selection_amd/lib/variants/libkth_$lib.so"; fi
  for per in ${PERS:-auto}; do
    P=$per; [ "$per" = auto ] && P=""
    KTH_LIB=$L KTH_MAIN_WG_PER_CU=$P timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/v.log 2>&1; rc=$?; [ $rc -le 1 ] || { echo bench rc=$rc; tail -20 gpurun_out/v.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/v.log').read().strip().splitlines()[-1]); print('$lib per=$per', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms main', round(d['roofline']['avg_launch_ms'],4), 'frac', round(d['roofline']['frac'],4), d['verified'])"
  done
done
