# sample chunk size A/B: 1024-key (default) vs 4096-key chunks, select bench + head stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
V=$PWD/mpi-k-selection_amd/lib/variants
for rep in 1 2; do
for lib in default $V/libkth_ck64.so; do
  if [ $lib = default ]; then unset KTH_LIB; else export KTH_LIB=$lib; fi
  timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$(basename $lib)', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms; main', round(r['avg_launch_ms'],4), 'whole', round(d.get('whole_select_ms_events'),4), 'cand', d.get('candidates'), d['verified'])"
done
done
export KTH_LIB=$V/libkth_ck64stamps.so
KTH_STAMPS=1 timeout -k 10 120 python -u tools/stamps_probe.py 30 > gpurun_out/st4.log 2>&1 || exit 1
grep -A1 "select 3" gpurun_out/st4.log
