# k_head fast gather: parity (select paths), select bench x3, head stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/h_parity.log 2>&1; rc=$?
tail -2 gpurun_out/h_parity.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms; main', round(r['avg_launch_ms'],4), 'whole', round(d.get('whole_select_ms_events'),4), 'cand', d.get('candidates'), d['verified'])"
done
KTH_LIB=$PWD/mpi-k-selection_amd/lib/variants/libkth_stamps.so KTH_STAMPS=1 timeout -k 10 120 python -u tools/stamps_probe.py 30 > gpurun_out/st5.log 2>&1 || exit 1
grep -A4 "select 3" gpurun_out/st5.log | grep "launch"
