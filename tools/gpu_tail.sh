# k_finish tail (last workgroup finishes the small bin alone): parity, bench, stamps
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_topk.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/tail_parity.log 2>&1; rc=$?
tail -3 gpurun_out/tail_parity.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms; main', round(r['avg_launch_ms'],4), 'whole', round(d.get('whole_select_ms_events'),4), 'cand', d.get('candidates'), d['verified'])"
done
bash tools/gpu_stamps.sh
