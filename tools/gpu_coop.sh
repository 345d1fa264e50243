# cooperative head/finish kernels: parity first, then A/B vs per-level launches, rocprof, full GPU suite
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/coop_parity.log 2>&1; rc=$?
tail -5 gpurun_out/coop_parity.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2; do
for cfg in "KTH_COOP=0" "KTH_COOP=1 KTH_HEAD_SLACK=0" "KTH_COOP=1 KTH_HEAD_SLACK=1.05" "KTH_COOP=1 KTH_HEAD_SLACK=1.5" "KTH_COOP=1 KTH_HEAD_SLACK=3"; do
  env $cfg timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$cfg', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms; main', round(r['avg_launch_ms'],4), 'whole', round(d.get('whole_select_ms_events'),4), 'cand', d.get('candidates'), d['verified'])"
done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/coop_prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/coop_prof.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/coop_prof.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/coop_prof/run_kernel_trace.csv
timeout -k 10 600 python -u -m pytest tests/ -x -q --timeout 120 --timeout-method thread -m gpu > gpurun_out/coop_pytest.log 2>&1; rc=$?
tail -5 gpurun_out/coop_pytest.log
[ $rc -eq 0 ] || exit $rc
# (appended) rows k-th vs top-k instruction mix
WL="--rows-dtype=i32 --rows-dtype=i32,--topk --rows-dtype=f32 --rows-dtype=f32,--topk" bash tools/gpu_rows_pmc2.sh
