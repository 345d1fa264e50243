# select + top-k: parity, select bench x3, top-k benches, rocprof of the select
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_topk.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/st_parity.log 2>&1; rc=$?
tail -2 gpurun_out/st_parity.log; [ $rc -eq 0 ] || exit 1
for rep in 1 2 3; do
  timeout -k 10 120 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/ab.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab.log').read().strip().splitlines()[-1]); r=d['roofline']; print(round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms; main', round(r['avg_launch_ms'],4), 'whole', round(d.get('whole_select_ms_events'),4), d['verified'])"
done
rm -f gpurun_out/topk_bench.jsonl
for k in 1024 16385 1048576 536870912; do
  timeout -k 10 120 python -u bench.py --workload topk --k $k --steps 10 --warmup 3 > gpurun_out/tk.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/tk.log; exit 1; }
  tail -1 gpurun_out/tk.log >> gpurun_out/topk_bench.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/tk.log').read().strip().splitlines()[-1]); r=d['roofline']; print('k=$k', round(d['ms_per_step'],4), 'ms', round(d['value'],1), 'Gkeys/s frac', round(r['frac'],3), d['verified'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/bench_prof.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/prof/run_kernel_trace.csv
