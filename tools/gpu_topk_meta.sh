# top-k for k > n/1024 from the streaming pass's row counts: parity, benches, rocprof
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_topk.py -x -q --timeout 200 --timeout-method thread -m gpu > gpurun_out/topk_parity.log 2>&1; rc=$?
tail -3 gpurun_out/topk_parity.log; [ $rc -eq 0 ] || exit 1
for k in 64 1024 16384 16385 1048576 16777216 536870912; do
  timeout -k 10 120 python -u bench.py --workload topk --k $k --steps 10 --warmup 3 > gpurun_out/tk.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/tk.log; exit 1; }
  tail -1 gpurun_out/tk.log >> gpurun_out/topk_bench.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/tk.log').read().strip().splitlines()[-1]); r=d['roofline']; print('k=$k', round(d['ms_per_step'],4), 'ms', round(d['value'],1), 'Gkeys/s frac', round(r['frac'],3), d['verified'])"
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/tk_prof -o run --output-format csv -- python3 bench.py --workload topk --k 1048576 --steps 5 --warmup 2 > gpurun_out/tk_prof.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/tk_prof.log; exit 1; }
python3 tools/prof_summary.py gpurun_out/tk_prof/run_kernel_trace.csv | head -14
