# top-k benches and the sharded protocol at world 1 (evidence for DESIGN)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -f gpurun_out/topk_bench.jsonl
for k in 1024 16385 1048576 16777216 536870912; do
  timeout -k 10 120 python -u bench.py --workload topk --k $k --steps 10 --warmup 3 > gpurun_out/tk.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/tk.log; exit 1; }
  tail -1 gpurun_out/tk.log >> gpurun_out/topk_bench.jsonl
  python3 -c "import json; d=json.loads(open('gpurun_out/tk.log').read().strip().splitlines()[-1]); r=d['roofline']; print('k=$k', round(d['ms_per_step'],4), 'ms', round(d['value'],1), 'Gkeys/s frac', round(r['frac'],3), d['verified'])"
done
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29535
timeout -k 10 180 python -u bench.py --dist --no-cpu-baseline > gpurun_out/dist1.log 2>&1 || { echo rc=$?; tail -20 gpurun_out/dist1.log; exit 1; }
tail -1 gpurun_out/dist1.log > gpurun_out/dist1.json
python3 -c "import json; d=json.load(open('gpurun_out/dist1.json')); print('dist world1', round(d['value'],1), round(d['ms_per_step'],4), d['config']['parallelism'], d['config'].get('rccl_world'), d['verified'])"
