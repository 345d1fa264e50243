# rows workloads (BASELINE config 5): k-th per row and top-k per row, int32 and f32, k = 64
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for args in "--rows-dtype i32" "--rows-dtype f32" "--rows-dtype i32 --topk" "--rows-dtype f32 --topk"; do
  timeout -k 10 120 python -u bench.py --workload rows $args --k 64 --steps 20 --warmup 3 > gpurun_out/rows.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 gpurun_out/rows.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/rows.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$args', round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us frac', round(r['frac'],3), d['verified'])"
done
