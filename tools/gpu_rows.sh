# batched rows (BASELINE config 5): int32 / f32, several k
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for dt in i32 f32; do for k in 1 64 2048 4096; do
  timeout -k 10 120 python -u bench.py --workload rows --rows-dtype $dt --k $k --steps 10 --warmup 2 > gpurun_out/rows.log 2>&1 || { echo rows $dt $k rc=$?; tail -20 gpurun_out/rows.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/rows.log').read().strip().splitlines()[-1]); print('$dt k=$k', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms kern', round(d['roofline']['avg_launch_ms'],4), round(d['roofline']['achieved']), 'GB/s', d['verified'])"
done; done
