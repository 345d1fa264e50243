# sharded protocol on one GPU (one-rank RCCL group): bench, kernel trace, world-1 test
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 180 python -u bench.py --dist --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/dist_b.log 2>&1 || { echo bench rc=$?; tail -20 gpurun_out/dist_b.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/dist_b.log').read().strip().splitlines()[-1]); print('dist', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms main', round(d['roofline']['avg_launch_ms'],4), d['verified'])"
  timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/b.log 2>&1 || { echo bench rc=$?; tail -20 gpurun_out/b.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/b.log').read().strip().splitlines()[-1]); print('single', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms main', round(d['roofline']['avg_launch_ms'],4), d['verified'])"
done
rm -rf gpurun_out/dist_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/dist_prof -o run -- python3 bench.py --dist --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/dist_prof.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/dist_prof.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests -x -q --timeout 120 --timeout-method thread -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/pytest.log
exit $rc
