set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r2_bench0.json 2> gpurun_out/r2_bench0.err || { echo bench rc=$?; tail -20 gpurun_out/r2_bench0.err; exit 1; }
cat gpurun_out/r2_bench0.json
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r2_prof0 -o run -- python3 -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/r2_prof0.log 2>&1 || { echo prof rc=$?; tail gpurun_out/r2_prof0.log; exit 1; }
find gpurun_out/r2_prof0 -name '*kernel_stats.csv' | head -1 | xargs head -12
