set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 ./tools/stream_probe 30 > gpurun_out/probe.log 2>&1 || { echo probe rc=$?; cat gpurun_out/probe.log; exit 1; }
cat gpurun_out/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/bench_prof.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/bench_prof.log; exit 1; }
tail -3 gpurun_out/bench_prof.log
find gpurun_out/prof_r1 -name "*stats*" | head
