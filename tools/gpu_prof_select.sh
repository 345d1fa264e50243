# rocprof kernel trace + stats of the driver's bench command (the headline select),
# and the per-call kernel durations (tools/prof_calls.py).  Usage: bash tools/gpu_prof_select.sh <tag> [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-prof}; shift; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_select -o run --output-format csv -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/prof_select.log 2>&1 || { echo prof rc=$?; tail -20 $O/prof_select.log; exit 1; }
python3 tools/prof_summary.py $O/prof_select/run_kernel_trace.csv > $O/prof_select_summary.txt 2>&1 || true
python3 tools/prof_calls.py $O/prof_select/run_kernel_trace.csv > $O/prof_select_calls.txt 2>&1 || true
head -20 $O/prof_select_summary.txt; head -8 $O/prof_select_calls.txt
