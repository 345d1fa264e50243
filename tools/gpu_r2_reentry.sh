# round-2 re-entry: smoke, select bench + rocprof, full GPU suite, rows benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
PROF=1 bash tools/gpu_check.sh || exit 1
bash tools/gpu_rows_bench.sh || exit 1
