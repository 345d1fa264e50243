# round-2 resume check: smoke, select bench, GPU tests, rows benches
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_check.sh || exit 1
bash tools/gpu_rows_bench.sh || exit 1
