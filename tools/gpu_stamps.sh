# Phase stamps of the select (stamps builds, KTH_STAMPS=1): for each given
# variant library, the last 3 selects' per-launch stamp lines.
# Usage: [BENCH_ARGS="--family all_equal"] gpurun -- bash tools/gpu_stamps.sh <tag> <variant>...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-stamps}; shift; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for v in "$@"; do
  KTH_LIB=$PWD/mpi-k-selection_amd/lib/variants/libkth_$v.so KTH_STAMPS=1 timeout -k 10 200 python -u bench.py --steps 3 --warmup 40 --no-cpu-baseline $BENCH_ARGS > $O/$v$SUFFIX.json 2> $O/$v$SUFFIX.err || { echo "$v rc=$?"; tail -20 $O/$v$SUFFIX.err; exit 1; }
  echo "== $v $BENCH_ARGS"; grep "kth-stamps launch" $O/$v$SUFFIX.err | tail -3
done
