# A/B of library variants (lib/variants/libkth_<name>.so, make variant) on one
# workload: rocprof kernel averages per variant.  VARIANTS="a b", ARGS="bench args"
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/var; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
for v in base $VARIANTS; do
  lib=mpi-k-selection_amd/lib/variants/libkth_$v.so; [ $v = base ] && lib=mpi-k-selection_amd/lib/libkth.so
  KTH_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o run --output-format csv -- python3 bench.py $ARGS > $O/$v.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "$v rc=$rc"; tail -20 $O/$v.log; exit 1; }
  echo "== $v"; python3 tools/prof_summary.py $(find $O/$v -name "*kernel_trace.csv" | head -1) 0 | head -${TOPN:-6}
done
