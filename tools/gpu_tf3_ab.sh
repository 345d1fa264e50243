# k_main<3> cost split: row tags vs row words (diagnostic variants; results of the variants are wrong on purpose)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for v in default nostore noscan noroww norows; do
  if [ $v = default ]; then export KTH_LIB=; else export KTH_LIB=$PWD/mpi-k-selection_amd/lib/variants/libkth_$v.so; fi
  [ -n "$KTH_LIB" ] || unset KTH_LIB
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/ab_$v -o run --output-format csv -- python3 bench.py --workload topk --k 1048576 --steps 8 --warmup 2 > gpurun_out/ab_$v.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "prof rc=$rc"; tail -20 gpurun_out/ab_$v.log; exit 1; }
  echo "== $v"; grep -E "k_main" gpurun_out/ab_$v/run_kernel_stats.csv | cut -d, -f1-4
done
