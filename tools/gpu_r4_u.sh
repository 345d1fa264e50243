# Round 4 (u): k_topk_write loads the next tile's keys before this tile's
# copy-out stores (a fixed store count, so the wait covers the prefetch only);
# top-k parity, then k_topk_write against the build without it (noprefetch)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4u; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
echo "== top-k tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_topk.py > $O/topk_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error" $O/topk_tests.log | head -30; tail -5 $O/topk_tests.log; exit 1; }
tail -1 $O/topk_tests.log
L=$PWD/mpi-k-selection_amd/lib
for k in 1024 1048576 134217728 536870912; do
  for v in base noprefetch; do
    lib=$L/variants/libkth_$v.so; [ $v = base ] && lib=$L/libkth.so
    KTH_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_${v}_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 5 --warmup 2 --no-cpu-baseline > $O/p_${v}_$k.log 2>&1 || { echo prof rc=$?; tail -20 $O/p_${v}_$k.log; exit 1; }
    echo "k=$k $v $(python3 tools/prof_summary.py $O/p_${v}_$k/run_kernel_trace.csv 0 | grep -E 'k_topk_write' | cut -c1-80)"
  done
done
echo done
