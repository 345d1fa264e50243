# Round 4 (r): k_main<5>'s dense staging slots by mbcnt of the four ballots and
# dummy-slot writes (default) against the wave scan + exec-masked writes
# (scandense variant): top-k parity, then k_main<5> at k = 2^20 .. 2^26
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4r; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
echo "== top-k tests"
timeout -k 10 600 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_topk.py > $O/topk_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error" $O/topk_tests.log | head -30; tail -5 $O/topk_tests.log; exit 1; }
tail -1 $O/topk_tests.log
L=$PWD/mpi-k-selection_amd/lib
for rep in 1 2; do
for k in 1048576 16777216 33554432 67108864; do
  for v in base scandense; do
    lib=$L/variants/libkth_$v.so; [ $v = base ] && lib=$L/libkth.so
    KTH_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_${v}_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 5 --warmup 2 --no-cpu-baseline > $O/p_${v}_$k.log 2>&1 || { echo prof rc=$?; tail -20 $O/p_${v}_$k.log; exit 1; }
    echo "k=$k $v $(python3 tools/prof_summary.py $O/p_${v}_$k/run_kernel_trace.csv 0 | grep -E 'k_main' | cut -c1-80)"
  done
done
done
echo done
