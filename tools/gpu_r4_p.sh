# Round 4 (p): what k_tk5_write's output stores cost: timing-only builds with
# no stores (tkw_nostore) and with the stores folded onto 64 Ki L2-resident
# slots (tkw_smallout), against the default build, k = 2^24 / 2^26
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4p; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
L=$PWD/mpi-k-selection_amd/lib
for k in 16777216 67108864; do
  for v in base tkw_nostore tkw_smallout; do
    lib=$L/variants/libkth_$v.so; [ $v = base ] && lib=$L/libkth.so
    KTH_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_${v}_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 5 --warmup 2 --no-cpu-baseline > $O/p_${v}_$k.log 2>&1; rc=$?
    [ $rc -le 1 ] || { echo prof rc=$rc; tail -20 $O/p_${v}_$k.log; exit 1; }
    echo "k=$k $v"; python3 tools/prof_summary.py $O/p_${v}_$k/run_kernel_trace.csv 0 | grep -E "tk5_write|k_main"
  done
done
echo done
