# Round 4 (s): a larger per-wave staging region (KTH_WREG 3072 / 4096 words,
# default 2048): fewer flushes of k_main<5> at high density, fewer workgroups
# per CU; k_main<5> at k = 2^24 / 2^26 and the plain select's k_main<0>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4s; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
L=$PWD/mpi-k-selection_amd/lib
for v in base wreg3072 wreg4096; do
  lib=$L/variants/libkth_$v.so; [ $v = base ] && lib=$L/libkth.so
  for k in 16777216 67108864; do
    KTH_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_${v}_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 5 --warmup 2 --no-cpu-baseline > $O/p_${v}_$k.log 2>&1 || { echo prof rc=$?; tail -20 $O/p_${v}_$k.log; exit 1; }
    echo "k=$k $v $(python3 tools/prof_summary.py $O/p_${v}_$k/run_kernel_trace.csv 0 | grep -E 'k_main' | cut -c1-80) | $(tail -1 $O/p_${v}_$k.log | cut -c1-120)"
  done
  KTH_LIB=$lib timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sel_$v.log 2>&1 || { echo sel rc=$?; tail -20 $O/sel_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/sel_$v.log').read().strip().splitlines()[-1]); print('select $v', round(d['value'],1), 'Gkeys/s', round(d['roofline']['avg_launch_ms']*1e3,1), 'us k_main')"
done
echo done
