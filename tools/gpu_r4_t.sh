# Round 4 (t): the select's k_main<0> with a larger per-wave candidate region
# (KTH_WREG 2560 / 3072 words against 2048): driver-command bench and rocprof
# per-kernel times, twice, on one box
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4t; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
L=$PWD/mpi-k-selection_amd/lib
for rep in 1 2; do
for v in base wreg2560 wreg3072; do
  lib=$L/variants/libkth_$v.so; [ $v = base ] && lib=$L/libkth.so
  KTH_LIB=$lib timeout -k 10 120 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/sel_$v.log 2>&1 || { echo sel rc=$?; tail -20 $O/sel_$v.log; exit 1; }
  KTH_LIB=$lib timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p_${v}_$rep -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/p_${v}.log 2>&1 || { echo prof rc=$?; tail -20 $O/p_${v}.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/sel_$v.log').read().strip().splitlines()[-1]); print('select $v', round(d['value'],1), 'Gkeys/s')"
  python3 tools/prof_summary.py $O/p_${v}_$rep/run_kernel_trace.csv | grep -E "k_main|k_finish|k_head" | cut -c1-80
done
done
echo done
