# rocprof kernel trace of the bench for the default library and variants (LIBS)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for lib in ${LIBS:-default}; do
  if [ "$lib" = default ]; then L=""; else L="$PWD/mpi-k-selection_amd/lib/variants/libkth_$lib.so"; fi
  KTH_LIB=$L KTH_MAIN_WG_PER_CU=${PER:-5} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$lib -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_$lib.log 2>&1 || { echo prof rc=$?; tail -20 gpurun_out/prof_$lib.log; exit 1; }
  echo "== $lib"; python3 tools/prof_summary.py gpurun_out/prof_$lib/run_kernel_trace.csv
done
