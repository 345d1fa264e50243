# rocprof kernel stats of the config-5 workloads and two top-k calls on the final build
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/rowsprof; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
i=0
for args in "--workload rows --rows-dtype i32 --k 64" "--workload rows --rows-dtype f32 --k 64" "--workload rows --rows-dtype i32 --topk --k 64" "--workload rows --rows-dtype f32 --topk --k 64" "--workload rows --rows-dtype i32 --rows-input dup --k 64" "--workload rows --rows-dtype f32 --rows-input dup --k 64" "--workload topk --k 1048576" "--workload topk --k 67108864"; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/p$i -o run --output-format csv -- python3 bench.py $args --steps 10 --warmup 2 --no-cpu-baseline > $O/p$i.log 2>&1 || { echo "prof $args rc=$?"; tail -20 $O/p$i.log; exit 1; }
  echo "== $args" >> $O/summary.txt
  python3 tools/prof_summary.py $O/p$i/run_kernel_trace.csv 0 >> $O/summary.txt
done
cat $O/summary.txt
