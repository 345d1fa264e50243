# The round's committed evidence: the default bench line (+ CPU baselines), rocprof kernel
# stats, PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes) for the
# select path, and the same for the batched-rows path (int32 and f32).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/profiles; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
pmc() {  # pmc NAME KERNEL_SUBSTR LOG2N FAMILY -- bench args
  local name=$1 kern=$2 l2=$3 fam=$4; shift 5
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c -d $O/pmc_${name}_$c -o run --output-format csv -- python3 bench.py "$@" > $O/pmc_${name}_$c.log 2>&1 || { echo pmc $name $c rc=$?; tail -20 $O/pmc_${name}_$c.log; exit 1; }
  done
  F=$(find $O/pmc_${name}_FETCH_SIZE -name "*counter_collection.csv" | head -1)
  W=$(find $O/pmc_${name}_WRITE_SIZE -name "*counter_collection.csv" | head -1)
  python3 tools/pmc_traffic.py "$F" "$W" "$kern" $l2 $fam $O/pmc_traffic_$name.json || exit 1
}
echo "== select: PMC"
pmc select k_main 30 uniform_half -- --steps 3 --warmup 1 --no-cpu-baseline
cp $O/pmc_traffic_select.json profiles/pmc_traffic.json
echo "== select: bench"
timeout -k 10 400 python -u bench.py > $O/bench.log 2>&1 || { echo bench rc=$?; tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
echo "== select: rocprof"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_select -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > $O/prof_select.log 2>&1 || { echo prof rc=$?; tail -20 $O/prof_select.log; exit 1; }
python3 tools/prof_summary.py $O/prof_select/run_kernel_trace.csv > $O/select_summary.txt; head -8 $O/select_summary.txt
for dt in i32 f32; do
  echo "== rows $dt"
  pmc rows_$dt rows_reg 28 rows_$dt -- --workload rows --rows-dtype $dt --k 64 --steps 3 --warmup 1
  cp $O/pmc_traffic_rows_$dt.json profiles/
  timeout -k 10 120 python -u bench.py --workload rows --rows-dtype $dt --k 64 --steps 20 --warmup 3 > $O/rows_$dt.log 2>&1 || { echo rows rc=$?; tail -20 $O/rows_$dt.log; exit 1; }
  tail -1 $O/rows_$dt.log
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof_rows_$dt -o run --output-format csv -- python3 bench.py --workload rows --rows-dtype $dt --k 64 --steps 10 --warmup 2 > $O/prof_rows_$dt.log 2>&1 || { echo prof rc=$?; tail -20 $O/prof_rows_$dt.log; exit 1; }
done
echo done
