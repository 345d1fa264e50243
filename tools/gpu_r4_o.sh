# Round 4 (o): HBM traffic of the top-k rows kernel (is the output written
# without read-for-ownership fills?), both dtypes
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4o; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
pmc2() {
  local name=$1; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c -d $O/pmc_${name}_$c -o run --output-format csv -- python3 bench.py "$@" > $O/pmc_${name}_$c.log 2>&1 || { echo pmc $name $c rc=$?; tail -20 $O/pmc_${name}_$c.log; exit 1; }
  done
}
csv() { find $O/pmc_$1_$2 -name "*counter_collection.csv" | head -1; }
for dt in i32 f32; do
  pmc2 rows_topk_$dt -- --workload rows --rows-dtype $dt --topk --k 64 --steps 3 --warmup 1
  python3 tools/pmc_traffic.py $(csv rows_topk_$dt FETCH_SIZE) $(csv rows_topk_$dt WRITE_SIZE) rows_reg 28 rows_topk_$dt $O/pmc_traffic_rows_topk_$dt.json 33554432 | grep -E "read_bytes|write_bytes|over"
done
echo done
