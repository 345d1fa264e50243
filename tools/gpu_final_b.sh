# Evidence (b): PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE
# passes) on the final build for the select, the rows (k-th and top-k) and the
# staged top-k; the 2^33 lines; the SQ instruction mix of k_main and the rows
# kernels.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/fb; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
pmc2() {  # pmc2 NAME -- bench args: two passes, csv paths in $O/pmc_NAME_{FETCH,WRITE}_SIZE
  local name=$1; shift 2
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 180 rocprofv3 --pmc $c -d $O/pmc_${name}_$c -o run --output-format csv -- python3 bench.py "$@" > $O/pmc_${name}_$c.log 2>&1 || { echo pmc $name $c rc=$?; tail -20 $O/pmc_${name}_$c.log; exit 1; }
  done
}
csv() { find $O/pmc_$1_$2 -name "*counter_collection.csv" | head -1; }
echo "== PMC select"
pmc2 select -- --steps 3 --warmup 1 --no-cpu-baseline
python3 tools/pmc_traffic.py $(csv select FETCH_SIZE) $(csv select WRITE_SIZE) k_main 30 uniform_half $O/pmc_traffic.json | tail -4
for dt in i32 f32; do
  echo "== PMC rows $dt"
  pmc2 rows_$dt -- --workload rows --rows-dtype $dt --k 64 --steps 3 --warmup 1
  python3 tools/pmc_traffic.py $(csv rows_$dt FETCH_SIZE) $(csv rows_$dt WRITE_SIZE) rows_reg 28 rows_$dt $O/pmc_traffic_rows_$dt.json | tail -4
done
for dt in i32 f32; do
  echo "== PMC top-k rows $dt"
  pmc2 rows_topk_$dt -- --workload rows --rows-dtype $dt --topk --k 64 --steps 3 --warmup 1
  python3 tools/pmc_traffic.py $(csv rows_topk_$dt FETCH_SIZE) $(csv rows_topk_$dt WRITE_SIZE) rows_reg 28 rows_topk_$dt $O/pmc_traffic_rows_topk_$dt.json 33554432 | tail -4
done
for k in 1048576 67108864 134217728 536870912; do
  echo "== PMC top-k k=$k"
  pmc2 topk_$k -- --workload topk --k $k --steps 3 --warmup 1 --no-cpu-baseline
  python3 tools/pmc_topk.py $(csv topk_$k FETCH_SIZE) $(csv topk_$k WRITE_SIZE) 30 uniform_half $k $O/pmc_traffic_topk_k$k.json
done
echo "== request sizes of the staged pass (k_main<5>, dword loads since round 6): TCC_EA0_RDREQ vs its 128-B part"
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_32B_sum -d $O/rdreq_tk -o run --output-format csv -- python3 bench.py --workload topk --k 67108864 --steps 3 --warmup 1 --no-cpu-baseline > $O/rdreq_tk.log 2>&1 || { echo rdreq rc=$?; tail -20 $O/rdreq_tk.log; exit 1; }
python3 tools/sq_mix.py $O/rdreq_tk "k_main<5>" 64 "k_main<5> k=2^26 read requests per launch (x 64 keys: raw counts)"
echo "== 2^33 lines"
timeout -k 10 300 python -u bench.py --log2n 33 --steps 10 --warmup 3 --no-cpu-baseline > $O/b33.log 2>&1 || { echo b33 rc=$?; tail -20 $O/b33.log; exit 1; }
tail -1 $O/b33.log | cut -c1-300
timeout -k 10 300 python -u bench.py --log2n 30 --local-shards 8 --steps 10 --warmup 3 --no-cpu-baseline > $O/b8.log 2>&1 || { echo b8 rc=$?; tail -20 $O/b8.log; exit 1; }
tail -1 $O/b8.log | cut -c1-300
echo "== SQ mix per 64-key slot: select k_main<0> vs staged top-k k_main<5> (k = 2^20, 2^26)"
C="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES"
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/sq_sel -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_sel.log 2>&1 || { echo sq rc=$?; tail -20 $O/sq_sel.log; exit 1; }
python3 tools/sq_mix.py $O/sq_sel "k_main<0>" 1073741824 "select k_main<0>"
for k in 1048576 67108864; do
  timeout -s KILL 120 rocprofv3 --pmc $C -d $O/sq_tk_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 3 --warmup 1 --no-cpu-baseline > $O/sq_tk_$k.log 2>&1 || { echo sq rc=$?; tail -20 $O/sq_tk_$k.log; exit 1; }
  python3 tools/sq_mix.py $O/sq_tk_$k "k_main<5>" 1073741824 "top-k k=$k k_main<5>"
done
echo "== SQ mix of the rows kernels per 64-key slot (k-th and top-k, i32 and f32)"
timeout -k 10 600 bash tools/gpu_rows_pmc_sq.sh > $O/rows_sq.txt 2>&1 || { echo rows sq rc=$?; tail -20 $O/rows_sq.txt; exit 1; }
cat $O/rows_sq.txt
echo done
