# two separate PMC passes (FETCH_SIZE, WRITE_SIZE) over a short bench run
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 180 rocprofv3 --pmc $c -d gpurun_out/pmc_$c -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_$c.log 2>&1 || { echo pmc $c rc=$?; tail -20 gpurun_out/pmc_$c.log; exit 1; }
done
F=$(find gpurun_out/pmc_FETCH_SIZE -name "*counter_collection.csv" | head -1)
W=$(find gpurun_out/pmc_WRITE_SIZE -name "*counter_collection.csv" | head -1)
python3 tools/pmc_traffic.py "$F" "$W" "k_main" 30 uniform_half gpurun_out/pmc_traffic.json
