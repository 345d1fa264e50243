# Round-4 diagnostics: the config-3 tests (2^33 one array, 8 local shards,
# lockstep), the warmup ramp of the select, and the per-call kernel times of
# the driver's bench command under rocprof.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/diag; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
echo "== config-3 + sharded + runtime tests"
timeout -k 10 600 python -u -m pytest -x -v --timeout 180 --timeout-method thread tests/test_gpu_config3.py tests/test_gpu_sharded.py tests/test_gpu_runtime.py > $O/tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo "== warmup probe"
timeout -k 10 180 python -u tools/warmup_probe.py > $O/warmup.jsonl 2> $O/warmup.err || { echo warmup rc=$?; tail -20 $O/warmup.err; exit 1; }
cat $O/warmup.jsonl
echo "== 2^33 probe"
timeout -k 10 300 python -u tools/probe_2e33.py 33 uniform_half 5 > $O/p33.jsonl 2> $O/p33.err || { echo p33 rc=$?; tail -20 $O/p33.err; exit 1; }
cat $O/p33.jsonl
echo "== bench lines: default (driver command), 2^33 one array, 8 local shards"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b30.log 2>&1 || { echo b30 rc=$?; tail -20 $O/b30.log; exit 1; }
tail -1 $O/b30.log | cut -c1-600
timeout -k 10 300 python -u bench.py --log2n 33 --steps 10 --warmup 3 --no-cpu-baseline > $O/b33.log 2>&1 || { echo b33 rc=$?; tail -20 $O/b33.log; exit 1; }
tail -1 $O/b33.log | cut -c1-600
timeout -k 10 300 python -u bench.py --log2n 30 --local-shards 8 --steps 10 --warmup 3 --no-cpu-baseline > $O/b8.log 2>&1 || { echo b8 rc=$?; tail -20 $O/b8.log; exit 1; }
tail -1 $O/b8.log | cut -c1-600
echo "== rocprof of the driver's bench command"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/prof.log 2>&1 || { echo prof rc=$?; tail -20 $O/prof.log; exit 1; }
python3 tools/prof_calls.py $O/prof/run_kernel_trace.csv
echo done
