# The sharded protocol on one MI355X: its GPU tests, then the config-3 shapes
# (8 local shards x 2^30 through kth_sharded_*, and one array of 2^33) and the
# one-rank RCCL protocol (bench.py --dist), with a kernel trace of the local-shard run.
# Usage: gpurun -- bash tools/gpu_dist.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-dist}; O=gpurun_out/$T; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest ${TESTS:-tests/test_gpu_config3.py tests/test_gpu_sharded.py tests/test_gpu_runtime.py tests/test_cgm_driver.py tests/test_gpu_parity.py::test_dist_world1_nccl} -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|assert" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 300 python -u bench.py --local-shards 8 --steps 10 --warmup 3 --no-cpu-baseline > $O/local8.json 2> $O/local8.err || { echo local8 rc=$?; tail -20 $O/local8.err; exit 1; }
timeout -k 10 300 python -u bench.py --log2n 33 --steps 10 --warmup 3 --no-cpu-baseline > $O/one33.json 2> $O/one33.err || { echo one33 rc=$?; tail -20 $O/one33.err; exit 1; }
timeout -k 10 300 python -u bench.py --dist --steps 20 --warmup 5 --no-cpu-baseline > $O/dist1.json 2> $O/dist1.err || { echo dist1 rc=$?; tail -20 $O/dist1.err; exit 1; }
python3 - <<PY
import json
for f in ("local8", "one33", "dist1"):
    d = json.loads(open("$O/%s.json" % f).read().strip().splitlines()[-1])
    print(f, round(d["value"], 1), d["unit"], round(d["ms_per_step"], 4), "ms", "verified", d["verified"])
PY
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$O/prof_local8 -o run -- python3 $GRAFT_REPO_ROOT/bench.py --local-shards 8 --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/$O/prof_local8.log 2>&1 || { echo prof rc=$?; tail -5 $GRAFT_REPO_ROOT/$O/prof_local8.log; exit 1; }
echo done
