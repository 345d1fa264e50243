# The whole -m gpu suite (one process), smoke(), and the default bench line.
# Usage: gpurun -- bash tools/gpu_suite.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-suite}; O=gpurun_out/$T; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error" $O/gpu_tests.log | head -20; tail -5 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke rc=$?; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo bench rc=$?; tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('bench', round(d['value'],1), d['unit'], round(d['ms_per_step'],4), 'ms frac', round(d['roofline']['frac'],3), 'verified', d['verified'])"
