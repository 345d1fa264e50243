# Round 4 (g): candidate staging through a collector register (one LDS write
# per 64 candidates) against the per-slot LDS append (KTH_STAGE_COLLECT=0):
# parity, the warmup transient (k_main per call after an idle start), and the
# driver's bench command, alternating libraries on one box.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4g; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
echo "== select parity (parity + config 3 + sharded + runtime)"
timeout -k 10 900 python -u -m pytest -x -q --timeout 180 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_config3.py tests/test_gpu_sharded.py tests/test_gpu_runtime.py tests/test_gpu_topk.py > $O/tests.log 2>&1 || { echo tests rc=$?; grep -E "FAIL|Error|error" $O/tests.log | head -30; tail -5 $O/tests.log; exit 1; }
tail -1 $O/tests.log
echo "== transient: k_main per call after idle"
for v in base nocollect; do
  lib=mpi-k-selection_amd/lib/variants/libkth_$v.so; [ $v = base ] && lib=mpi-k-selection_amd/lib/libkth.so
  KTH_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace -d $O/bump_$v -o run --output-format csv -- python3 tools/bump_probe.py uniform_half > $O/bump_$v.log 2>&1 || { echo "bump $v rc=$?"; tail -20 $O/bump_$v.log; exit 1; }
  echo "$v:"; python3 tools/prof_calls.py $(find $O/bump_$v -name "*kernel_trace.csv" | head -1) | grep "k_main" | cut -c1-520
done
echo "== driver bench command, alternating"
for v in base nocollect base nocollect; do
  lib=mpi-k-selection_amd/lib/variants/libkth_$v.so; [ $v = base ] && lib=mpi-k-selection_amd/lib/libkth.so
  KTH_LIB=$PWD/$lib timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/b_$v.log 2>&1 || { echo "bench $v rc=$?"; tail -20 $O/b_$v.log; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/b_$v.log').read().strip().splitlines()[-1])
print('$v', round(d['value'],1), 'ms', round(d['ms_per_step'],4), 'ev', round(d['ms_per_step_events'],4), 'k_main', round(d['roofline']['avg_launch_ms'],4), d['verified'])"
done
echo done
