# quick loop (needs `make -C mpi-k-selection_amd variant V=stamps VFLAGS=-DKTH_STAMPS_BUILD`): stamps of the streaming pass, bench per grid size, core GPU tests
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp

KTH_LIB=$PWD/mpi-k-selection_amd/lib/variants/libkth_stamps.so KTH_STAMPS=1 timeout -k 10 120 python -u tools/stamps_probe.py 30 > gpurun_out/st.log 2>&1 || { echo stamps rc=$?; tail gpurun_out/st.log; exit 1; }
grep -A30 "select 3" gpurun_out/st.log | grep -E "kth-stamps"
for per in ${PERS:-""}; do
  KTH_MAIN_WG_PER_CU=$per timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/q.log 2>&1 || { echo bench rc=$?; tail -20 gpurun_out/q.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/q.log').read().strip().splitlines()[-1]); print('per=${per:-auto}', round(d['value'],1), 'Gkeys/s', round(d['ms_per_step'],4), 'ms main', round(d['roofline']['avg_launch_ms'],4), 'total', round(d['whole_select_ms_events'],4), d['verified'])"
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -m gpu ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/pytest.log
exit $rc
