# phase stamps of the select's launches (diagnostic build): default and KTH_HEAD_SLACK=0
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for cfg in "KTH_HEAD_SLACK=1.5" "KTH_HEAD_SLACK=0" ${EXTRA_CFGS}; do
  echo "== $cfg"
  env $cfg KTH_LIB=$PWD/mpi-k-selection_amd/lib/variants/libkth_stamps.so KTH_STAMPS=1 timeout -k 10 120 python -u tools/stamps_probe.py 30 > gpurun_out/st.log 2>&1 || { echo stamps rc=$?; tail gpurun_out/st.log; exit 1; }
  grep -A12 "select 3" gpurun_out/st.log | grep -E "kth-stamps launch"
done
