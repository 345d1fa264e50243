# Round 4: k_head phase stamps, the select (median) against top-k k = 1024
# (k_head ~24 us under top-k, ~13 us in the select)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4head; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
L=$PWD/mpi-k-selection_amd/lib/variants/libkth_stamps.so
KTH_LIB=$L KTH_STAMPS=1 timeout -k 10 120 python -u bench.py --steps 3 --warmup 2 --no-cpu-baseline > $O/sel.log 2> $O/sel.err || { echo rc=$?; tail -20 $O/sel.err; exit 1; }
KTH_LIB=$L KTH_STAMPS=1 timeout -k 10 120 python -u bench.py --workload topk --k 1024 --steps 3 --warmup 2 --no-cpu-baseline > $O/tk.log 2> $O/tk.err || { echo rc=$?; tail -20 $O/tk.err; exit 1; }
echo "== select"; grep "kth-stamps" $O/sel.err | tail -30
echo "== topk"; grep "kth-stamps" $O/tk.err | tail -30
