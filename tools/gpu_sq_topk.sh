# SQ instruction mix of the select's streaming pass and of the staged top-k
# pass k_main<5> (bench.py --workload topk), per 64-key wave slot, for each
# library variant (base = lib/libkth.so, else lib/variants/libkth_<v>.so).
# Two --pmc passes of 8 SQ counters each.  Usage: [K=67108864] gpurun -- bash tools/gpu_sq_topk.sh <tag> <variant>...
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-sqtopk}; shift; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
C1="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES"
C2="SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_BUSY_CYCLES"
K=${K:-67108864}
for v in "$@"; do
  lib=mpi-k-selection_amd/lib/libkth.so; [ $v = base ] || lib=mpi-k-selection_amd/lib/variants/libkth_$v.so
  for p in 1 2; do
    eval C=\$C$p
    KTH_LIB=$PWD/$lib timeout -s KILL 120 rocprofv3 --pmc $C -d $O/${v}_$p -o run --output-format csv -- python3 bench.py --workload topk --k $K --steps 3 --warmup 1 > $O/${v}_$p.log 2>&1 || { echo "pmc $v $p rc=$?"; tail -20 $O/${v}_$p.log; exit 1; }
    python3 tools/sq_mix.py $O/${v}_$p "k_main<" $((1 << 30)) "$v k=$K k_main pass $p"
  done
done
