# A/B of library variants on the rows workloads (BASELINE config 5, 65536 x 4096):
# one bench line per (variant, workload), variants interleaved per workload.
# Usage: VARIANTS="r5" [ROUNDS=2] gpurun -- bash tools/gpu_rows_ab.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-rows_ab}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
W=${WORKLOADS:-"--rows-dtype|f32|--rows-input|dup|--k|2048 --rows-dtype|f32|--rows-input|dup|--k|64 --rows-dtype|i32|--k|64 --rows-dtype|f32|--k|64 --rows-dtype|i32|--topk|--k|64 --rows-dtype|f32|--topk|--k|64"}
for r in $(seq 1 ${ROUNDS:-2}); do
for w in $W; do
  args=${w//|/ }
  for v in base $VARIANTS; do
    lib=mpi-k-selection_amd/lib/libkth.so; [ $v = base ] || lib=mpi-k-selection_amd/lib/variants/libkth_$v.so
    KTH_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --workload rows $args --steps 20 --warmup 3 > $O/run.log 2>&1; rc=$?
    [ $rc -le 1 ] || { echo "$v $args rc=$rc"; tail -20 $O/run.log; exit 1; }
    tail -1 $O/run.log >> $O/$v.jsonl
    python3 -c "import json; d=json.loads(open('$O/run.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$v', '$args', round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us', d['verified'])"
  done
done
done
