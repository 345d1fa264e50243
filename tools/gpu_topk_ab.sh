# A/B of top-k library variants: whole-call times (bench.py --workload topk)
# for each k, then rocprof kernel averages at the largest k.
# Usage: VARIANTS="a b" KS="134217728 536870912" bash tools/gpu_topk_ab.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-topk_ab}; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
# DIAG_OK=1: diagnostic variants (wrong results by design) may fail verification (bench rc 1)
# a variant is a library (lib/variants/libkth_<v>.so) or env:NAME=VALUE (the base library under that setting)
varlib() { e=""; f=${1//[:=]/_}; lib=mpi-k-selection_amd/lib/variants/libkth_$1.so
  case $1 in base) lib=mpi-k-selection_amd/lib/libkth.so ;; env:*) lib=mpi-k-selection_amd/lib/libkth.so; e=${1#env:} ;; esac; }
for v in base $VARIANTS; do
  varlib $v
  for k in ${KS:-67108864 134217728 536870912}; do
    ( [ -z "$e" ] || export "$e"; KTH_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --workload topk --k $k --steps 10 --warmup 3 --no-cpu-baseline >> $O/$f.jsonl 2>$O/$f.err ) || { rc=$?; [ "$DIAG_OK.$rc" = "1.1" ] || { echo "$v k=$k rc=$rc"; tail -20 $O/$f.err; exit 1; }; }
  done
  python3 -c "
import json
for l in open('$O/$f.jsonl'):
    d = json.loads(l); print('$v', 'k', d['config']['k'], round(d['ms_per_step'], 3), 'ms', round(d['value'], 1), 'Gkeys/s', 'verified', d['verified'])"
done
for v in base $VARIANTS; do
  varlib $v
  for k in ${PROF_KS:-134217728 536870912}; do
    ( [ -z "$e" ] || export "$e"; KTH_LIB=$PWD/$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_${f}_$k -o run --output-format csv -- python3 bench.py --workload topk --k $k --steps 5 --warmup 2 > $O/prof_${f}_$k.log 2>&1 ) || { rc=$?; [ "$DIAG_OK.$rc" = "1.1" ] || { echo "prof $v rc=$rc"; tail -5 $O/prof_${f}_$k.log; exit 1; }; }
    echo "== $v k=$k"; python3 tools/prof_summary.py $O/prof_${f}_$k/run_kernel_trace.csv 0 | head -8
  done
done
