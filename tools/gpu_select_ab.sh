# A/B of select library variants on the driver's bench command, interleaved
# (base, v1, .., base, v1, ..) ROUNDS times to average out box drift.  A
# variant is a library (lib/variants/libkth_<v>.so) or env:NAME=VALUE (the
# base library under that environment setting).
# Usage: VARIANTS="a env:KTH_X=0" ROUNDS=3 bash tools/gpu_select_ab.sh <tag> [bench args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-select_ab}; shift; O=gpurun_out/$T; mkdir -p $O; export TMPDIR=/tmp
for i in $(seq 1 ${ROUNDS:-3}); do
  for v in base $VARIANTS; do
    lib=mpi-k-selection_amd/lib/variants/libkth_$v.so; e=""
    case $v in base) lib=mpi-k-selection_amd/lib/libkth.so ;; env:*) lib=mpi-k-selection_amd/lib/libkth.so; e=${v#env:} ;; esac
    f=${v//[:=]/_}
    env $e KTH_LIB=$PWD/$lib timeout -k 10 120 python -u bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" >> $O/$f.jsonl 2>>$O/$f.err || { echo "$v rc=$?"; tail -20 $O/$f.err; exit 1; }
  done
done
for v in base $VARIANTS; do
  f=${v//[:=]/_}
  python3 -c "
import json
v = [json.loads(l) for l in open('$O/$f.jsonl') if l.startswith('{')]
print('$v', ' '.join('%.1f' % d['value'] for d in v), 'Gkeys/s; ms', ' '.join('%.4f' % d['ms_per_step'] for d in v), 'verified', all(d['verified'] for d in v))"
done
