# Round 4 (l): where top-k rows spend their time: timing-only builds without the
# staging pass (dnostage), without the list / rank / copy-out tail (dnotail),
# without both (dboth), against the default build.  Diagnostic builds give wrong
# results (verified false); only their kernel times are read.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4l; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
L=mpi-k-selection_amd/lib
for rep in 1 2; do
for lib in $L/libkth.so $L/variants/libkth_dnostore.so $L/variants/libkth_tkw5.so $L/variants/libkth_dnotail.so; do
  for args in "--rows-dtype i32 --topk" "--rows-dtype f32 --topk"; do
    KTH_LIB=$lib timeout -k 10 120 python -u bench.py --workload rows $args --k 64 --steps 20 --warmup 3 --no-cpu-baseline > $O/rows.log 2>&1; rc=$?
    [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 $O/rows.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/rows.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$(basename $lib)', '$args', round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us', d['verified'])"
  done
done
done
echo done
