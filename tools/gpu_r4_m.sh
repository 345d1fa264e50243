# Round 4 (m): output stores of the rows kernels: non-temporal top-k stores
# (ntstore) and a timing-only k-th build without its per-row store (dnoout)
set -o pipefail
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4m; rm -rf $O; mkdir -p $O; export TMPDIR=/tmp
L=mpi-k-selection_amd/lib
one() {  # lib args
  KTH_LIB=$1 timeout -k 10 120 python -u bench.py --workload rows $2 --k 64 --steps 20 --warmup 3 --no-cpu-baseline > $O/rows.log 2>&1; rc=$?
  [ $rc -le 1 ] || { echo "bench rc=$rc"; tail -20 $O/rows.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/rows.log').read().strip().splitlines()[-1]); r=d['roofline']; print('$(basename $1)', '$2', round(d['value'],1), 'Gkeys/s kernel', round(r['avg_launch_ms']*1e3,1), 'us', d['verified'])"
}
for rep in 1 2; do
  for lib in $L/libkth.so $L/variants/libkth_dnoout.so; do one $lib "--rows-dtype i32" || exit 1; one $lib "--rows-dtype f32" || exit 1; done
  for lib in $L/libkth.so $L/variants/libkth_ntstore.so; do one $lib "--rows-dtype i32 --topk" || exit 1; one $lib "--rows-dtype f32 --topk" || exit 1; done
done
echo done
