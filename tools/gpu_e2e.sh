# The seq drop-in's one-shot cost at the shipped size (n = 1e8, k = 250 and
# k = n/2): apps/kth_seq end to end (HIP runtime + ctx creation, host-to-device
# staging, first-call select) with its --breakdown, beside the reference's own
# shipped program on the same seeded input (KO_TIME seeds its srand(time)).
# Usage: bash tools/gpu_e2e.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-e2e}; O=gpurun_out/$T; mkdir -p $O
B=mpi-k-selection_amd/bin/kth_seq
# plain (the printed time includes the HIP runtime's start), then --breakdown
# (the runtime started before the timed call and timed apart)
for args in "100000000 250 12345" "100000000 0 12345 --median"; do
  for extra in "" "" --breakdown --breakdown; do
    echo "== kth_seq $args $extra" >> $O/kth_seq.out
    timeout -k 10 120 $B $args $extra >> $O/kth_seq.out 2>> $O/kth_seq.err || { echo "kth_seq rc=$?"; tail -5 $O/kth_seq.err; exit 1; }
  done
done
cat $O/kth_seq.out; grep breakdown $O/kth_seq.err
# (the reference's `void main` leaves a garbage exit status: its output line is the check)
for p in seq_shipped seq_median_shipped; do
  ( time KO_TIME=12345 timeout -k 10 200 ./oracle/_ref/$p ) > $O/ref_$p.out 2>&1
  grep -q "Solution found" $O/ref_$p.out || { echo "reference $p failed"; tail -5 $O/ref_$p.out; exit 1; }
  echo "== reference $p"; cat $O/ref_$p.out
done
