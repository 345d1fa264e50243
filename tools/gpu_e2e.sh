# The seq drop-in's one-shot cost at the shipped size (n = 1e8, k = 250 and
# k = n/2): apps/kth_seq end to end (HIP runtime + ctx creation, host-to-device
# staging, first-call select) with its --breakdown, beside the reference's own
# shipped program on the same seeded input (KO_TIME seeds its srand(time)).
# Usage: bash tools/gpu_e2e.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"; T=${1:-e2e}; O=gpurun_out/$T; mkdir -p $O
B=mpi-k-selection_amd/bin/kth_seq
for args in "100000000 250 12345" "100000000 0 12345 --median"; do
  for i in 1 2; do
    timeout -k 10 120 $B $args --breakdown >> $O/kth_seq.out 2>> $O/kth_seq.err || { echo "kth_seq rc=$?"; tail -5 $O/kth_seq.err; exit 1; }
  done
done
cat $O/kth_seq.out; grep breakdown $O/kth_seq.err
( time KO_TIME=12345 timeout -k 10 200 ./oracle/_ref/seq_shipped ) > $O/ref_seq.out 2>&1 || { echo "ref rc=$?"; tail -5 $O/ref_seq.out; exit 1; }
( time KO_TIME=12345 timeout -k 10 200 ./oracle/_ref/seq_median_shipped ) > $O/ref_seq_median.out 2>&1 || { echo "ref median rc=$?"; tail -5 $O/ref_seq_median.out; exit 1; }
cat $O/ref_seq.out $O/ref_seq_median.out
