#!/usr/bin/env bash
# build_ref.sh -- compile the REFERENCE programs from their sources where they lie
# under /root/reference into oracle/_ref/ (git-ignored).  TEST INFRASTRUCTURE ONLY.
#
#   _ref/libvector_ref.so   vector.c unmodified (VecQuickSort + VecGet = the seq
#                           select block, kth-problem-seq.c:32-33)
#   _ref/seq_shipped        kth-problem-seq.c  + vector.c, unmodified (n=1e8, k=250)
#   _ref/seq_median_shipped kth-problem-seq.c~ + vector.c, unmodified (k=n/2)
#   _ref/cgm_shipped        TODO-kth-problem-cgm.c  + vector.c, unmodified (n=1e8, k=150)
#   _ref/cgm_median_shipped TODO-kth-problem-cgm.c~ + vector.c, unmodified (k=n/2)
#   _ref/cgm_param          TODO-kth-problem-cgm.c with n and k read from KO_N/KO_K:
#                           the two constant lines (:45, :48) are rewritten by sed in a
#                           pipe straight into the compiler; no copy is written to disk.
# Every program is linked with ref_shim.c (--wrap=time,--wrap=VecAdd) for seeding
# and input replacement; see ref_shim.c.  Needs gcc and MPICH's mpicc.
set -euo pipefail
REF=${REF:-/root/reference}
MPICC=${MPICC:-/opt/conda/bin/mpicc}
HERE=$(cd "$(dirname "$0")" && pwd)
OUT="$HERE/_ref"
if [ ! -f "$REF/vector.c" ]; then
    echo "build_ref: $REF not present; skipping reference build" >&2
    exit 0
fi
mkdir -p "$OUT"
WRAP="-Wl,--wrap=time -Wl,--wrap=VecAdd"
CFLAGS="-O2 -w"

gcc $CFLAGS -fPIC -shared -o "$OUT/libvector_ref.so" "$REF/vector.c"
gcc $CFLAGS -I"$REF" -o "$OUT/seq_shipped" "$REF/kth-problem-seq.c" "$REF/vector.c" "$HERE/ref_shim.c" $WRAP
gcc $CFLAGS -I"$REF" -o "$OUT/seq_median_shipped" -x c "$REF/kth-problem-seq.c~" -x none "$REF/vector.c" "$HERE/ref_shim.c" $WRAP

if [ -x "$MPICC" ]; then
    export MPICH_CC=gcc
    "$MPICC" $CFLAGS -I"$REF" -o "$OUT/cgm_shipped" "$REF/TODO-kth-problem-cgm.c" "$REF/vector.c" "$HERE/ref_shim.c" $WRAP
    "$MPICC" $CFLAGS -I"$REF" -o "$OUT/cgm_median_shipped" -x c "$REF/TODO-kth-problem-cgm.c~" -x none "$REF/vector.c" "$HERE/ref_shim.c" $WRAP
    SED_N='s/const int MAX_NUMBERS = 100000000;/const int MAX_NUMBERS = ko_env_int("KO_N", 100000000);/'
    SED_K='s/int k = 150;/int k = ko_env_int("KO_K", 150);/'
    # both substitutions must hit exactly once
    [ "$(sed -e "$SED_N" -e "$SED_K" "$REF/TODO-kth-problem-cgm.c" | grep -c ko_env_int)" = 2 ] \
        || { echo "build_ref: CGM parameter lines not found" >&2; exit 1; }
    sed -e "$SED_N" -e "$SED_K" "$REF/TODO-kth-problem-cgm.c" \
        | "$MPICC" $CFLAGS -I"$REF" -include "$HERE/ref_shim.h" -o "$OUT/cgm_param" \
            -x c - -x none "$REF/vector.c" "$HERE/ref_shim.c" $WRAP
else
    echo "build_ref: $MPICC missing; CGM reference binaries not built" >&2
fi
echo "build_ref: ok -> $OUT"
