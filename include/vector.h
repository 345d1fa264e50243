/*
 * vector.h -- ABI twin of the reference's IntVector (vector.h:7-33).
 *
 * Same struct layout ({int size; int capacity; int *data;}, 16 bytes on LP64)
 * and the same 17 prototypes, so that the reference drivers
 * (kth-problem-seq.c, TODO-kth-problem-cgm.c) compile and link unmodified
 * against libkth.so.  Implementation: mpi-k-selection_amd/csrc/vector.c.
 *
 * Deliberate differences from /root/reference/vector.c (each a reference
 * defect):
 *   - VecQuickSort / VecBinarySearch compare with (a > b) - (a < b) instead of
 *     `*a - *b` (vector.c:6-8 overflows for keys more than INT_MAX apart).
 *   - VecQuickSort2 sorts with the same comparator (the reference's hand-written
 *     quicksort, vector.c:10-50, is O(n^2) and recurses n deep on equal keys).
 *   - MaxFind and VecBinarySearch2 check for NULL before dereferencing
 *     (vector.c:146, :268).
 *   - VecAdd's capacity doubling is computed in size_t (vector.c:81 overflows
 *     in int for capacity >= 2^29).
 *   Kept as in the reference: VecGet/VecSet/VecErase in-band sentinels, and
 *   AverageFind returning the SUM (vector.c:162-171), so callers see the same
 *   values.
 *
 * Added: VecKthSelect -- the drop-in for the select block
 *     VecQuickSort(pVec); solution = VecGet(pVec, k - 1);   (kth-problem-seq.c:32-33)
 * computed on the GPU by kth_select_i32 (include/kth.h) without sorting.
 */
#ifndef _VECTOR_H
#define _VECTOR_H

#define TRUE 1
#define FALSE 0

typedef struct {
    int size;     /* number of elements */
    int capacity; /* allocated elements */
    int *data;    /* elements           */
} IntVector, *IntVectorPtr;

#ifdef __cplusplus
extern "C" {
#endif

IntVectorPtr VecNew(int initialCapacity);
int VecAdd(IntVectorPtr vector, int element);
void VecDelete(IntVectorPtr vector);
int VecErase(IntVectorPtr vector, int position);
int MinFind(IntVectorPtr vector);
int MaxFind(IntVectorPtr vector);
double AverageFind(IntVectorPtr vector);
int VecGetCapacity(IntVectorPtr vector);
int VecGetSize(IntVectorPtr vector);
int VecIsFull(IntVectorPtr vector);
int VecSet(IntVectorPtr vector, int position, int element);
int VecGet(IntVectorPtr vector, int position);
int VecSearch(IntVectorPtr vector, int startPos, int element);

void VecQuickSort(IntVectorPtr vector);
void VecQuickSort2(IntVectorPtr vector);

int VecBinarySearch(IntVectorPtr vector, int element);
int VecBinarySearch2(IntVectorPtr vector, int element);

/* k-th smallest (1-based k) of the vector's elements, on the GPU; the vector
 * is not modified.  VecGet-style in-band sentinels: -1 if vector or data is
 * NULL, -2 if k is out of [1, size] (vector.c:209-218), -3 on a device error.
 * Equivalent to `VecQuickSort(v); VecGet(v, k - 1)` (kth-problem-seq.c:32-33). */
int VecKthSelect(IntVectorPtr vector, int k);

/* Same with an explicit status (0 or a KTH_E* code) and the value in *out. */
int VecKthSelectEx(IntVectorPtr vector, int k, int *out);

#ifdef __cplusplus
}
#endif
#endif /* _VECTOR_H */
