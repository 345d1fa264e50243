/*
 * vector.c -- IntVector, the reference's host container (vector.h:7-33,
 * vector.c:1-287), re-implemented for libkth.so.  Differences from the
 * reference are listed in include/vector.h.
 */
#include "vector.h"

#include <stdint.h>
#include <stdlib.h>

#include "kth.h"

/* Overflow-free order; the reference's `*a - *b` (vector.c:6-8) is not. */
static int cmp_int(const void *x, const void *y)
{
    int a = *(const int *)x, b = *(const int *)y;
    return (a > b) - (a < b);
}

IntVectorPtr VecNew(int initialCapacity)
{
    if (initialCapacity < 0)
        return NULL;
    IntVectorPtr v = (IntVectorPtr)malloc(sizeof(IntVector));
    if (!v)
        return NULL;
    /* malloc(0) may return NULL; keep data non-NULL so accessors work */
    v->data = (int *)malloc((size_t)(initialCapacity > 0 ? initialCapacity : 1) * sizeof(int));
    if (!v->data) {
        free(v);
        return NULL;
    }
    v->size = 0;
    v->capacity = initialCapacity;
    return v;
}

int VecAdd(IntVectorPtr v, int element)
{
    if (!v || !v->data)
        return -1;
    if (v->size >= v->capacity) {
        size_t cap = v->capacity > 0 ? (size_t)v->capacity * 2 : 1;
        if (cap > (size_t)INT32_MAX)
            cap = (size_t)INT32_MAX;
        if (cap <= (size_t)v->size)
            return -1;
        int *nd = (int *)realloc(v->data, cap * sizeof(int));
        if (!nd)
            return -1;
        v->data = nd;
        v->capacity = (int)cap;
    }
    v->data[v->size] = element;
    return v->size++;
}

void VecDelete(IntVectorPtr v)
{
    if (v) {
        free(v->data);
        free(v);
    }
}

int VecErase(IntVectorPtr v, int position)
{
    if (!v || !v->data || v->size == 0)
        return -1;
    if (position < 0 || position >= v->size)
        return -1;
    /* O(1): move the last element into the hole (vector.c:114-119) */
    v->data[position] = v->data[--v->size];
    return position;
}

int MinFind(IntVectorPtr v)
{
    if (!v || !v->data)
        return -1;
    int m = v->data[0];
    for (int i = 1; i < v->size; i++)
        if (v->data[i] < m)
            m = v->data[i];
    return m;
}

int MaxFind(IntVectorPtr v)
{
    if (!v || !v->data)
        return -1;
    int m = v->data[0];
    for (int i = 1; i < v->size; i++)
        if (v->data[i] > m)
            m = v->data[i];
    return m;
}

double AverageFind(IntVectorPtr v)
{
    /* The reference returns the sum, not the mean (vector.c:162-171); kept so
     * callers observe the same value. */
    double s = 0;
    if (!v || !v->data)
        return 0;
    for (int i = 0; i < v->size; ++i)
        s += v->data[i];
    return s;
}

int VecGetCapacity(IntVectorPtr v)
{
    if (!v || !v->data)
        return -1;
    return v->capacity;
}

int VecGetSize(IntVectorPtr v)
{
    if (!v || !v->data)
        return -1;
    return v->size;
}

int VecIsFull(IntVectorPtr v)
{
    if (!v || !v->data)
        return TRUE;
    return v->size == v->capacity ? TRUE : FALSE;
}

int VecSet(IntVectorPtr v, int position, int element)
{
    if (!v || !v->data)
        return -1;
    if (position >= v->size || position < 0)
        return -2;
    v->data[position] = element;
    return element;
}

int VecGet(IntVectorPtr v, int position)
{
    if (!v || !v->data)
        return -1;
    if (position >= v->size || position < 0)
        return -2;
    return v->data[position];
}

int VecSearch(IntVectorPtr v, int startPos, int element)
{
    if (!v || !v->data)
        return -1;
    if (startPos >= v->size)
        return -1;
    if (startPos < 0)
        startPos = 0;
    for (int i = startPos; i < v->size; i++)
        if (v->data[i] == element)
            return i;
    return -1;
}

void VecQuickSort(IntVectorPtr v)
{
    if (v && v->data && v->size > 1)
        qsort(v->data, (size_t)v->size, sizeof(int), cmp_int);
}

void VecQuickSort2(IntVectorPtr v)
{
    VecQuickSort(v);
}

int VecBinarySearch(IntVectorPtr v, int element)
{
    if (!v || !v->data || v->size <= 0)
        return -1;
    int *p = (int *)bsearch(&element, v->data, (size_t)v->size, sizeof(int), cmp_int);
    return p ? (int)(p - v->data) : -1;
}

int VecBinarySearch2(IntVectorPtr v, int element)
{
    if (!v || !v->data)
        return -1;
    int beg = 0, end = v->size - 1;
    while (beg <= end) {
        int mid = beg + (end - beg) / 2;
        if (v->data[mid] == element)
            return mid;
        if (element < v->data[mid])
            end = mid - 1;
        else
            beg = mid + 1;
    }
    /* like the reference (vector.c:286), fall back to a linear scan so an
     * unsorted vector still finds the element */
    return VecSearch(v, 0, element);
}

int VecKthSelectEx(IntVectorPtr v, int k, int *out)
{
    if (!v || !v->data || !out)
        return KTH_EINVAL;
    if (k < 1 || k > v->size)
        return KTH_EINVAL;
    int32_t r = 0;
    int rc = kth_select_i32((const int32_t *)v->data, (int64_t)v->size, (int64_t)k, &r);
    if (rc == KTH_OK)
        *out = (int)r;
    return rc;
}

int VecKthSelect(IntVectorPtr v, int k)
{
    if (!v || !v->data)
        return -1;
    if (k < 1 || k > v->size)
        return -2;
    int r = 0;
    return VecKthSelectEx(v, k, &r) == KTH_OK ? r : -3;
}
