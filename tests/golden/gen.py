"""Synthetic key families, numpy edition.

Bit-for-bit the same as ``ko_gen`` (oracle/kth_oracle.c) and the device
generator ``kth_fill_synthetic`` (include/kth.h); tests pin all three against
each other.  Counter-based (splitmix64 of the global index), so any shard of an
input can be generated independently of the others.
"""
import numpy as np

UNIFORM_FULL, UNIFORM_HALF, UNIFORM_REF, ALL_EQUAL, FEW_DISTINCT, SORTED_ASC, SORTED_DESC, MOD_1000 = range(8)
NAMES = {
    UNIFORM_FULL: "uniform_full",
    UNIFORM_HALF: "uniform_half",
    UNIFORM_REF: "uniform_ref",
    ALL_EQUAL: "all_equal",
    FEW_DISTINCT: "few_distinct",
    SORTED_ASC: "sorted_asc",
    SORTED_DESC: "sorted_desc",
    MOD_1000: "mod_1000",
}
BY_NAME = {v: k for k, v in NAMES.items()}
FEW = np.array([-5, 0, 7, 123456789], dtype=np.int32)
DEFAULT_SEED = 0x5EED0001

_G = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def hash64(seed, idx):
    """splitmix64(seed + (i + 1) * golden) for a uint64 index array."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (idx.astype(np.uint64) + np.uint64(1)) * _G
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        return z ^ (z >> np.uint64(31))


def gen(n, dist, seed=DEFAULT_SEED, param=0, offset=0, n_total=None, chunk=1 << 24):
    """Keys for global indices [offset, offset+n) of an input of n_total keys."""
    if n_total is None:
        n_total = offset + n
    out = np.empty(n, dtype=np.int32)
    step = 1
    if 0 < n_total <= 0xFFFFFFFF:
        step = max(1, min(0xFFFFFFFF, (1 << 32) // n_total))
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        i = np.arange(offset + s, offset + e, dtype=np.uint64)
        h = hash64(seed, i)
        hi = (h >> np.uint64(32)).astype(np.uint32)
        if dist == UNIFORM_FULL:
            v = hi.view(np.int32)
        elif dist == UNIFORM_HALF:
            v = hi.view(np.int32) >> 1
        elif dist == UNIFORM_REF:
            v = (hi % np.uint32(99999999)).astype(np.int32) + 1
        elif dist == ALL_EQUAL:
            v = np.full(e - s, param, dtype=np.int32)
        elif dist == FEW_DISTINCT:
            v = FEW[(h >> np.uint64(62)).astype(np.int64)]
        elif dist == SORTED_ASC:
            with np.errstate(over="ignore"):
                v = (np.uint32(0x80000000) + i.astype(np.uint32) * np.uint32(step)).view(np.int32)
        elif dist == SORTED_DESC:
            with np.errstate(over="ignore"):
                v = (np.uint32(0x7FFFFFFF) - i.astype(np.uint32) * np.uint32(step)).view(np.int32)
        elif dist == MOD_1000:
            v = (hi % np.uint32(1000)).astype(np.int32)
        else:
            raise ValueError(dist)
        out[s:e] = v
    return out


def kth_true(a, k):
    """k-th smallest (1-based) by numpy partition -- used only as a cross-check."""
    return int(np.partition(a, k - 1)[k - 1])
