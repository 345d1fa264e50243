"""CPU restatement of the per-rank device steps of the sharded protocol
(kth_dist_* in mpi-k-selection_amd/csrc/kth_api.hip + kth_kernels.hip).

TEST INFRASTRUCTURE ONLY: lets tests/test_dist_gloo.py run the product's
orchestration (kselect.dist.DistSelector) on gloo with world_size > 1 on CPU.
The slot layout, window ranks, decide and digit-pick rules restate the device
code, and the tunable constants (sample size and chunk layout, window z,
candidate capacity) are read from libkth.so itself (kth_dist_sample_size,
kth_sample_chunk, kth_window_z, kth_dist_cand_capacity; no GPU needed), so the
all-reduced slots carry the same numbers a GPU run does --
tests/test_gpu_parity.py::test_dist_backend_slots_match checks that slot by slot.
"""
import math

import numpy as np
import torch

from kselect import LIB

NCOUNTS, DIGIT, NBINS = 8, 11, 2048
STATS_WORDS = NCOUNTS + 2 * NBINS
DDIG, DNB = 12, 4096  # the sharded protocol's candidate / fallback digits (kth_kernels.hip DDIG)
DONE_SLOT = 3  # KTH_DIST_DONE
DIST_FULL_D0 = 32 - 2 * DDIG
C_LT, C_EQLO, C_EQHI, C_IN, C_OVF = range(5)
MAIN, CAND, FULL, DONE = "main", "cand", "full", "done"
WINDOW_Z = float(LIB.kth_window_z())
SAMPLE_CHUNK = int(LIB.kth_sample_chunk())
WINDOW_SLACK64 = int(LIB.kth_window_slack64())
SAMPLE_DIGITS = (11, 11, 10)  # k_head's digits of a 32-bit sample key


def sample_size(n_local):
    return int(LIB.kth_dist_sample_size(int(n_local)))


def window_ranks(n, k, s):
    """kth_api.hip window_ranks: +-(z sigma + 2) around p*s, p = k/n."""
    p = k / n
    r = p * s
    sig = math.sqrt(max(1.0, s * p * (1.0 - p)))
    lo = math.floor(r - WINDOW_Z * sig - 2.0)
    hi = math.ceil(r + WINDOW_Z * sig + 2.0)
    r_lo = 0 if lo < 1.0 else int(lo)
    r_hi = s + 1 if hi > s else int(max(1.0, hi))
    return r_lo, r_hi


def cand_capacity(n):
    return int(LIB.kth_dist_cand_capacity(int(n)))


def cand_domain(lo, hi):
    """kth_kernels.hip cand_domain: keys lo < x < hi as x - base in [0, 2^W),
    base = lo + 1; the first digit d0 bits, the later ones DDIG."""
    base = (lo + 1) & 0xFFFFFFFF
    if hi - lo < 2:
        return base, 0, 0
    W = (hi - lo - 2).bit_length()
    nd = (W + DDIG - 1) // DDIG
    return base, W, W - DDIG * (nd - 1 if nd else 0)


def sample_indices(n_local, s_local):
    """k_gather's layout (include/kth.h kth_sample_chunk): ceil(s/C) chunks of
    C consecutive keys, chunk c at key c * (n / ceil(s/C)); the last chunk holds
    the remaining s mod C keys.  Indices past the shard read as order key 0."""
    C = SAMPLE_CHUNK
    nch = (s_local + C - 1) // C
    stride = n_local // nch
    idx = (np.arange(nch, dtype=np.int64)[:, None] * stride + np.arange(C, dtype=np.int64)[None, :]).ravel()
    return idx[:s_local]


class CpuBackend:
    def __init__(self, cap=None):
        self.cap_override = cap

    # -- allocation (CPU tensors) -----------------------------------------
    def sample_size(self, n_local):
        return sample_size(n_local)

    def alloc_slots(self):
        return torch.zeros((3, STATS_WORDS), dtype=torch.int64)

    def alloc_sample(self, s):
        return torch.empty(s, dtype=torch.int32)

    def alloc_out(self):
        return torch.empty(1, dtype=torch.int32)

    def select_all(self, keys, n, k, out):
        out[0] = int(np.sort(keys.numpy()[:n])[k - 1])

    # -- steps --------------------------------------------------------------
    def begin(self, slots, n_total, k):
        self.slots = slots
        slots.zero_()
        self.n, self.k = n_total, k
        self.mode = None
        self.levels, self.result_slot = None, None

    def sample(self, shard, n_local, out, s_local):
        idx = sample_indices(n_local, s_local)
        ok = idx < n_local
        keys = np.zeros(s_local, dtype=np.uint32)
        keys[ok] = shard.numpy()[idx[ok]].view(np.uint32) ^ np.uint32(0x80000000)
        out.numpy()[:] = keys.view(np.int32)

    def window(self, sample_all, s_total):
        """k_head over the gathered sample (kth_dist_window): the window ranks'
        keys digit by digit; after each digit the window may stop at the picked
        bins' edges when those hold at most WINDOW_SLACK64/64 times the sample
        keys of the exact window (kth_kernels.hip early_window)."""
        r_lo, r_hi = window_ranks(self.n, self.k, s_total)
        srt = np.sort(sample_all.numpy().view(np.uint32))
        a0, a1 = 1 <= r_lo <= s_total, 1 <= r_hi <= s_total
        self.mode = MAIN
        if (a0 or a1) and WINDOW_SLACK64 and s_total % 64 == 0:
            want = (r_hi if a1 else s_total) - (r_lo if a0 else 1) + 1
            done = 0
            for d in SAMPLE_DIGITS[:-1]:  # the last digit resolves the exact keys
                done += d
                sh = np.uint32(32 - done)
                pre = srt >> sh
                p0 = int(srt[r_lo - 1] >> sh) if a0 else 0
                p1 = int(srt[r_hi - 1] >> sh) if a1 else 0
                below0 = int(np.searchsorted(pre, np.uint32(p0), side="left")) if a0 else 0
                upto1 = int(np.searchsorted(pre, np.uint32(p1), side="right")) if a1 else s_total
                if upto1 >= below0 and (upto1 - below0) * 64 <= want * WINDOW_SLACK64:
                    w = 32 - done
                    self.lo = p0 << w if a0 else 0
                    self.hi = ((p1 << w) | ((1 << w) - 1)) if a1 else 0xFFFFFFFF
                    return
        self.lo = int(srt[r_lo - 1]) if a0 else 0
        self.hi = int(srt[r_hi - 1]) if a1 else 0xFFFFFFFF

    def scan(self, shard, n_local):
        """k_main<0> (counts, candidates) + k_dscan_hist (the candidates'
        first digit into the same slot)."""
        u = shard.numpy()[:n_local].view(np.uint32) ^ np.uint32(0x80000000)
        lo, hi = np.uint32(self.lo), np.uint32(self.hi)
        inside = (u > lo) & (u < hi)
        self.cand = u[inside]
        cap = self.cap_override or cand_capacity(max(n_local, 1))
        s0 = self.slots[0]
        s0[C_LT] = int((u < lo).sum())
        s0[C_EQLO] = int((u == lo).sum())
        s0[C_EQHI] = int((u == hi).sum())
        s0[C_IN] = int(inside.sum())
        s0[C_OVF] = 1 if self.cand.size > cap else 0
        self.keys = u
        base, W, d0 = cand_domain(self.lo, self.hi)
        if W and self.cand.size:
            v = (self.cand[:cap].astype(np.uint64) - np.uint64(base)) & np.uint64(0xFFFFFFFF)
            bins = (v >> np.uint64(W - d0)) & np.uint64((1 << d0) - 1)
            s0[NCOUNTS:NCOUNTS + DNB] = torch.from_numpy(np.bincount(bins.astype(np.int64), minlength=DNB))
        return 0

    def _decide(self, c):
        """kth_kernels.hip decide_dist."""
        L, E1, E2r, M, ovf = (int(x) for x in c[:5])
        E2 = 0 if self.lo == self.hi else E2r
        k = self.k
        self.base, self.W, self.d0, self.prefix, self.done, self.kr = 0, 32, 0, 0, 0, k
        if L < k <= L + E1:
            self.mode, self.answer = DONE, self.lo
        elif L + E1 < k <= L + E1 + M and ovf == 0:
            self.base, self.W, self.d0 = cand_domain(self.lo, self.hi)
            self.kr = k - L - E1
            self.mode = CAND
            if self.W == 0:
                self.mode, self.answer = DONE, self.base
        elif L + E1 + M < k <= L + E1 + M + E2:
            self.mode, self.answer = DONE, self.hi
        else:
            self.mode, self.d0 = FULL, DIST_FULL_D0
        self.path = "fallback" if self.mode == FULL else "window"

    def _live(self):
        return self.mode in (CAND, FULL) and self.done < self.W

    def _digit(self):
        return min(self.d0 if self.done == 0 else DDIG, self.W - self.done)

    def _pick(self, slot):
        if not self._live():
            return
        d = self._digit()
        h = slot[NCOUNTS:NCOUNTS + DNB].numpy()
        cum = np.cumsum(h)
        b = int(np.searchsorted(cum, self.kr, side="left"))
        assert b < (1 << d), "histogram holds fewer than k keys"
        below = int(cum[b - 1]) if b else 0
        self.kr -= below
        self.prefix = (self.prefix << d) | b
        self.done += d
        if self.done == self.W:
            self.mode, self.answer = DONE, (self.base + self.prefix) & 0xFFFFFFFF

    def _hist(self, slot):
        slot.zero_()
        if not self._live():
            return
        dom = self.cand if self.mode == CAND else self.keys
        v = (dom.astype(np.uint64) - np.uint64(self.base)) & np.uint64(0xFFFFFFFF)
        d = self._digit()
        if self.done:
            v = v[(v >> np.uint64(self.W - self.done)) == np.uint64(self.prefix)]
        bins = (v >> np.uint64(self.W - self.done - d)) & np.uint64((1 << d) - 1)
        slot[NCOUNTS:NCOUNTS + DNB] = torch.from_numpy(np.bincount(bins.astype(np.int64), minlength=DNB))

    def level(self, shard, n_local, level):
        """k_dlevel: level 0 decides and picks the first digit from the scan's
        slot, and counts the level calls that return a slot (DistStatus);
        later levels pick; each histograms the next digit; KTH_DIST_DONE once
        no digit is left."""
        U = self.slots
        if level >= 1 and level >= self.levels:
            self.result_slot = level % 3
            return DONE_SLOT
        src, acc = U[level % 3], U[(level + 1) % 3]
        if level == 0:
            self._decide(src)
            if self.mode == CAND:
                self._pick(src)
        else:
            self._pick(src)
        if level == 0:
            left = self.W - self.done - self._digit() if self._live() else 0
            self.levels = 1 + (left + DDIG - 1) // DDIG
        self._hist(acc)
        return (level + 1) % 3

    def result(self, out):
        self._pick(self.slots[self.result_slot])
        assert self.mode == DONE, self.mode
        out[0] = int(np.uint32(self.answer ^ 0x80000000).view(np.int32))
