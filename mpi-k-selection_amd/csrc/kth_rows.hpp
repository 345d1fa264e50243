// kth_rows.hpp -- batched per-row k-th selection (BASELINE config 5: rows x
// cols int32/float32, the top-k / MoE-routing shape), one wavefront per row.
//
// Lane l of a wave holds keys l*4 + 256*j + {0..3} of its row (16-byte
// coalesced loads: one KiB per wave-instruction) as order-preserving u32 in
// registers; the tail past `cols` is padded with 0xFFFFFFFF, which is exact
// for any k <= cols (padding sorts last, and a valid key equal to it is the
// same value).  Four 8-bit radix digits, each from a wave-private 256-bin LDS
// histogram of the keys still matching the prefix; lane l owns bins
// 4l..4l+3, and one wave scan of the per-lane sums plus a ballot picks the
// digit.  The first pass counts into R0 histogram copies (lane % R0 picks
// one; a 257-word copy stride puts a bin's copies in different banks): on
// skewed rows -- float keys of uniform(-1, 1) share a handful of exponent
// bytes -- a whole wave-instruction lands on one bin, and LDS atomics on one
// address serialise.  Later passes see few keys and use one copy.  Waves never
// wait for each other (no barriers); a pass whose picked bin holds a single
// key ends the row early.  Four waves (rows) per 256-thread workgroup,
// grid-strided.  Included by kth_kernels.hip.
#pragma once

namespace kth {

constexpr int RW_BLOCK = 256;
constexpr int RW_BINS = 256;
constexpr int RW_STRIDE = RW_BINS + 1;  // words between histogram copies

// Raw bits of a key (inverse of the order-preserving transform).
template <bool F32>
__device__ __forceinline__ uint32_t raw_of_key(uint32_t key) {
    return F32 ? f32_of_key(key) : (uint32_t)i32_of_key(key);
}

// TOPK = false: out[r] = the k-th smallest of row r.
// TOPK = true: vals[r*k ..] / idx[r*k ..] = the k smallest keys of row r and
// their columns, in column order; of the keys equal to the k-th, the first
// ones by column.  flip = 0xFFFFFFFF selects the k largest instead (the key
// order reversed: ~key).
template <bool F32, int KPL, bool VEC, int R0, bool TOPK>
__global__ __launch_bounds__(RW_BLOCK) void k_rows_reg(const uint32_t *__restrict__ m, u64 rows, uint32_t cols,
                                                      uint32_t k, uint32_t *__restrict__ out, uint32_t flip,
                                                      uint32_t *__restrict__ vals, int32_t *__restrict__ idx) {
    static_assert(KPL % 4 == 0, "16-byte loads");
    __shared__ uint32_t hist_all[RW_BLOCK / WAVE][R0 * RW_STRIDE];
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    uint32_t *hist = hist_all[wid];
    const u64 wave0 = (u64)blockIdx.x * (RW_BLOCK / WAVE) + wid, nwaves = (u64)gridDim.x * (RW_BLOCK / WAVE);
    for (u64 r = wave0; r < rows; r += nwaves) {  // wave-uniform
        const uint32_t *row = m + r * (u64)cols;
        uint32_t key[KPL];
#pragma unroll
        for (int j = 0; j < KPL / 4; ++j) {
            const uint32_t e = (uint32_t)(j * WAVE + lane) * 4u;  // first element of this lane's vector j
            uint4 x;
            if (VEC) {
                x = e < cols ? load_nt(reinterpret_cast<const uint4 *>(row + e)) : make_uint4(0u, 0u, 0u, 0u);
            } else {
                x.x = e + 0 < cols ? row[e + 0] : 0u;
                x.y = e + 1 < cols ? row[e + 1] : 0u;
                x.z = e + 2 < cols ? row[e + 2] : 0u;
                x.w = e + 3 < cols ? row[e + 3] : 0u;
            }
            const uint32_t v[4] = {x.x, x.y, x.z, x.w};
#pragma unroll
            for (int q = 0; q < 4; ++q)
                key[4 * j + q] = e + q < cols ? ((F32 ? key_of_f32(v[q]) : key_of_i32(v[q])) ^ flip) : 0xFFFFFFFFu;
        }
        uint32_t prefix = 0, kk = k, answer = 0;
        bool found = false;
        for (int pass = 0; pass < 4; ++pass) {  // wave-uniform
            const int shift = 24 - 8 * pass;
            const uint32_t pmask = pass ? 0xFFFFFFFFu << (32 - 8 * pass) : 0u;
            const int copies = pass ? 1 : R0;
            for (int i = lane; i < copies * RW_STRIDE; i += WAVE) hist[i] = 0;
            __builtin_amdgcn_wave_barrier();
            uint32_t *mine = hist + (pass ? 0 : (lane % R0) * RW_STRIDE);
#pragma unroll
            for (int j = 0; j < KPL; ++j)
                if ((key[j] & pmask) == prefix) atomicAdd(&mine[(key[j] >> shift) & 0xFFu], 1u);
            __builtin_amdgcn_wave_barrier();
            uint32_t h[4] = {0u, 0u, 0u, 0u};  // bins 4*lane .. 4*lane + 3, summed over the copies
            for (int c = 0; c < copies; ++c) {
                const uint32_t *b = hist + c * RW_STRIDE + 4 * lane;
#pragma unroll
                for (int q = 0; q < 4; ++q) h[q] += b[q];
            }
            const uint32_t sum = h[0] + h[1] + h[2] + h[3];
            uint32_t incl = sum;
#pragma unroll
            for (int o = 1; o < WAVE; o <<= 1) {
                const uint32_t y = __shfl_up(incl, o, WAVE);
                if (lane >= o) incl += y;
            }
            const uint32_t excl = incl - sum;
            const unsigned long long bm = __ballot(kk > excl && kk <= incl);
            const int L = bm ? __ffsll((long long)bm) - 1 : 0;
            uint32_t bin = 0, below = excl, cnt = 0;
            if (lane == L) {
                bool f = false;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (!f && below + h[q] >= kk) {
                        bin = (uint32_t)(4 * L + q);
                        cnt = h[q];
                        f = true;
                    } else if (!f) {
                        below += h[q];
                    }
                }
            }
            bin = __shfl(bin, L, WAVE);
            below = __shfl(below, L, WAVE);
            cnt = __shfl(cnt, L, WAVE);
            kk -= below;
            prefix |= bin << shift;
            if (cnt == 1 && pass < 3) {  // the single key with this prefix is the answer
                const uint32_t nmask = 0xFFFFFFFFu << shift;
                uint32_t val = 0;
                bool have = false;
#pragma unroll
                for (int j = 0; j < KPL; ++j)
                    if (!have && (key[j] & nmask) == prefix) {
                        val = key[j];
                        have = true;
                    }
                const unsigned long long hm = __ballot(have);
                answer = __shfl(val, __ffsll((long long)hm) - 1, WAVE);
                found = true;
                break;
            }
            __builtin_amdgcn_wave_barrier();  // the next zeroing after every lane's histogram reads
        }
        if (!found) answer = prefix;
        if (!TOPK) {
            if (lane == 0) out[r] = raw_of_key<F32>(answer ^ flip);
        } else {
            // Compaction in column order.  Group j holds columns (64*j + lane)*4 + q:
            // lane-major, then q.  For each q a ballot of the selected keys and
            // mbcnt (set bits in lower lanes) give every key its position: the
            // keys selected before it = taken + sum_q mbcnt(ballot_q) + those of
            // its own lane with a smaller q.  Ties: the keys equal to the k-th are
            // ranked by column the same way, and the first kk of them are taken.
            uint32_t taken = 0, eq_seen = 0;
            const u64 obase = r * (u64)k;
            const bool stage = 2 * k <= (uint32_t)(R0 * RW_STRIDE);  // fits the wave's histogram words
            auto below_lane = [](unsigned long long b) {  // set bits of b in lanes below this one
                return __builtin_amdgcn_mbcnt_hi((uint32_t)(b >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)b, 0u));
            };
#pragma unroll
            for (int j = 0; j < KPL / 4; ++j) {
                const uint32_t e = (uint32_t)(j * WAVE + lane) * 4u;
                bool lt[4], eq[4], sel[4];
                uint32_t eq_below = 0, eq_tot = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool valid = e + q < cols;
                    lt[q] = valid && key[4 * j + q] < answer;
                    eq[q] = valid && key[4 * j + q] == answer;
                    const unsigned long long be = __ballot(eq[q]);
                    eq_below += below_lane(be);
                    eq_tot += (uint32_t)__popcll(be);
                }
                uint32_t rank = eq_seen + eq_below;  // tie rank of this lane's first equal key
                uint32_t pos = taken, tot = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    sel[q] = lt[q] || (eq[q] && rank < kk);
                    rank += eq[q] ? 1u : 0u;
                    const unsigned long long bs = __ballot(sel[q]);
                    pos += below_lane(bs);
                    tot += (uint32_t)__popcll(bs);
                }
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    if (sel[q]) {
                        const uint32_t x = raw_of_key<F32>(key[4 * j + q] ^ flip);
                        if (stage) {  // the histogram is free now: stage (value, column) pairs
                            hist[2 * pos] = x;
                            hist[2 * pos + 1] = e + q;
                        } else {
                            if (vals) vals[obase + pos] = x;
                            if (idx) idx[obase + pos] = (int32_t)(e + q);
                        }
                        ++pos;
                    }
                taken += tot;
                eq_seen += eq_tot;
                __builtin_amdgcn_sched_barrier(0);  // keep the groups apart: no hoisting across them (VGPRs)
            }
            if (stage) {  // coalesced copy-out of the staged pairs
                __builtin_amdgcn_wave_barrier();
                for (uint32_t i = lane; i < k; i += WAVE) {
                    if (vals) vals[obase + i] = hist[2 * i];
                    if (idx) idx[obase + i] = (int32_t)hist[2 * i + 1];
                }
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
}

}  // namespace kth
