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
#ifndef KTH_TOPK_RELOAD
#define KTH_TOPK_RELOAD 1
#endif
constexpr bool TOPK_RELOAD = KTH_TOPK_RELOAD;  // top-k compaction re-reads full rows from L2
#ifndef KTH_TOPK_KEYS_COMPACT
#define KTH_TOPK_KEYS_COMPACT 1
#endif
constexpr bool TOPK_KEYS_COMPACT = KTH_TOPK_KEYS_COMPACT;  // unstaged full top-k rows compact from key[]
#ifndef KTH_TOPK_NT
#define KTH_TOPK_NT 1  // top-k rows load with the non-temporal hint too (the staged path reads a row once)
#endif
#ifndef KTH_ROWS_WAVES
#define KTH_ROWS_WAVES 4  // waves per SIMD the register budget is held to (<= 128 VGPRs)
#endif
#ifndef KTH_TOPK_ROWS_WAVES
#define KTH_TOPK_ROWS_WAVES KTH_ROWS_WAVES  // the same for the top-k rows kernels
#endif
constexpr int RW_BINS = 256;
constexpr int RW_STRIDE = RW_BINS + 4;  // words between histogram copies: 16-B aligned, a bin's copies in different banks

// Zero bins 0..255 of `copies` histogram copies: one 16-byte store per lane per copy.
__device__ __forceinline__ void zero_hist(uint32_t *hist, int copies, int lane) {
    for (int c = 0; c < copies; ++c)
        reinterpret_cast<uint4 *>(hist + c * RW_STRIDE)[lane] = make_uint4(0u, 0u, 0u, 0u);
}

// Raw bits of a key (inverse of the order-preserving transform).
template <bool F32>
__device__ __forceinline__ uint32_t raw_of_key(uint32_t key) {
    return F32 ? f32_of_key(key) : (uint32_t)i32_of_key(key);
}

// Cross-lane steps on DPP (row shifts and row broadcasts) and readlane: no
// LDS round trip and no per-lane address registers (__shfl's bpermute
// addresses are loop-invariant, get hoisted out of the row loop and spilled).
constexpr int DPP_ROW_SHR = 0x110, DPP_BCAST15 = 0x142, DPP_BCAST31 = 0x143;

template <int CTRL, int ROWS>
__device__ __forceinline__ uint32_t dpp(uint32_t old, uint32_t x) {
    return (uint32_t)__builtin_amdgcn_update_dpp((int)old, (int)x, CTRL, ROWS, 0xF, false);
}

// Inclusive prefix sum over the wave (lane 63 holds the total).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
    x += dpp<DPP_ROW_SHR + 1, 0xF>(0u, x);
    x += dpp<DPP_ROW_SHR + 2, 0xF>(0u, x);
    x += dpp<DPP_ROW_SHR + 4, 0xF>(0u, x);
    x += dpp<DPP_ROW_SHR + 8, 0xF>(0u, x);
    x += dpp<DPP_BCAST15, 0xA>(0u, x);
    x += dpp<DPP_BCAST31, 0xC>(0u, x);
    return x;
}

// Wave-wide reduction, result wave-uniform (op(a, b) commutative; id its identity).
template <typename Op>
__device__ __forceinline__ uint32_t wave_reduce(uint32_t x, uint32_t id, Op op) {
    x = op(x, dpp<DPP_ROW_SHR + 1, 0xF>(id, x));
    x = op(x, dpp<DPP_ROW_SHR + 2, 0xF>(id, x));
    x = op(x, dpp<DPP_ROW_SHR + 4, 0xF>(id, x));
    x = op(x, dpp<DPP_ROW_SHR + 8, 0xF>(id, x));
    x = op(x, dpp<DPP_BCAST15, 0xA>(id, x));
    x = op(x, dpp<DPP_BCAST31, 0xC>(id, x));
    return __builtin_amdgcn_readlane(x, 63);
}

__device__ __forceinline__ uint32_t lane_val(uint32_t x, int l) { return __builtin_amdgcn_readlane(x, l); }
__device__ __forceinline__ u64 lane_val(u64 x, int l) {
    return ((u64)lane_val((uint32_t)(x >> 32), l) << 32) | lane_val((uint32_t)x, l);
}

// Pick the bin holding the kk-th key from a wave-private 256-bin histogram
// (`copies` copies RW_STRIDE words apart): lane l owns bins 4l..4l+3; one wave
// scan of the per-lane sums and a ballot find the bin.  Returns the bin, the
// keys in bins below it and the keys in it (wave-uniform).
__device__ __forceinline__ void wave_pick(const uint32_t *hist, int copies, int lane, uint32_t kk, uint32_t &bin,
                                          uint32_t &below, uint32_t &cnt) {
    uint32_t h[4] = {0u, 0u, 0u, 0u};
    for (int c = 0; c < copies; ++c) {
        const uint4 b = reinterpret_cast<const uint4 *>(hist + c * RW_STRIDE)[lane];
        h[0] += b.x;
        h[1] += b.y;
        h[2] += b.z;
        h[3] += b.w;
    }
    const uint32_t sum = h[0] + h[1] + h[2] + h[3];
    const uint32_t incl = wave_incl_scan(sum);
    const uint32_t excl = incl - sum;
    const unsigned long long bm = __ballot(kk > excl && kk <= incl);
    const int L = bm ? __ffsll((long long)bm) - 1 : 0;
    uint32_t b = 0, bl = excl, c = 0;
    if (lane == L) {
        bool f = false;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            if (!f && bl + h[q] >= kk) {
                b = (uint32_t)(4 * L + q);
                c = h[q];
                f = true;
            } else if (!f) {
                bl += h[q];
            }
        }
    }
    bin = lane_val(b, L);
    below = lane_val(bl, L);
    cnt = lane_val(c, L);
}

__device__ __forceinline__ uint32_t wave_min_u32(uint32_t x) {
    return wave_reduce(x, 0xFFFFFFFFu, [](uint32_t a, uint32_t b) { return min(a, b); });
}
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t x) {
    return wave_reduce(x, 0u, [](uint32_t a, uint32_t b) { return max(a, b); });
}

// An opaque copy of a wave-uniform value: per-key expressions built on it are
// neither hoisted out of a loop nor shared with an earlier loop, which would
// keep one extra VGPR per key live (the keys already take KPL of them).
__device__ __forceinline__ uint32_t opaque(uint32_t x) {
    uint32_t y;
    asm volatile("s_mov_b32 %0, %1" : "=s"(y) : "s"(__builtin_amdgcn_readfirstlane(x)));
    return y;
}
__device__ __forceinline__ float opaque(float x) { return __uint_as_float(opaque(__float_as_uint(x))); }

// The first kernel's selection (A/B reference, KTH_ROWS_LEGACY): four 8-bit
// radix digits of the raw order key, the first counted into R0 copies.
// Returns the kk-th smallest of the lane keys; kk becomes its rank among the
// keys equal to it.
template <int KPL, int R0>
__device__ __forceinline__ uint32_t row_select_radix(const uint32_t (&key)[KPL], uint32_t *hist, int lane,
                                                     uint32_t &kk) {
    uint32_t prefix = 0;
    for (int pass = 0; pass < 4; ++pass) {  // wave-uniform
        const int shift = 24 - 8 * pass;
        const uint32_t pmask = pass ? 0xFFFFFFFFu << (32 - 8 * pass) : 0u;
        const int copies = pass ? 1 : R0;
        zero_hist(hist, copies, lane);
        __builtin_amdgcn_wave_barrier();
        uint32_t *mine = hist + (pass ? 0 : (lane % R0) * RW_STRIDE);
#pragma unroll
        for (int j = 0; j < KPL; ++j)
            if ((key[j] & pmask) == prefix) atomicAdd(&mine[(key[j] >> shift) & 0xFFu], 1u);
        __builtin_amdgcn_wave_barrier();
        uint32_t bin, below, cnt;
        wave_pick(hist, copies, lane, kk, bin, below, cnt);
        kk -= below;
        prefix |= bin << shift;
        __builtin_amdgcn_wave_barrier();  // the next zeroing after every lane's histogram reads
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
            return lane_val(val, __ffsll((long long)hm) - 1);
        }
    }
    return prefix;
}

// Float value of an order key in the selection order (ascending; for flip =
// ~0, the negated value, so that it ascends as the flipped keys do).
__device__ __forceinline__ float sel_value(uint32_t x, uint32_t flip) {
    const uint32_t key = x ^ flip;
    const uint32_t raw = (key & 0x80000000u) ? (key & 0x7FFFFFFFu) : ~key;
    const float v = __uint_as_float(raw);
    return flip ? -v : v;
}

// Range-normalised selection.  Pass A buckets every key by a monotone
// (non-decreasing) map b(x) into 256 bins spanning the row's own [kmin, kmax]:
//   int keys / non-finite float rows: b(x) = min(255, (x - kmin) >> sh), the
//       top 8 bits of the row's key range;
//   finite float rows: b(x) = min(255, (value(x) - vmin) * 256 / (vmax - vmin)),
//       linear in the VALUE, so uniform floats fill the bins evenly instead of
//       piling onto a few exponent bytes (LDS atomics on one address serialise).
// Rounding of the float map is monotone, so b is monotone and the keys of the
// picked bin B are exactly the keys of one interval [amin, amax]: the later
// passes are 8-bit radix digits of x - amin over that interval only.  Exact
// for any input; only the speed depends on the distribution.  Padding keys
// (0xFFFFFFFF, past `cols`) sort last and are bucketed like any key (the float
// map clamps them to bin 255); since k <= cols they never become the answer.
template <bool F32, int KPL, int R0>
__device__ __forceinline__ uint32_t row_select_range(const uint32_t (&key)[KPL], uint32_t *hist, int lane,
                                                     uint32_t &kk, uint32_t cols, uint32_t flip) {
    // the row's valid key range (padding excluded)
    uint32_t lmin = 0xFFFFFFFFu, lmax = 0u;
    const bool ragged = cols != (uint32_t)(KPL * WAVE);
    if (!ragged) {
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            lmin = min(lmin, key[j]);
            lmax = max(lmax, key[j]);
        }
    } else {
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const uint32_t e = (uint32_t)((j / 4) * WAVE + lane) * 4u + (j & 3);
            lmin = min(lmin, key[j]);
            lmax = max(lmax, e < cols ? key[j] : 0u);
        }
    }
    const uint32_t kmin = wave_min_u32(lmin), kmax = wave_max_u32(lmax);
    if (kmin == kmax) return kmin;  // kk is the rank among equal keys already

    // ---- pass A
    bool fmap = false;
    float fs = 0.f, fo = 0.f;
    if (F32) {
        const float vmin = sel_value(kmin, flip), vmax = sel_value(kmax, flip);
        const float range = vmax - vmin;
        const float scale = 256.0f / range;
        fmap = __builtin_isfinite(vmin) && __builtin_isfinite(vmax) && __builtin_isfinite(range) && range > 0.f &&
               __builtin_isfinite(scale) && scale > 0.f;
        fs = scale;
        fo = vmin;
    }
    const uint32_t span0 = kmax - kmin;
    const uint32_t W0 = 32u - (uint32_t)__clz(span0);
    const uint32_t sh = W0 > 8u ? W0 - 8u : 0u;
    // b(x); the parameters are passed in so that a second evaluation can take
    // opaque copies (no per-key values shared between the two loops)
    auto bucket = [&](uint32_t x, uint32_t lo, uint32_t hi, uint32_t shf, float o, float sc, uint32_t fl) -> uint32_t {
        if (F32 && fmap) {
            const float t = (sel_value(x, fl) - o) * sc;
            const uint32_t b = (uint32_t)__builtin_amdgcn_fmed3f(t, 0.f, 255.f);
            return x > hi ? 255u : b;
        }
        return min(255u, (x - lo) >> shf);
    };
    zero_hist(hist, R0, lane);
    __builtin_amdgcn_wave_barrier();
    {
        uint32_t *mine = hist + (lane % R0) * RW_STRIDE;
#pragma unroll
        for (int j = 0; j < KPL; ++j) atomicAdd(&mine[bucket(key[j], kmin, kmax, sh, fo, fs, flip)], 1u);
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t bin, below, cnt;
    wave_pick(hist, R0, lane, kk, bin, below, cnt);
    kk -= below;
    __builtin_amdgcn_wave_barrier();  // later zeroing after every lane's reads

    // ---- the picked bin as an interval [base, base + span], digits done so far
    uint32_t base, span, W, done, prefix;
    if (F32 && fmap) {
        uint32_t amin = 0xFFFFFFFFu, amax = 0u;
        const float o2 = opaque(fo), s2 = opaque(fs);
        const uint32_t hi2 = opaque(kmax), fl2 = opaque(flip);
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const bool in = bucket(key[j], kmin, hi2, sh, o2, s2, fl2) == bin;
            amin = in ? min(amin, key[j]) : amin;
            amax = in ? max(amax, key[j]) : amax;
        }
        amin = wave_min_u32(amin);
        amax = wave_max_u32(amax);
        if (amin == amax) return amin;
        base = amin;
        span = amax - amin;
        W = 32u - (uint32_t)__clz(span);
        done = 0;
        prefix = 0;
        cnt = 0;  // unknown as an interval count: run at least one digit
    } else {
        base = kmin;
        span = span0;
        W = W0;
        done = W0 - sh;
        prefix = bin;
    }
    // ---- 8-bit digits of x - base over the live interval
    while (true) {  // wave-uniform
        const uint32_t ob = opaque(base);
        auto live = [&](uint32_t x, uint32_t dn, uint32_t pf) {
            const uint32_t v = x - ob;
            return v <= span && (dn == 0 || (v >> (W - dn)) == pf);
        };
        if (done == W) return ob + prefix;
        if (cnt == 1) {  // the single live key is the answer
            uint32_t val = 0;
            bool have = false;
#pragma unroll
            for (int j = 0; j < KPL; ++j)
                if (!have && live(key[j], done, prefix)) {
                    val = key[j];
                    have = true;
                }
            const unsigned long long hm = __ballot(have);
            return lane_val(val, __ffsll((long long)hm) - 1);
        }
        const uint32_t d = min(8u, W - done);
        const uint32_t s = W - done - d, m = (1u << d) - 1u;
        zero_hist(hist, 1, lane);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int j = 0; j < KPL; ++j)
            if (live(key[j], done, prefix)) atomicAdd(&hist[((key[j] - ob) >> s) & m], 1u);
        __builtin_amdgcn_wave_barrier();
        wave_pick(hist, 1, lane, kk, bin, below, cnt);
        kk -= below;
        prefix = (prefix << d) | bin;
        done += d;
        __builtin_amdgcn_wave_barrier();
    }
}

// v_min3_f32 / v_max3_f32 without the IEEE-mode input canonicalisation the
// compiler adds around fminf/fmaxf (the row is NaN-checked separately).
__device__ __forceinline__ float min3f(float a, float b, float c) {
    float d;
    asm("v_min3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}
__device__ __forceinline__ float max3f(float a, float b, float c) {
    float d;
    asm("v_max3_f32 %0, %1, %2, %3" : "=v"(d) : "v"(a), "v"(b), "v"(c));
    return d;
}

// Value-linear bin of a finite float: clamp(fma(v, s, o), 0, 255).  fma and
// the clamp are monotone (rounding is), so the bin is a non-decreasing
// function of v, hence of the order key.
__device__ __forceinline__ uint32_t vbin(float v, float s, float o) {
    return (uint32_t)__builtin_amdgcn_fmed3f(__builtin_fmaf(v, s, o), 0.f, 255.f);
}

// The kk-th of the keys in [amin, amin + 8) when that interval holds it (its
// keys are the smallest kk or more of the range counted): every lane counts
// its keys of each value in 8-bit fields of two registers (no LDS atomics),
// one wave sum per pair of values in 16-bit fields.  kk becomes the rank among
// the answer's equal keys, *eq_out their number.
template <int KPL>
__device__ __forceinline__ uint32_t row_count_small(const uint32_t (&key)[KPL], uint32_t amin, uint32_t &kk,
                                                    uint32_t *eq_out) {
    // value d = x - amin of every key in [amin, amin + 8): field d & 3 of c[d >> 2]
    const uint32_t ob = opaque(amin);
    uint32_t c0 = 0, c1 = 0;
#pragma unroll
    for (int j = 0; j < KPL; ++j) {
        const uint32_t d = key[j] - ob;
        const uint32_t inc = 1u << ((d & 3u) << 3);
        c0 += d < 4u ? inc : 0u;
        c1 += d - 4u < 4u ? inc : 0u;
    }
    // (a lane counts <= KPL <= 64 keys a value: 8-bit fields; the wave sums in 16-bit fields)
    const auto add = [](uint32_t a, uint32_t b) { return a + b; };
    const uint32_t s01 = wave_reduce(c0 & 0x00FF00FFu, 0u, add), s23 = wave_reduce((c0 >> 8) & 0x00FF00FFu, 0u, add);
    const uint32_t s45 = wave_reduce(c1 & 0x00FF00FFu, 0u, add), s67 = wave_reduce((c1 >> 8) & 0x00FF00FFu, 0u, add);
    const uint32_t n[8] = {s01 & 0xFFFFu, s23 & 0xFFFFu, s01 >> 16, s23 >> 16,
                           s45 & 0xFFFFu, s67 & 0xFFFFu, s45 >> 16, s67 >> 16};
    uint32_t d = 0, acc = 0;
#pragma unroll
    for (int q = 0; q < 8; ++q)
        if (acc < kk) {  // wave-uniform
            d = (uint32_t)q;
            acc += n[q];
        }
    kk -= acc - n[d];
    if (eq_out) *eq_out = n[d];
    return amin + d;
}

// A picked bin of more than 64 keys (duplicate-heavy or clustered rows; was:
// four masked 8-bit radix sweeps of the whole row, ~24-35 VALU ops and four
// LDS atomics a key, and the atomics of a few-valued row serialise on a few
// addresses).  b is monotone, so bin B's keys are exactly the order keys of
// one interval [amin, amax] (min / max over the bin, one pass):
//   amin == amax: one value (a value-linear float row with values spaced wider
//       than a bin): it is the answer;
//   amax - amin < 8: at most 8 values: every lane counts its keys of each
//       value in 8-bit fields of two registers (no LDS atomics), one wave sum
//       per pair of values in 16-bit fields, then the kk-th;
//   wider (clustered rows): the masked radix sweeps of the whole row
//       (row_select_radix, rank kk_row in the row).
// kk is the rank within bin B on entry and within the answer's equal keys on
// return; key[] holds order keys (xor flip) on return when KEYS_OUT (else
// float rows may keep raw bits).
template <bool F32, int KPL, bool KEYS_OUT, typename ToKeys>
__device__ __forceinline__ uint32_t row_select_dense_bin(uint32_t (&key)[KPL], uint32_t *hist, int lane, uint32_t &kk,
                                                         uint32_t kk_row, uint32_t flip, bool vmap, float fs, float fo,
                                                         uint32_t bin, uint32_t cnt, uint32_t *eq_out,
                                                         ToKeys &&to_keys) {
    uint32_t amin = 0xFFFFFFFFu, amax = 0u;
    if (F32 && !KEYS_OUT && vmap && vbin(-0.f, fs, fo) == bin && vbin(0.f, fs, fo) == bin) {  // wave-uniform
        // bin B holds the value 0 (config 5's duplicate-heavy median: round(u *
        // 8) / 8 puts 1/16 of a row on +-0).  When the row's zeros are exactly
        // B's keys, their -0.0 / +0.0 counts decide: two compares a key counted
        // on the scalar unit, no min / max pass over the bin, and k-th rows keep
        // their raw bits (round 5 took the min / max pass, then these counts,
        // then converted every key)
        uint32_t cn = 0, cz = 0;
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            cn += (uint32_t)__popcll(__ballot(key[j] == 0x80000000u));
            cz += (uint32_t)__popcll(__ballot((key[j] << 1) == 0u));
            if (j % 4 == 3) __builtin_amdgcn_sched_barrier(0);  // (the masks die at once: no SGPR build-up)
        }
        if (cz == cnt) {  // wave-uniform: every key of B is a zero
            const uint32_t kn = key_of_f32(0x80000000u) ^ flip, kp = key_of_f32(0u) ^ flip, cp = cz - cn;
            const bool nfirst = kn < kp;  // the smaller order key first (flip: the k largest)
            const uint32_t c1 = nfirst ? cn : cp, c2 = nfirst ? cp : cn;
            if constexpr (KEYS_OUT) to_keys();
            if (kk <= c1) {
                if (eq_out) *eq_out = c1;
                return nfirst ? kn : kp;
            }
            kk -= c1;
            if (eq_out) *eq_out = c2;
            return nfirst ? kp : kn;
        }
    }
    if (F32 && vmap) {  // key[] holds raw float bits
        const float s2 = opaque(fs);
        float o2;
        asm volatile("v_mov_b32 %0, %1" : "=v"(o2) : "s"(opaque(fo)));
        const uint32_t ob = opaque(bin), fl = opaque(flip);
        // The bin's value range from float min / max (no order key per key):
        // vbin(v) == B  <=>  lo <= fma(v, s, o) and !(fma >= hi), with lo = -inf
        // for B = 0 and hi = NaN for B = 255 (the clamps); keys outside the bin
        // enter as +-inf.
        const float lo_t = ob == 0u ? -__builtin_inff() : (float)ob;
        const float hi_t = ob == 255u ? __builtin_nanf("") : (float)(ob + 1u);
        float vlo = __builtin_inff(), vhi = -__builtin_inff();
#pragma unroll
        for (int j = 0; j < KPL; j += 2) {
            const float a = __uint_as_float(key[j]), b = __uint_as_float(key[j + 1]);
            const float ta = __builtin_fmaf(a, s2, o2), tb = __builtin_fmaf(b, s2, o2);
            const bool ia = ta >= lo_t && !(ta >= hi_t), ib = tb >= lo_t && !(tb >= hi_t);
            vlo = min3f(vlo, ia ? a : __builtin_inff(), ib ? b : __builtin_inff());
            vhi = max3f(vhi, ia ? a : -__builtin_inff(), ib ? b : -__builtin_inff());
        }
        vlo = __uint_as_float(wave_reduce(__float_as_uint(vlo), 0x7F800000u, [](uint32_t x, uint32_t y) {
            return __float_as_uint(min3f(__uint_as_float(x), __uint_as_float(y), __uint_as_float(y)));
        }));
        vhi = __uint_as_float(wave_reduce(__float_as_uint(vhi), 0xFF800000u, [](uint32_t x, uint32_t y) {
            return __float_as_uint(max3f(__uint_as_float(x), __uint_as_float(y), __uint_as_float(y)));
        }));
        // the ends as order keys; an end at zero does not tell its sign (min /
        // max see -0 == +0, the keys -0 < +0): the zeros present stand in for
        // it (every zero of the row is in this bin then: one value, one bin)
        auto end_key = [&](float v) { return key_of_f32(__float_as_uint(v)) ^ fl; };
        if (vlo != 0.f) {
            amin = min(amin, end_key(vlo));
            amax = max(amax, end_key(vlo));
        }
        if (vhi != 0.f) {
            amin = min(amin, end_key(vhi));
            amax = max(amax, end_key(vhi));
        }
        if (vlo == 0.f || vhi == 0.f) {  // wave-uniform
            // the row's -0.0 / +0.0 counts: one compare a key, counted on the
            // scalar unit (ballot + popcount, no wave sum); a bin of zeros
            // only (vlo == vhi == 0) holds all of them: +0.0 = cnt - (-0.0)
            uint32_t cn = 0, cp = 0;
#pragma unroll
            for (int j = 0; j < KPL; ++j) cn += (uint32_t)__popcll(__ballot(key[j] == 0x80000000u));
            if (vlo == 0.f && vhi == 0.f) {  // wave-uniform
                cp = cnt - cn;
            } else {
#pragma unroll
                for (int j = 0; j < KPL; ++j) cp += (uint32_t)__popcll(__ballot(key[j] == 0u));
            }
            const uint32_t kn = end_key(-0.0f), kp = end_key(0.0f);
            if (cn) {
                amin = min(amin, kn);
                amax = max(amax, kn);
            }
            if (cp) {
                amin = min(amin, kp);
                amax = max(amax, kp);
            }
            if (cn && cp && amin == min(kn, kp) && amax == max(kn, kp)) {
                // the bin is the two zeros: the kk-th from their counts
                const uint32_t c1 = amin == kn ? cn : cp, c2 = amin == kn ? cp : cn;
                to_keys();
                if (kk <= c1) {
                    if (eq_out) *eq_out = c1;
                    return amin;
                }
                kk -= c1;
                if (eq_out) *eq_out = c2;
                return amax;
            }
        }
        to_keys();
    } else {
        const uint32_t ob = opaque(bin);
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            const bool in = (key[j] >> 24) == ob;
            amin = in ? min(amin, key[j]) : amin;
            amax = in ? max(amax, key[j]) : amax;
        }
    }
    amin = wave_min_u32(amin);
    amax = wave_max_u32(amax);
    const uint32_t span = amax - amin;
    if (span == 0) {
        if (eq_out) *eq_out = cnt;
        return amin;
    }
    if (span < 8) return row_count_small<KPL>(key, amin, kk, eq_out);
    // wider intervals (clustered rows; rare): the masked radix sweeps of the row
    const uint32_t ans = row_select_radix<KPL, 4>(key, hist, lane, kk_row);
    kk = kk_row;
    if (eq_out) {
        uint32_t e = 0;
#pragma unroll
        for (int j = 0; j < KPL; ++j) e += key[j] == ans ? 1u : 0u;
        *eq_out = wave_reduce(e, 0u, [](uint32_t a, uint32_t b) { return a + b; });
    }
    return ans;
}

// Fast path for full rows (cols = 64 * KPL, 16-byte aligned): one histogram
// pass, then the keys of the picked bin go to an LDS list and are ranked there.
//   pass A: 256 bins of a monotone map b(x) -- the top byte of the order key
//       (int32, and float rows holding a NaN), or for NaN-free float rows a
//       bin LINEAR IN THE VALUE over (about) the row's own [vmin, vmax]
//       (vbin), so uniform floats fill the bins evenly instead of piling onto
//       a few exponent bytes.  Float keys stay raw bits until they are needed
//       as order keys; their value bins are kept, four to a register, for the
//       filter (no second fma / clamp per key);
//   filter: the keys of the picked bin B are appended to the wave's LDS list
//       (ballot + mbcnt, only on the slots where some lane has one);
//   rank: with L <= 64 listed keys, lane i ranks list[i] against the list.
// b is monotone, so the bin's keys are exactly the keys between two order
// keys, and the kk-th of the row is the kk-th (after the keys below B) of the
// list.  A bin of more than 64 keys (duplicate-heavy or clustered rows) goes
// to row_select_dense_bin.  On return key[] holds order
// keys (xor flip) when KEYS_OUT (top-k compaction); else float rows may keep
// raw bits.  *eq_out: how many keys of the row equal the answer.
// Top-k rows (STAGE): the filter pass also stages every key of the bins up to
// B -- all the kept keys and the rest of bin B -- as (value, column) pairs in
// column order, and after the rank step one ordered compaction of those pairs
// writes the row's top-k (*topk_done = true).  No second look at the row.  The
// pairs need 2 * (below + cnt) words after the list; rows whose bins do not fit,
// or whose bin B is too full for the list, leave *topk_done false for the
// caller's general compaction.
struct TopkOut {
    uint32_t k;
    uint32_t *vals;
    int32_t *idx;
    u64 obase;
};
constexpr int STAGE_OFF = WAVE;  // staged keys start after the list's 64 words, their columns STAGE_CAP later
template <int R0>
constexpr uint32_t stage_cap() { return (uint32_t)(R0 * RW_STRIDE - STAGE_OFF) / 2; }

template <bool F32, int KPL, int R0, bool KEYS_OUT, bool STAGE = false>
__device__ __forceinline__ uint32_t row_select_fast(uint32_t (&key)[KPL], uint32_t *hist, int lane, uint32_t &kk,
                                                    uint32_t flip, uint32_t *eq_out = nullptr,
                                                    const TopkOut *tko = nullptr, bool *topk_done = nullptr) {
    // a dense bin's radix fallback (row_select_dense_bin) counts into 4 copies
    // of the wave's histogram: the caller sizes it R0 * RW_STRIDE words
    static_assert(R0 >= 4, "row_select_dense_bin needs at least 4 histogram copies per wave");
    auto to_keys = [&]() {
#pragma unroll
        for (int j = 0; j < KPL; ++j) {
            asm volatile("" : "+v"(key[j]));  // no sharing with earlier conversions (one live copy)
            key[j] = key_of_f32(key[j]) ^ flip;
        }
    };
    bool vmap = false;  // wave-uniform: value-linear bins (F32 rows without NaN)
    float fs = 0.f, fo = 0.f;
    if constexpr (F32) {  // key[] holds raw float bits
        // The bin map's range comes from every 4th key: keys outside it clamp
        // into the end bins, which stays monotone (and exact), so the range only
        // has to be close.  Infinities clamp the same way.  NaNs (last in the
        // order) would not, so every key is tested for one: an unordered compare
        // of two keys per instruction, straight into a wave mask.
        float vmin = __uint_as_float(key[0]), vmax = vmin;
        unsigned long long nanm = 0;
#pragma unroll
        for (int j = 0; j < KPL; j += 2) {
            const float a = __uint_as_float(key[j]), b = __uint_as_float(key[j + 1]);
            nanm |= __builtin_amdgcn_ballot_w64(a != a || b != b);
            if (j % 8 == 4) {
                const float c = __uint_as_float(key[j - 4]);
                vmin = min3f(vmin, a, c);
                vmax = max3f(vmax, a, c);
            }
        }
        vmin = __uint_as_float(wave_reduce(__float_as_uint(vmin), 0x7F800000u, [](uint32_t a, uint32_t b) {
            return __float_as_uint(min3f(__uint_as_float(a), __uint_as_float(b), __uint_as_float(b)));
        }));
        vmax = __uint_as_float(wave_reduce(__float_as_uint(vmax), 0xFF800000u, [](uint32_t a, uint32_t b) {
            return __float_as_uint(max3f(__uint_as_float(a), __uint_as_float(b), __uint_as_float(b)));
        }));
        const float range = vmax - vmin, scale = 256.0f / range;
        vmap = nanm == 0 && __builtin_isfinite(range) && range > 0.f && __builtin_isfinite(scale) && scale > 0.f;
        // bins ascend with the selection order: ascending v (flip = 0) or descending
        fs = flip ? -scale : scale;
        fo = flip ? vmax * scale : -vmin * scale;
        fs = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(fs)));
        fo = __uint_as_float(__builtin_amdgcn_readfirstlane(__float_as_uint(fo)));
        if (!vmap) to_keys();
    }
    if constexpr (!F32) {
        // Few-valued int rows (BASELINE config 5's duplicate-heavy variant):
        // their top-byte histogram sends a whole wave's keys to one or two LDS
        // addresses, and the atomics serialise (~2x the row's time).  When the
        // first key slot holds at most two top bytes (~never for spread-out
        // rows: three wave-uniform tests), the row's range decides: within 8
        // values the answer is counted in registers, no histogram at all.
        const uint32_t t0 = key[0] >> 24, b0 = __builtin_amdgcn_readfirstlane(t0);
        unsigned long long mm = __ballot(t0 == b0);
        if (~mm != 0ull) {  // wave-uniform
            const uint32_t b1 = (uint32_t)__builtin_amdgcn_readlane((int)t0, __builtin_ctzll(~mm));
            mm |= __ballot(t0 == b1);
        }
        if (mm == ~0ull) {  // wave-uniform
            uint32_t lmin = key[0], lmax = key[0];
#pragma unroll
            for (int j = 1; j < KPL; ++j) {
                lmin = min(lmin, key[j]);
                lmax = max(lmax, key[j]);
            }
            const uint32_t kmin = wave_min_u32(lmin), kmax = wave_max_u32(lmax);
            if (kmax - kmin < 8u) return row_count_small<KPL>(key, kmin, kk, eq_out);
        }
    }
    zero_hist(hist, R0, lane);
    __builtin_amdgcn_wave_barrier();
    uint32_t *mine = hist + (lane % R0) * RW_STRIDE;
    // each loop exists once per map (no per-key branch on the map)
    if (F32 && vmap) {
#pragma unroll
        for (int j = 0; j < KPL; ++j) atomicAdd(&mine[vbin(__uint_as_float(key[j]), fs, fo)], 1u);
    } else {
#pragma unroll
        for (int j = 0; j < KPL; ++j) atomicAdd(&mine[key[j] >> 24], 1u);
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t bin, below, cnt;
    wave_pick(hist, R0, lane, kk, bin, below, cnt);
    __builtin_amdgcn_wave_barrier();  // every lane's histogram reads before the list overwrites it
    if (cnt > (uint32_t)WAVE) {
        kk -= below;
        return row_select_dense_bin<F32, KPL, KEYS_OUT>(key, hist, lane, kk, kk + below, flip, vmap, fs, fo, bin, cnt,
                                                        eq_out, to_keys);
    }
    kk -= below;

    // filter the bin's keys into the list (the histogram words)
    // The lanes holding one (the compare's mask is the execution mask of the
    // store, so the position is mbcnt of exec: no per-key boolean in a VGPR).
    uint32_t fill = 0;
    auto append = [&](bool in, uint32_t x) __attribute__((always_inline)) {
        const unsigned long long B = __ballot(in);
        if (in) {
            const unsigned long long E = __builtin_amdgcn_read_exec();
            hist[fill + __builtin_amdgcn_mbcnt_hi((uint32_t)(E >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)E, 0u))] = x;
        }
        fill += (uint32_t)__popcll(B);
    };
    const bool stage = STAGE && below + cnt <= stage_cap<R0>();  // wave-uniform
    if (STAGE && stage) {
        // One pass stages every key of the bins up to B -- the kept keys and the
        // rest of bin B -- as (key, column) pairs in column order: per group of
        // 4 keys a lane (columns e + q, lane-major), the four ballots give each
        // lane its position.  Order keys are staged as they are (value-linear
        // rows: raw bits); the rank step's list is then read back from the
        // staged pairs (no second compare and append per key).
        // keys and columns in two arrays: adjacent 4-byte stores would merge into
        // one 8-byte store, which pairs every key with a neighbour register and
        // doubles the keys' VGPRs (spills)
        uint32_t *skey = hist + STAGE_OFF, *scol = skey + stage_cap<R0>();
        uint32_t staged = 0;
        uint32_t e0;
        asm volatile("v_lshlrev_b32 %0, 2, %1" : "=v"(e0) : "v"(lane));  // per row: not hoisted and spilled
        const float s2 = opaque(fs);
        float o2;
        asm volatile("v_mov_b32 %0, %1" : "=v"(o2) : "s"(opaque(fo)));
        const uint32_t ob = opaque(bin);
        const uint32_t hi_edge = opaque(bin << 24) | 0x00FFFFFFu;
        // value-linear rows: vbin(v) <= B  <=>  !(fma(v, s, o) >= B + 1), the
        // same fma as pass A and one compare (no clamp, no convert): for t in
        // [0, 255] trunc(t) <= B iff t < B + 1; t < 0 lands in bin 0 and passes;
        // bin 255 (B = 255) keeps every key, +inf included: the threshold is
        // then NaN and the unordered compare is true
        const float thr = opaque(ob == 255u ? __builtin_nanf("") : (float)(ob + 1u));
        // one loop per map (no per-key branch on it)
        auto stage_rows = [&](auto vm) __attribute__((always_inline)) {
            constexpr bool VM = decltype(vm)::value;
#pragma unroll
            for (int g = 0; g < KPL / 4; ++g) {
                bool c[4];
                unsigned long long bc[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const uint32_t x = key[4 * g + q];
                    if constexpr (VM)
                        c[q] = !(__builtin_fmaf(__uint_as_float(x), s2, o2) >= thr);
                    else
                        c[q] = x <= hi_edge;
                    bc[q] = __ballot(c[q]);
                }
                const unsigned long long any = bc[0] | bc[1] | bc[2] | bc[3];
                const uint32_t colg = e0 + (uint32_t)(g * WAVE * 4);
                // no lane stages two keys of the group (the usual case: ~80 of a
                // row's 4096 keys are staged): the lane's key goes to slot
                // staged + mbcnt(any), one pair of stores, selects instead of a
                // ballot + mbcnt chain per key slot
                const unsigned long long coll = (bc[0] & bc[1]) | ((bc[0] | bc[1]) & bc[2]) |
                                                ((bc[0] | bc[1] | bc[2]) & bc[3]);
                if (any != 0 && coll == 0) {  // wave-uniform
                    const uint32_t pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(any >> 32),
                                                                   __builtin_amdgcn_mbcnt_lo((uint32_t)any, staged));
                    // (selects on the ballots in asm: written as ?: the compiler turns
                    // the chain into a lane-indexed load of key[] from scratch)
                    uint32_t val = key[4 * g], q;
                    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(val) : "v"(val), "v"(key[4 * g + 1]), "s"(bc[1]));
                    asm("v_cndmask_b32_e64 %0, 0, 1, %1" : "=v"(q) : "s"(bc[1]));
                    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(val) : "v"(val), "v"(key[4 * g + 2]), "s"(bc[2]));
                    asm("v_cndmask_b32_e64 %0, %1, 2, %2" : "=v"(q) : "v"(q), "s"(bc[2]));
                    asm("v_cndmask_b32_e64 %0, %1, %2, %3" : "=v"(val) : "v"(val), "v"(key[4 * g + 3]), "s"(bc[3]));
                    asm("v_cndmask_b32_e64 %0, %1, 3, %2" : "=v"(q) : "v"(q), "s"(bc[3]));
                    if (c[0] || c[1] || c[2] || c[3]) {
                        skey[pos] = val;
                        scol[pos] = colg + q;
                    }
                    staged += (uint32_t)__popcll(any);
                } else if (any != 0) {  // wave-uniform
                    uint32_t pos = staged;
#pragma unroll
                    for (int q = 0; q < 4; ++q)
                        pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bc[q] >> 32),
                                                        __builtin_amdgcn_mbcnt_lo((uint32_t)bc[q], pos));
#pragma unroll
                    for (int q = 0; q < 4; ++q) {
                        if (c[q]) {
                            skey[pos] = key[4 * g + q];
                            scol[pos] = colg + (uint32_t)q;
                        }
                        pos += c[q] ? 1u : 0u;
                        staged += (uint32_t)__popcll(bc[q]);
                    }
                }
                __builtin_amdgcn_sched_barrier(0);  // keep the groups apart: no hoisting across them (VGPRs)
            }
        };
#ifndef KTH_DIAG_ROWS_NOSTAGE  // (timing diagnostics only: wrong results)
        if (F32 && vmap)
            stage_rows(std::true_type{});
        else
            stage_rows(std::false_type{});
#endif
#ifdef KTH_DIAG_ROWS_NOTAIL
        *topk_done = true;
        return staged;
#endif
        __builtin_amdgcn_wave_barrier();
        // the list: the staged keys of bin B (a handful of rounds over <= nc pairs)
        for (uint32_t i0 = 0; i0 < staged; i0 += WAVE) {  // wave-uniform
            const uint32_t i = i0 + (uint32_t)lane;
            const uint32_t x = i < staged ? skey[i] : 0u;
            const bool inb = i < staged && ((F32 && vmap) ? vbin(__uint_as_float(x), s2, o2) == ob : (x >> 24) == ob);
            append(inb, x);
        }
    } else if (F32 && vmap) {
        // the bin recomputed exactly as pass A did (fma, clamp, convert) and one
        // compare: a single mask per key.  The offset sits in a VGPR (an fma reads
        // at most one SGPR on gfx9); opaque copies keep pass A's per-key values
        // from being kept live until here.
        const float s2 = opaque(fs);
        float o2;
        asm volatile("v_mov_b32 %0, %1" : "=v"(o2) : "s"(opaque(fo)));
        const uint32_t ob = opaque(bin);
#pragma unroll
        for (int j = 0; j < KPL; ++j) append(vbin(__uint_as_float(key[j]), s2, o2) == ob, key[j]);
    } else {
        const uint32_t lo = opaque(bin << 24);  // top-byte bin B = keys [B << 24, +2^24)
#pragma unroll
        for (int j = 0; j < KPL; ++j) append(key[j] - lo <= 0x00FFFFFFu, key[j]);
    }
    __builtin_amdgcn_wave_barrier();
    const uint32_t L = cnt;  // == fill
    if (F32 && vmap) {  // raw bits -> order keys, in the list
        if ((uint32_t)lane < L) hist[lane] = key_of_f32(hist[lane]) ^ flip;
        __builtin_amdgcn_wave_barrier();
    }
    const uint32_t my = (uint32_t)lane < L ? hist[lane] : 0u;
    uint32_t lt = 0, le = 0;
    // wave-uniform trip counts, broadcast reads: four list keys a 16-byte read
    // (one read and no loop bookkeeping per key), then the last L % 4
    uint32_t i = 0;
    for (; i + 4 <= L; i += 4) {
        const uint4 y = *reinterpret_cast<const uint4 *>(hist + i);
        lt += (y.x < my ? 1u : 0u) + (y.y < my ? 1u : 0u) + (y.z < my ? 1u : 0u) + (y.w < my ? 1u : 0u);
        le += (y.x <= my ? 1u : 0u) + (y.y <= my ? 1u : 0u) + (y.z <= my ? 1u : 0u) + (y.w <= my ? 1u : 0u);
    }
    for (; i < L; ++i) {
        const uint32_t y = hist[i];
        lt += y < my ? 1u : 0u;
        le += y <= my ? 1u : 0u;
    }
    const unsigned long long bm = __ballot((uint32_t)lane < L && lt < kk && kk <= le);
    const int f = bm ? __ffsll((long long)bm) - 1 : 0;
    const uint32_t answer = lane_val(my, f);
    kk -= lane_val(lt, f);
    if (eq_out) *eq_out = lane_val(le, f) - lane_val(lt, f);  // every key equal to the answer is listed
    __builtin_amdgcn_wave_barrier();
    if (STAGE && stage) {
        // the staged pairs in column order: keep the keys below the k-th and the
        // first kk keys equal to it (ties by column).  (Staging the kept pairs in
        // LDS for one pass of 16-byte stores measured the same: the output's
        // cost is its DRAM writes, not the store instructions.)
        const uint32_t *skey = hist + STAGE_OFF, *scol = skey + stage_cap<R0>();
        const uint32_t nc = below + cnt;
        uint32_t out = 0, eq_seen = 0;
        for (uint32_t b0 = 0; b0 < nc; b0 += WAVE) {  // wave-uniform
            const uint32_t i = b0 + (uint32_t)lane;
            const bool valid = i < nc;
            const uint2 pr = valid ? make_uint2(skey[i], scol[i]) : make_uint2(0u, 0u);
            const uint32_t u = (F32 && vmap) ? key_of_f32(pr.x) ^ flip : pr.x;
            const bool lt2 = valid && u < answer, eq2 = valid && u == answer;
            const unsigned long long be = __ballot(eq2);
            const uint32_t rank = eq_seen + __builtin_amdgcn_mbcnt_hi((uint32_t)(be >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)be, 0u));
            const bool keep = lt2 || (eq2 && rank < kk);
            const unsigned long long bk = __ballot(keep);
            const uint32_t pos = out + __builtin_amdgcn_mbcnt_hi((uint32_t)(bk >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bk, 0u));
#ifndef KTH_DIAG_ROWS_NOSTORE  // (timing diagnostics only: no output)
            if (keep) {
                if (tko->vals) tko->vals[tko->obase + pos] = (F32 && vmap) ? pr.x : raw_of_key<F32>(pr.x ^ flip);
                if (tko->idx) tko->idx[tko->obase + pos] = (int32_t)pr.y;
            }
#else
            asm volatile("" ::"v"(pos), "v"(pr.x), "v"(pr.y), "v"((uint32_t)keep));
#endif
            out += (uint32_t)__popcll(bk);
            eq_seen += (uint32_t)__popcll(be);
        }
        *topk_done = true;
        __builtin_amdgcn_wave_barrier();
        return answer;
    }
    if (KEYS_OUT && F32 && vmap) to_keys();
    return answer;
}

// TOPK = false: out[r] = the k-th smallest of row r.
// TOPK = true: vals[r*k ..] / idx[r*k ..] = the k smallest keys of row r and
// their columns, in column order; of the keys equal to the k-th, the first
// ones by column.  flip = 0xFFFFFFFF selects the k largest instead (the key
// order reversed: ~key).
// FULL: cols == 64 * KPL and 16-byte aligned rows (unguarded loads, row_select_fast).
template <bool F32, int KPL, bool VEC, int R0, bool TOPK, bool FULL>
__global__ __launch_bounds__(RW_BLOCK, !VEC ? 1 : (TOPK && !(TOPK_RELOAD && FULL)) ? 2 : TOPK ? KTH_TOPK_ROWS_WAVES : KTH_ROWS_WAVES) void k_rows_reg(const uint32_t *__restrict__ m, u64 rows, uint32_t cols,
                                                      uint32_t k, uint32_t *__restrict__ out, uint32_t flip,
                                                      uint32_t *__restrict__ vals, int32_t *__restrict__ idx) {
    static_assert(KPL % 4 == 0, "16-byte loads");
    __shared__ __attribute__((aligned(16))) uint32_t hist_all[RW_BLOCK / WAVE][R0 * RW_STRIDE];
    const int lane = threadIdx.x & (WAVE - 1), wid = threadIdx.x / WAVE;
    uint32_t *hist = hist_all[wid];
    // One row per wave (the grid covers the rows): a row loop let the compiler
    // hoist per-row address arithmetic out of it and spill it (the top-k
    // variants sit at the 128-VGPR budget of 4 waves per SIMD).
    const u64 r = (u64)blockIdx.x * (RW_BLOCK / WAVE) + wid;
    if (r < rows) {  // wave-uniform
        const uint32_t *row = m + r * (u64)cols;
        uint32_t key[KPL];
        uint32_t kk = k, answer, eqn = 0;  // eqn: keys equal to the answer (FULL rows; 0 = unknown)
        bool topk_done = false;            // the fast path wrote the row's top-k itself
        if (FULL) {
#pragma unroll
            for (int j = 0; j < KPL / 4; ++j) {
                // (top-k rows whose bins cannot be staged re-read the row; with
                // the non-temporal hint that re-read comes from HBM, not L2 -- rare)
                const uint4 *src = reinterpret_cast<const uint4 *>(row + (j * WAVE + lane) * 4);
                const uint4 x = TOPK && !KTH_TOPK_NT ? *src : load_nt(src);
                key[4 * j + 0] = x.x;
                key[4 * j + 1] = x.y;
                key[4 * j + 2] = x.z;
                key[4 * j + 3] = x.w;
            }
            if (!F32) {
#pragma unroll
                for (int j = 0; j < KPL; ++j) {
                    key[j] = key_of_i32(key[j]) ^ flip;
                    // opaque: later uses of the raw value recompute it from the key
                    // instead of keeping the loaded word live beside it (VGPRs)
                    if (TOPK) asm volatile("" : "+v"(key[j]));
                }
            }
#ifdef KTH_ROWS_LEGACY
            if (F32) {
#pragma unroll
                for (int j = 0; j < KPL; ++j) key[j] = key_of_f32(key[j]) ^ flip;
            }
            answer = row_select_radix<KPL, R0>(key, hist, lane, kk);
#else
#ifndef KTH_DIAG_ROWS_SMALLOUT
            const TopkOut tko{k, vals, idx, r * (u64)k};
#else  // (timing only: every row's output to one of 64 row slots, L2-resident)
            const TopkOut tko{k, vals, idx, (r & 63) * (u64)k};
#endif
            answer = row_select_fast<F32, KPL, R0, TOPK, TOPK>(key, hist, lane, kk, TOPK ? flip : 0u,
                                                                TOPK ? &eqn : nullptr, &tko, &topk_done);
#endif
        } else {
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
#ifdef KTH_ROWS_LEGACY
        answer = row_select_radix<KPL, R0>(key, hist, lane, kk);
#else
        answer = row_select_range<F32, KPL, R0>(key, hist, lane, kk, cols, flip);
#endif
        }
        if (!TOPK) {
#ifndef KTH_DIAG_ROWS_NOOUT
            if (lane == 0) out[r] = raw_of_key<F32>(answer ^ flip);
#else
            asm volatile("" ::"v"(answer));
#endif
        } else if (!topk_done) {
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
            // One group of 4 keys (columns e .. e + 3) of this lane.
            auto group = [&](uint32_t e, const uint32_t (&g)[4]) __attribute__((always_inline)) {
                bool lt[4], eq[4], sel[4];
                uint32_t eq_below = 0, eq_tot = 0;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    const bool valid = FULL || e + q < cols;
                    lt[q] = valid && g[q] < answer;
                    eq[q] = valid && g[q] == answer;
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
                        const uint32_t x = raw_of_key<F32>(g[q] ^ flip);
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
            };
            // Every key equal to the k-th is kept (kk == eqn: always for rows of
            // distinct keys): the kept keys are exactly key <= answer, one compare
            // each.  Per group, the four ballots of the kept keys give each lane its
            // position (mbcnt of the lanes below, plus its own earlier q); the
            // (value, column) pairs go to LDS as one 8-byte write.
            auto group_all = [&](uint32_t e, const uint32_t (&g)[4]) __attribute__((always_inline)) {
                bool sel[4];
                unsigned long long bs[4];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    sel[q] = g[q] <= answer;
                    bs[q] = __ballot(sel[q]);
                }
                if ((bs[0] | bs[1] | bs[2] | bs[3]) == 0) return;  // wave-uniform
                uint32_t pos = taken;
#pragma unroll
                for (int q = 0; q < 4; ++q)
                    pos = __builtin_amdgcn_mbcnt_hi((uint32_t)(bs[q] >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)bs[q], pos));
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    if (sel[q]) {
                        const uint32_t x = raw_of_key<F32>(g[q] ^ flip);
                        if (stage) {
                            reinterpret_cast<uint2 *>(hist)[pos] = make_uint2(x, e + q);
                        } else {
                            if (vals) vals[obase + pos] = x;
                            if (idx) idx[obase + pos] = (int32_t)(e + q);
                        }
                    }
                    pos += sel[q] ? 1u : 0u;
                    taken += (uint32_t)__popcll(bs[q]);
                }
            };
            const bool all_ties = FULL && kk == eqn;
            if (TOPK_KEYS_COMPACT && !F32 && TOPK_RELOAD && FULL) {
                // int rows: key[] still holds the row's order keys (KEYS_OUT):
                // compact from the registers -- the re-read below comes from HBM
                // (the row was loaded non-temporal), a second pass over the
                // row's bytes.  (Float rows: the same code made the kernel
                // spill 200 B in its prologue.)
#pragma unroll
                for (int j = 0; j < KPL / 4; ++j) {
                    const uint32_t g[4] = {key[4 * j], key[4 * j + 1], key[4 * j + 2], key[4 * j + 3]};
                    group((uint32_t)(j * WAVE + lane) * 4u, g);
                    __builtin_amdgcn_sched_barrier(0);  // keep the groups apart: no hoisting across them (VGPRs)
                }
            } else if (TOPK_RELOAD && FULL && all_ties) {
                // the row again, from L2, every group's load in flight at once (the
                // keys' registers are free by now): one round trip per row, not
                // one per two groups
                const uint4 *src = reinterpret_cast<const uint4 *>(row);
                uint4 xr[KPL / 4];
#pragma unroll
                for (int j = 0; j < KPL / 4; ++j) xr[j] = src[j * WAVE + lane];
                // columns from a per-row copy of 4 * lane: hoisted out of the row
                // loop, the sixteen group columns were spilled to scratch
                uint32_t e0;
                asm volatile("v_lshlrev_b32 %0, 2, %1" : "=v"(e0) : "v"(lane));
#pragma unroll
                for (int j = 0; j < KPL / 4; ++j) {
                    const uint32_t raw[4] = {xr[j].x, xr[j].y, xr[j].z, xr[j].w};
                    uint32_t g[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) g[q] = (F32 ? key_of_f32(raw[q]) : key_of_i32(raw[q])) ^ flip;
                    group_all(e0 + (uint32_t)(j * WAVE * 4), g);
                    __builtin_amdgcn_sched_barrier(0);  // keep the groups apart: no hoisting across them (VGPRs)
                }
            } else if (TOPK_RELOAD && FULL) {
                // FULL rows re-read their keys here (from L2: loaded without the
                // non-temporal hint), two groups ahead, in a rolled loop, instead of
                // keeping all KPL keys live through the compaction: 4 waves per
                // SIMD instead of 2.
                const uint4 *src = reinterpret_cast<const uint4 *>(row);
                uint4 nx = src[lane], nx2 = src[WAVE + lane];  // two groups in flight
#pragma unroll 1
                for (int j = 0; j < KPL / 4; ++j) {
                    const uint4 x = nx;
                    nx = nx2;
                    if (j + 2 < KPL / 4) nx2 = src[(j + 2) * WAVE + lane];
                    const uint32_t raw[4] = {x.x, x.y, x.z, x.w};
                    uint32_t g[4];
#pragma unroll
                    for (int q = 0; q < 4; ++q) g[q] = (F32 ? key_of_f32(raw[q]) : key_of_i32(raw[q])) ^ flip;
                    group((uint32_t)(j * WAVE + lane) * 4u, g);
                }
            } else {
#pragma unroll
                for (int j = 0; j < KPL / 4; ++j) {
                    const uint32_t g[4] = {key[4 * j], key[4 * j + 1], key[4 * j + 2], key[4 * j + 3]};
                    group((uint32_t)(j * WAVE + lane) * 4u, g);
                    __builtin_amdgcn_sched_barrier(0);  // keep the groups apart: no hoisting across them (VGPRs)
                }
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
