// kth_topk.hpp -- top-k of one int32 array, gfx950.
//
// The k smallest (or largest) keys of n, with their int64 indices, written in
// index order; of the keys equal to the k-th, the first ones by index.  The
// reference has no top-k: its select block (kth-problem-seq.c:30-35) sorts and
// reads one index, and sort(a)[:k] is the top-k it implies.  After the k-th
// key v is known (select_async leaves it in d_status[0]), on 1024-key
// "wave tiles" (one wavefront each, no barriers in the streaming kernels):
//   k_topk_count   per tile, #better-than-v | #equal << 16; reads only the
//                  tiles the select's own streaming pass flagged as possibly
//                  holding output (k_main<TF>), all tiles otherwise
//   k_topk_bases   per 4096 tiles: each tile's offsets inside its block and
//                  the block's sums; the last workgroup: exclusive block
//                  bases, need = k - #better
//   k_topk_write   per tile that holds an output key: wave scan + scatter;
//                  tiles without output never load their keys.
// A kept key's slot is (#better before it) + min(#equal before it, need).
#pragma once
#include "kth_device.hpp"

namespace kth {

constexpr int TK_BLOCK = 256;
constexpr int TK_TILE = 1024;                     // keys per wave tile
constexpr int TK_KPL = TK_TILE / WAVE;            // 16 keys per lane
constexpr int TK_TILES_PER_BLOCK = TK_BLOCK * 16;  // reduce / down-sweep granularity (4096 tiles)
// scratch (u64 words): tile counts (u32, ntiles), tile offsets (u64, ntiles),
// block sums (2 per block), block bases (2 per block), meta [need, error]

// order test against the k-th key: flip = 0 for smallest, ~0 for largest
__device__ __forceinline__ bool tk_better(uint32_t u, uint32_t uv, uint32_t flip) { return (u ^ flip) < (uv ^ flip); }

__device__ __forceinline__ uint32_t wave_sum32(uint32_t x) {
    return (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_scan32(x), WAVE - 1);
}

// Pass 1: tile t = keys [1024 t, 1024 t + 1024); tcnt[t] = #better | #equal << 16.
// Lane l reads the 16-byte words l, l + 64, l + 128, l + 192 of its tile.
// Tiles the select's streaming pass proved empty of output are skipped: when
// k_main<TF> ran (tflags[2] == 1) and v lies on the window's near side of its
// far edge, a tile inside k_main's full tiles (rows of TK_MAIN_ROW keys after
// `head` unaligned keys; MAIN_UNROLL rows per tile, nfull tiles) whose rows
// carry no flag bit has no key <= v (>= v for largest): count 0, no loads.
constexpr u64 TK_MAIN_ROW = (u64)BLK * 4;  // keys per k_main row (one 16-B load per thread)
__device__ __forceinline__ bool tk_row_flagged(const uint8_t *fb, const RowWords &fl, u64 r) {
    const u64 t = r / MAIN_UNROLL;
    const uint32_t bit = 1u << (r % MAIN_UNROLL);
    return ((fb[fl_index(fl, t, 0)] | fb[fl_index(fl, t, 1)] | fb[fl_index(fl, t, 2)] | fb[fl_index(fl, t, 3)]) & bit) != 0u;
}

// META (after k_main<3/4>, 16-byte aligned keys): the first ncov tiles are
// k_main's rows; when v lies inside the window and no candidate was dropped
// (meta_ok), an unmarked row holds no key equal to lo or hi, so its #better is
// the sum of its four wave-row words (#<lo, or #>hi for largest) and k_topk_cands
// adds the candidates' share: no key of it is loaded.  Marked rows
// (TK_RECOUNT) are counted from the input.
__device__ __forceinline__ bool tk_meta_ok(const uint32_t *tflags, const int32_t *d_v, const SelState *st) {
    return tflags[2] == 1u && d_v[0] >= (int32_t)tflags[0] && d_v[0] <= (int32_t)tflags[1] && st->cnt[C_OVF] == 0;
}

// a tile count word: #better | #equal << 16, plus TK_RECOUNT (bit 31) on a
// META tile counted from the input (its candidates' share, added before, is overwritten)
__device__ __forceinline__ uint32_t tk_better_of(uint32_t c) { return c & 0xFFFFu; }
__device__ __forceinline__ uint32_t tk_equal_of(uint32_t c) { return (c >> 16) & 0x7FFFu; }

// STAGED (after k_main<5/6>): the first ncov tiles' staged entries hold every
// key on the kept side of the window's far edge, in index order per wave-row;
// when v lies inside the window and no segment overflowed, k_tk5_count /
// k_tk5_write handle those tiles from the entries alone.
__device__ __forceinline__ bool tk5_ok(const uint32_t *tflags, const int32_t *d_v) {
    return tflags[2] == 1u && tflags[3] == 0u && d_v[0] >= (int32_t)tflags[0] && d_v[0] <= (int32_t)tflags[1];
}

// MODE: 0 = flags (k_main<1/2>) or none, 1 = row words (k_main<3/4>), 2 = staged (k_main<5/6>)
template <bool ALIGNED, int MODE>
__global__ __launch_bounds__(TK_BLOCK) void k_topk_count(const uint32_t *__restrict__ keys, u64 n, u64 ntiles,
                                                         const int32_t *__restrict__ d_v, uint32_t flip,
                                                         uint32_t *__restrict__ tcnt,
                                                         const uint32_t *__restrict__ tflags, u64 head, u64 nfull,
                                                         const SelState *__restrict__ st, u64 ncov,
                                                         RowWords rwl = RowWords{1, 0}) {
    const uint32_t uv = key_of_i32((uint32_t)d_v[0]);
    const int lane = threadIdx.x & (WAVE - 1);
    const u64 nw = (u64)gridDim.x * (TK_BLOCK / WAVE);
    constexpr bool META = MODE == 1;
    const bool skip_ok =
        MODE == 0 && tflags[2] == 1u && (flip == 0u ? d_v[0] <= (int32_t)tflags[1] : d_v[0] >= (int32_t)tflags[0]);
    const bool meta_ok = META && tk_meta_ok(tflags, d_v, st);
    const bool staged_ok = MODE == 2 && tk5_ok(tflags, d_v);
    const uint32_t mark = meta_ok ? TK_RECOUNT : 0u;
    const uint8_t *fb = reinterpret_cast<const uint8_t *>(tflags + 4);  // MODE 0: k_main<1/2>'s flag bytes (rwl: fl_index)
    // each wave takes 64 tiles at a time: lane l tests tile tg + l's flags, the
    // wave then streams only the tiles that may hold output
    for (u64 tg = ((u64)blockIdx.x * (TK_BLOCK / WAVE) + threadIdx.x / WAVE) * WAVE; tg < ntiles; tg += nw * WAVE) {
        const u64 tl = tg + lane;
        bool act = tl < ntiles;
        if (staged_ok && tl < ncov) act = false;  // counted by k_tk5_count
        if (act && meta_ok && tl < ncov) {
            const uint32_t w0 = tflags[rw_index(rwl, tl, 0)], w1 = tflags[rw_index(rwl, tl, 1)],
                           w2 = tflags[rw_index(rwl, tl, 2)], w3 = tflags[rw_index(rwl, tl, 3)];
            if (((w0 | w1 | w2 | w3) & TK_RECOUNT) == 0u) {
                tcnt[tl] += w0 + w1 + w2 + w3;  // k_topk_cands ran first: add to the candidates' share
                act = false;
            }
        }
        if (act && skip_ok && tl * TK_TILE >= head) {
            const u64 b0 = tl * TK_TILE, last = (b0 + TK_TILE < n ? b0 + TK_TILE : n) - 1;
            const u64 ra = (b0 - head) / TK_MAIN_ROW, rb = (last - head) / TK_MAIN_ROW;
            if (rb / MAIN_UNROLL < nfull && !tk_row_flagged(fb, rwl, ra) && !tk_row_flagged(fb, rwl, rb)) {
                act = false;
                tcnt[tl] = 0u;
            }
        }
        u64 todo = __ballot(act);
        while (todo) {  // two tiles per round: 8 loads in flight per lane
            const u64 t1 = tg + __builtin_ctzll(todo);
            todo &= todo - 1;
            const bool two = todo != 0;
            const u64 t2 = two ? tg + __builtin_ctzll(todo) : t1;
            if (two) todo &= todo - 1;
            uint32_t c1 = 0, c2 = 0;
            auto one = [&](uint32_t &c, uint32_t x) {
                const uint32_t u = key_of_i32(x);
                c += tk_better(u, uv, flip) ? 1u : 0u;
                c += u == uv ? 0x10000u : 0u;
            };
            const u64 b1 = t1 * TK_TILE, b2 = t2 * TK_TILE;
            if (ALIGNED && b1 + TK_TILE <= n && b2 + TK_TILE <= n) {
                uint4 q[8];
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    q[r] = load_nt(reinterpret_cast<const uint4 *>(keys + b1 + r * 256 + lane * 4));
                    q[4 + r] = load_nt(reinterpret_cast<const uint4 *>(keys + b2 + r * 256 + lane * 4));
                }
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    one(c1, q[r].x);
                    one(c1, q[r].y);
                    one(c1, q[r].z);
                    one(c1, q[r].w);
                    one(c2, q[4 + r].x);
                    one(c2, q[4 + r].y);
                    one(c2, q[4 + r].z);
                    one(c2, q[4 + r].w);
                }
            } else {
#pragma unroll
                for (int j = 0; j < TK_KPL; ++j) {
                    const u64 i1 = b1 + j * WAVE + lane, i2 = b2 + j * WAVE + lane;
                    if (i1 < n) one(c1, keys[i1]);
                    if (i2 < n) one(c2, keys[i2]);
                }
            }
            c1 = wave_sum32(c1);
            c2 = wave_sum32(c2);
            if (lane == 0) {
                tcnt[t1] = c1 | mark;
                if (two) tcnt[t2] = c2 | mark;
            }
        }
    }
}

// Pass 0 (META, before k_topk_count, into zeroed counts): the candidates'
// share of their rows' counts, one atomic per candidate better than or equal
// to v (no read: a row k_topk_count then counts from the input is simply
// overwritten there; rows past ncov carry row ~0u).  A wave takes TKC_U x 64
// consecutive candidates, lane l every 64th, with all their loads in flight
// (one candidate a lane waited a memory round trip per 64: 48 us at k = 2^27);
// each atomic instruction then covers 64 consecutive candidates, whose rows
// (~6 candidates a row at 2^30) share a few cache lines of the counts.  (Runs
// of 8 consecutive candidates per lane, one atomic per run of equal rows:
// fewer atomics, but each instruction's spread over ~64 lines: 68 us.)
// Then one atomic per run of equal rows among a wave-instruction's 64
// (k = 2^27 / 2^29: 34 / 42 us against 50 / 105 for one per candidate, and
// 48 / 102 with one candidate a lane).
constexpr int TKC_U = 8;  // candidates a lane loads together
__global__ __launch_bounds__(TK_BLOCK) void k_topk_cands(const uint32_t *__restrict__ cand,
                                                         const uint32_t *__restrict__ rows,
                                                         const u64 *__restrict__ cand_count, u64 cap,
                                                         const int32_t *__restrict__ d_v, uint32_t flip,
                                                         uint32_t *__restrict__ tcnt,
                                                         const uint32_t *__restrict__ tflags,
                                                         const SelState *__restrict__ st) {
    if (!tk_meta_ok(tflags, d_v, st)) return;
    const uint32_t uv = key_of_i32((uint32_t)d_v[0]);
    const u64 m = min(*cand_count, cap);
    const int lane = threadIdx.x & (WAVE - 1);
    const u64 nw = (u64)gridDim.x * (TK_BLOCK / WAVE);
    for (u64 b = ((u64)blockIdx.x * (TK_BLOCK / WAVE) + threadIdx.x / WAVE) * (TKC_U * WAVE); b < m;
         b += nw * (TKC_U * WAVE)) {
        uint32_t u[TKC_U], r[TKC_U];
#pragma unroll
        for (int q = 0; q < TKC_U; ++q) {
            const u64 i = b + (u64)q * WAVE + lane;
            r[q] = i < m ? rows[i] : ~0u;
            u[q] = i < m ? cand[i] : 0u;
        }
#pragma unroll
        for (int q = 0; q < TKC_U; ++q) {
            const uint32_t c = tk_better(u[q], uv, flip) ? 1u : (u[q] == uv ? 0x10000u : 0u);
            {
                // one atomic per run of equal rows among the wave's 64: the
                // run's last lane adds (prefix sum here) - (prefix sum at the
                // run before); prefix sums never decrease (fields <= 64), so
                // "at the run before" is a max-scan of the runs' last lanes
                const uint32_t rn = (uint32_t)__shfl_down((int)r[q], 1, WAVE);
                const bool last = lane == WAVE - 1 || rn != r[q];
                const uint32_t S = wave_incl_scan32(c);
                uint32_t T = last ? S : 0u;
                T = max(T, dpp32<0x111, 0xF>(T));
                T = max(T, dpp32<0x112, 0xF>(T));
                T = max(T, dpp32<0x114, 0xF>(T));
                T = max(T, dpp32<0x118, 0xF>(T));
                T = max(T, dpp32<0x142, 0xA>(T));
                T = max(T, dpp32<0x143, 0xC>(T));
                const uint32_t before = (uint32_t)__shfl_up((int)T, 1, WAVE);
                const uint32_t add = S - (lane == 0 ? 0u : before);
                // (~0u: past m, or outside k_main's rows: counted from the input)
                if (last && r[q] != ~0u && add) atomicAdd(&tcnt[r[q]], add);
            }
        }
    }
}

// A bracket failure (counts that do not hold the k-th; cannot happen for a
// correct v) is raised in the select's state (SelState.error =
// TK_ERR_BRACKET), which kth_ctx_last_stats reports; k_topk_write then
// writes nothing (meta[1]).
constexpr uint32_t TK_ERR_BRACKET = 32;

// Pass 2 (k_topk_bases, one workgroup per 4096 tiles): each
// workgroup writes its tiles' in-block offsets (toff) and its
// block's two sums (bsum, write-through), then arrives on a counter; the
// last to arrive scans the block sums into the block bases and meta (as
// a one-workgroup scan) and resets the counter.  (Round 4 had three
// launches here: block sums, the scan of them, the in-block offsets.)
__global__ __launch_bounds__(TK_BLOCK) void k_topk_bases(const uint32_t *__restrict__ tcnt, u64 ntiles,
                                                         u64 *__restrict__ toff, u64 *__restrict__ bsum,
                                                         u64 k, u64 *__restrict__ base, u64 *__restrict__ meta,
                                                         SelState *__restrict__ st, uint32_t *__restrict__ arrive) {
    __shared__ u64 wsum[TK_BLOCK / WAVE];
    __shared__ uint32_t s_last;
    const u64 t0 = (u64)blockIdx.x * TK_TILES_PER_BLOCK + threadIdx.x * 16;
    u64 v[16], sm = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
        const uint32_t c = t0 + j < ntiles ? tcnt[t0 + j] : 0u;
        v[j] = tk_better_of(c) | ((u64)tk_equal_of(c) << 32);
        sm += v[j];
    }
    u64 tot;
    u64 p = block_exclusive_scan<TK_BLOCK>(sm, wsum, &tot);  // per block < 2^32 keys: the halves cannot carry
#pragma unroll
    for (int j = 0; j < 16; ++j)
        if (t0 + j < ntiles) {
            toff[t0 + j] = p;
            p += v[j];
        }
    if (threadIdx.x == 0) {
        __hip_atomic_store(&bsum[2 * blockIdx.x], tot & 0xFFFFFFFFull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&bsum[2 * blockIdx.x + 1], tot >> 32, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        wait_mem();
        // release: this block's sums before its arrival; acquire: the last
        // arrival sees every block's sums
        s_last = __hip_atomic_fetch_add(arrive, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1u;
    }
    __syncthreads();
    if (!s_last) return;  // block-uniform
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // (every thread of the last block reads the sums)
    // the last workgroup: exclusive bases of the block sums, need and the bracket check
    const int G = (int)gridDim.x, per = (G + TK_BLOCK - 1) / TK_BLOCK, g0 = threadIdx.x * per;
    u64 sb = 0, se = 0;
    for (int j = 0; j < per; ++j)
        if (g0 + j < G) {
            sb += __hip_atomic_load(&bsum[2 * (g0 + j)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            se += __hip_atomic_load(&bsum[2 * (g0 + j) + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    u64 tb, te;
    u64 pb = block_exclusive_scan<TK_BLOCK>(sb, wsum, &tb);
    u64 pe = block_exclusive_scan<TK_BLOCK>(se, wsum, &te);
    for (int j = 0; j < per; ++j)
        if (g0 + j < G) {
            base[2 * (g0 + j)] = pb;
            base[2 * (g0 + j) + 1] = pe;
            pb += __hip_atomic_load(&bsum[2 * (g0 + j)], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            pe += __hip_atomic_load(&bsum[2 * (g0 + j) + 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    if (threadIdx.x == 0) {
        const bool ok = tb < k && k <= tb + te;
        meta[0] = ok ? k - tb : 0;
        meta[1] = ok ? 0 : 1;
        if (!ok && st) st->error = TK_ERR_BRACKET;
        *arrive = 0u;  // for the next call (every workgroup has arrived)
    }
}

// Pass 5: ordered compaction.  Each wave looks at 64 tiles at once (one per
// lane) and visits only those holding output keys.  Lane l owns keys
// [1024 t + 16 l, +16) of tile t, so a wave scan of the per-lane counts gives
// every kept key its slot in the tile's output range, which is contiguous:
// [bb + min(be, need), + #better + #kept ties).  Inside the range a key's
// slot is 32-bit arithmetic: with pb / pe the better / equal keys of the tile
// before it and cap = clamp(need - be, 0, 65535) the ties the tile may still
// take, a better key goes to pb + min(pe, cap), a tie with pe < cap to pb + pe.
// The pairs are staged in the wave's LDS and written out coalesced.
// Measured (rocprof averages, k = 2^27 / 2^29): nontemporal key loads 1436 /
// 2336 us against plain loads 1251 / 1934 (one box); four tiles a round
// against two 1261 / 2251 against 1304 / 2275 (another box).  Also measured
// and dropped there: nontemporal output stores (1433 / 2952) and issuing the
// next round's loads before placing this one (142 VGPRs; 1284 / 2279).
#ifndef KTH_TKW_TILES
#define KTH_TKW_TILES 4
#endif
constexpr int TKW_TILES = KTH_TKW_TILES;  // tiles a wave loads together in k_topk_write
template <bool ALIGNED, bool STAGED = false>
__global__ __launch_bounds__(TK_BLOCK) void k_topk_write(const uint32_t *__restrict__ keys, u64 n, u64 ntiles,
                                                         const int32_t *__restrict__ d_v, uint32_t flip,
                                                         const uint32_t *__restrict__ tcnt,
                                                         const u64 *__restrict__ toff, const u64 *__restrict__ bbase,
                                                         const u64 *__restrict__ meta, int32_t *__restrict__ vals,
                                                         int64_t *__restrict__ idx,
                                                         const uint32_t *__restrict__ tflags = nullptr, u64 ncov = 0) {
    __shared__ uint32_t s_val[TK_BLOCK / WAVE][TK_TILE];
    __shared__ uint16_t s_col[TK_BLOCK / WAVE][TK_TILE];
    if (meta[1]) return;
    const u64 need = meta[0];
    const uint32_t uv = key_of_i32((uint32_t)d_v[0]);
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    const u64 nw = (u64)gridDim.x * (TK_BLOCK / WAVE);
    const u64 t_from = STAGED && tk5_ok(tflags, d_v) ? ncov : 0;  // tiles below t_from: k_tk5_write
    // one round: up to TKW_TILES tiles of the wave's 64 (the next set bits of todo)
    struct Round {
        int src[TKW_TILES];  // lane (tile - tg) of each tile, -1 past the last
        uint32_t x[TKW_TILES][TK_KPL];
    };
    auto load_round = [&](Round &rd, u64 &todo, u64 tg) {
#pragma unroll
        for (int q = 0; q < TKW_TILES; ++q) {
            const bool has = todo != 0;  // wave-uniform
            rd.src[q] = has ? __builtin_ctzll(todo) : -1;
            if (has) todo &= todo - 1;
            const u64 tb = (tg + (u64)(has ? rd.src[q] : 0)) * TK_TILE;
            if (!has) {
#pragma unroll
                for (int j = 0; j < TK_KPL; ++j) rd.x[q][j] = 0u;
            } else if (ALIGNED && tb + TK_TILE <= n) {
#pragma unroll
                for (int r = 0; r < TK_KPL / 4; ++r) {
                    const uint4 *p4 = reinterpret_cast<const uint4 *>(keys + tb + (u64)lane * TK_KPL + 4 * r);
                    const uint4 v4 = *p4;
                    rd.x[q][4 * r] = v4.x;
                    rd.x[q][4 * r + 1] = v4.y;
                    rd.x[q][4 * r + 2] = v4.z;
                    rd.x[q][4 * r + 3] = v4.w;
                }
            } else {
#pragma unroll
                for (int j = 0; j < TK_KPL; ++j) {
                    const u64 i = tb + (u64)lane * TK_KPL + j;
                    rd.x[q][j] = i < n ? keys[i] : 0u;
                }
            }
        }
    };
    for (u64 tg = ((u64)blockIdx.x * (TK_BLOCK / WAVE) + w) * WAVE; tg < ntiles; tg += nw * WAVE) {
        if (tg + WAVE <= t_from) continue;  // wave-uniform
        // lane l: tile tg + l's bases and whether it holds output keys
        const u64 tl = tg + lane;
        uint32_t c_l = 0;
        u64 bb_l = 0, be_l = 0;
        if (tl < ntiles) {
            c_l = tcnt[tl];
            const u64 off = toff[tl], blk = tl / TK_TILES_PER_BLOCK;
            bb_l = bbase[2 * blk] + (off & 0xFFFFFFFFull);
            be_l = bbase[2 * blk + 1] + (off >> 32);
        }
        const bool act = tl >= t_from && (tk_better_of(c_l) != 0 || (tk_equal_of(c_l) != 0 && be_l < need));
        u64 todo = __ballot(act);
        // TKW_TILES tiles a round, all their loads in flight together (one
        // tile's 4 KiB a wave left the loads idle while the tile was placed
        // and copied out: k = 2^27 1398 -> 1346 us on one box, ~equal on
        // another).  (A layout in which each load instruction reads 1 KiB
        // contiguous, four wave scans a tile, measured no faster: 1377 vs
        // 1347 us at 2^27, 2339 vs 2322 at 2^29.)
        while (todo) {
            Round cur;
            load_round(cur, todo, tg);
#pragma unroll
            for (int q = 0; q < TKW_TILES; ++q) {
                const int src = cur.src[q];
                if (src < 0) break;  // wave-uniform
                const uint32_t c = (uint32_t)__builtin_amdgcn_readlane((int)c_l, src);
                const u64 bb = ((u64)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(bb_l >> 32), src) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)bb_l, src);
                const u64 be = ((u64)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(be_l >> 32), src) << 32) |
                               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)be_l, src);
                const u64 ce = tk_equal_of(c);
                const u64 room = be >= need ? 0 : need - be;               // ties this tile may take
                const uint32_t cap = (uint32_t)(room < 0xFFFFu ? room : 0xFFFFu);
                const uint32_t total = tk_better_of(c) + (uint32_t)(room < ce ? room : ce);  // output keys
                const u64 start = bb + (be < need ? be : need);             // and where they go
                const u64 tb = (tg + (u64)src) * TK_TILE;
                uint32_t mb = 0, me = 0;  // bit j: this lane's key j is better / equal
#pragma unroll
                for (int j = 0; j < TK_KPL; ++j) {
                    const bool in = tb + TK_TILE <= n || tb + (u64)lane * TK_KPL + j < n;
                    const uint32_t u = key_of_i32(cur.x[q][j]);
                    mb |= (uint32_t)(in && tk_better(u, uv, flip)) << j;
                    me |= (uint32_t)(in && u == uv) << j;
                }
                const uint32_t mine = (uint32_t)__popc(mb) | ((uint32_t)__popc(me) << 16);
                const uint32_t p = wave_incl_scan32(mine) - mine;
                if (mb | me) {
                    uint32_t pb = p & 0xFFFFu, pe = p >> 16;
#pragma unroll
                    for (int j = 0; j < TK_KPL; ++j) {
                        const uint32_t isb = (mb >> j) & 1u, ise = (me >> j) & 1u;
                        const uint32_t r = pb + min(pe, cap);
                        if (isb | (ise & (uint32_t)(pe < cap))) {
                            s_val[w][r] = cur.x[q][j];
                            s_col[w][r] = (uint16_t)(lane * TK_KPL + j);
                        }
                        pb += isb;
                        pe += ise;
                    }
                }
                __builtin_amdgcn_wave_barrier();
                for (uint32_t r = lane; r < total; r += WAVE) {  // coalesced copy-out
                    if (vals) vals[start + r] = (int32_t)s_val[w][r];
                    if (idx) idx[start + r] = (int64_t)(tb + s_col[w][r]);
                }
                __builtin_amdgcn_wave_barrier();  // copy-out reads before the next tile's staging
            }
        }
    }
}

// ------------------------------------------------ staged top-k (k_main<5/6>)
// Both kernels run on k_main's grid: workgroup b walks the tiles k_main's
// workgroup b streamed (t = b, b + G, ... < nfull), wave w its segment 4b + w,
// whose entries are the wave's wave-rows' staged keys back to back in that
// order (row words: counts).  Lane l takes one wave-row of each window of 64.

// The staged kernels' split: gridDim.x = G * S workgroups; workgroup
// (b, part) takes part `part` of the windows of k_main's workgroup b (its
// waves' segments), each window starting at the entry offsets k_main<5/6>
// recorded (seg.wstart), so no window waits for the one before it.
struct Tk5Part {
    u64 b, G, m, w_lo, w_hi;  // k_main workgroup, its grid, its wave-rows, windows [w_lo, w_hi)
};
__device__ __forceinline__ Tk5Part tk5_part(u64 nfull, u64 G) {
    Tk5Part t;
    t.G = G;
    t.b = blockIdx.x % G;
    const u64 part = blockIdx.x / G, S = gridDim.x / G;
    t.m = (nfull > t.b ? (nfull - 1 - t.b) / G + 1 : 0) * MAIN_UNROLL;
    const u64 nw = (t.m + WAVE - 1) / WAVE;
    t.w_lo = part * nw / S;
    t.w_hi = (part + 1) * nw / S;
    return t;
}
__device__ __forceinline__ uint32_t tk5_wstart(const uint32_t *wstart, uint32_t nwin, u64 b, int w, u64 win) {
    return win == 0 ? 0u : wstart[(b * (TK_BLOCK / WAVE) + (u64)w) * nwin + win];
}

// The entries of one wave-row, e in [0, c), KTH_TK5_BATCH loads in flight per
// lane (a rolled per-entry loop waited one memory round trip per entry; 4 in
// flight: one round trip per 4 entries); with sp, their positions are loaded
// beside them (f(x, p)).
#ifndef KTH_TK5_BATCH  // (16: k_tk5_write 56 / 121 / 400 us at k = 2^20 / 2^24 / 2^26; 4: 38 / 115 / 411)
#define KTH_TK5_BATCH 4
#endif
// (Three other k_tk5_write placements were measured and removed: staging each
// window's entries in LDS by coalesced chunks of 1024, 82 / 165 / 619 us at
// k = 2^20 / 2^24 / 2^26, and of 256 (1.25 KiB a wave), 137 / 252 / 982 us at
// k = 2^24 / 2^25 / 2^26 against this walk's 118 / 205 / 421; and taking the
// window's entries 64 at a time, one per lane, with each entry's wave-row
// found by a DPP max-scan over LDS-marked wave-row starts and its position from
// ballot prefix counts, 40 / 110 / 499 us against 38 / 112 / 427.  Timing-only
// builds at k = 2^26: no output stores 294 us, stores folded onto L2-resident
// slots 346, full 414.)
template <typename F>
__device__ __forceinline__ void tk5_entries(const int32_t *__restrict__ sv, const uint8_t *__restrict__ sp,
                                            uint32_t c, F &&f) {
    constexpr int B = KTH_TK5_BATCH;
    for (uint32_t e0 = 0; e0 < c; e0 += B) {
        int32_t x[B];
        uint8_t p[B];
#pragma unroll
        for (int q = 0; q < B; ++q) {
            x[q] = e0 + q < c ? sv[e0 + q] : 0;
            p[q] = sp && e0 + q < c ? sp[e0 + q] : (uint8_t)0;
        }
#pragma unroll
        for (int q = 0; q < B; ++q)
            if (e0 + q < c) f(x[q], p[q]);
    }
}

// A window's entries (the 64 wave-rows' staged keys, back to back from the
// window's first entry ws0) are brought into the wave's LDS in chunks of
// TK5_ECHUNK with coalesced loads, all of a lane's loads in flight at once
// (a lane walking its own wave-row's entries waited one memory round trip
// per few entries: k_tk5_count 165 us, k_tk5_write 394 us at k = 2^26).  Lane
// l then walks its wave-row's part of each chunk, [s0, s1) of the window,
// from LDS.  f(e, x) stages entry e (window-relative) of value x.
constexpr int TK5_ECHUNK = 1024;  // entries per wave and chunk
__device__ __forceinline__ uint32_t tk5_clip(uint32_t e, uint32_t c0, uint32_t cn) {  // window entry e in chunk [c0, c0 + cn)
    return e <= c0 ? 0u : (e - c0 < cn ? e - c0 : cn);
}
template <typename T, typename F>
__device__ __forceinline__ void tk5_chunk_load(const T *__restrict__ sv, uint32_t ws0, uint32_t c0, uint32_t cn,
                                               F &&f) {
    const int lane = threadIdx.x & (WAVE - 1);
    constexpr int PER = TK5_ECHUNK / WAVE;
    T x[PER];
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t e = (uint32_t)(q * WAVE + lane);
        x[q] = e < cn ? sv[ws0 + c0 + e] : (T)0;
    }
#pragma unroll
    for (int q = 0; q < PER; ++q) {
        const uint32_t e = (uint32_t)(q * WAVE + lane);
        if (e < cn) f(e, x[q]);
    }
}

// Per wave-row: #better | #equal << 16 -> wcnt; per row (the 4 wave-rows of
// its 4 waves, summed through LDS) -> tcnt.  Entries are read, the input is not.
// CHUNKED (dense windows, k >= n / 64): the window's entries come in by
// coalesced chunks (tk5_chunk_load); sparse windows walk each wave-row's few
// entries per lane (k = 2^20 / 2^24 / 2^26: lane walk 21.7 / 37.1 / 169 us,
// chunked 30.0 / 33.8 / 95 us).
template <bool CHUNKED>
__global__ __launch_bounds__(TK_BLOCK) void k_tk5_count(const int32_t *__restrict__ segv, u64 seg_cap,
                                                        const uint32_t *__restrict__ wstart, uint32_t nwin, u64 G,
                                                        const uint32_t *__restrict__ tflags, u64 nfull,
                                                        const int32_t *__restrict__ d_v, uint32_t flip,
                                                        uint32_t *__restrict__ wcnt, uint32_t *__restrict__ tcnt) {
    __shared__ uint32_t part[TK_BLOCK / WAVE][WAVE];
    __shared__ uint32_t ecode[TK_BLOCK / WAVE][CHUNKED ? TK5_ECHUNK : 1];  // an entry's #better | #equal << 16
    if (!tk5_ok(tflags, d_v)) return;  // grid-uniform
    const int32_t v = d_v[0];
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    const Tk5Part P = tk5_part(nfull, G);
    const int32_t *sv = segv + (P.b * (TK_BLOCK / WAVE) + w) * seg_cap;
    const uint32_t *ws = tflags + TF_W0 + (P.b * (TK_BLOCK / WAVE) + w) * rw_seg_words(nfull, G);  // this wave's row words
    uint32_t *ec = ecode[w];
    for (u64 win = P.w_lo; win < P.w_hi; ++win) {  // same trip count in the 4 waves
        const u64 j = win * WAVE + lane;
        const bool valid = j < P.m;
        const u64 r = (P.b + (j / MAIN_UNROLL) * P.G) * MAIN_UNROLL + j % MAIN_UNROLL;
        const uint32_t c = valid ? ws[j] : 0u;
        const uint32_t incl = wave_incl_scan32(c), s0 = incl - c;
        uint32_t word = 0;
        if constexpr (!CHUNKED) {
            uint32_t nb = 0, ne = 0;
            tk5_entries(sv + tk5_wstart(wstart, nwin, P.b, w, win) + s0, nullptr, c, [&](int32_t x, uint8_t) {
                nb += (flip == 0u ? x < v : x > v) ? 1u : 0u;
                ne += x == v ? 1u : 0u;
            });
            word = nb | ne << 16;
        } else {
            const uint32_t T = (uint32_t)__builtin_amdgcn_readlane((int)incl, WAVE - 1);  // the window's entries
            const uint32_t ws0 = tk5_wstart(wstart, nwin, P.b, w, win);
            for (uint32_t c0 = 0; c0 < T; c0 += TK5_ECHUNK) {  // wave-uniform
                const uint32_t cn = T - c0 < (uint32_t)TK5_ECHUNK ? T - c0 : (uint32_t)TK5_ECHUNK;
                tk5_chunk_load(sv, ws0, c0, cn, [&](uint32_t e, int32_t x) {
                    ec[e] = ((flip == 0u ? x < v : x > v) ? 1u : 0u) | (x == v ? 0x10000u : 0u);
                });
                __builtin_amdgcn_wave_barrier();
                const uint32_t lo = tk5_clip(s0, c0, cn), hi = tk5_clip(incl, c0, cn);
                for (uint32_t e = lo; e < hi; ++e) word += ec[e];
                __builtin_amdgcn_wave_barrier();  // the chunk's LDS is rewritten next
            }
        }
        if (valid) wcnt[r * (TK_BLOCK / WAVE) + w] = word;
        part[w][lane] = word;
        __syncthreads();
        if (w == 0 && valid) tcnt[r] = part[0][lane] + part[1][lane] + part[2][lane] + part[3][lane];
        __syncthreads();
    }
}

// The ordered compaction of the staged entries: a kept entry's slot is
// #better before it + min(#equal before it, need), as in k_topk_write; the
// wave-row's bases are its row's (toff, bbase) plus the earlier waves' counts
// in the row (wcnt), and the entries are in index order within the wave-row.
// The workgroup's 4 waves take the same 64 rows at a time (8 of k_main's
// 8-row tiles; wave w: quarter w of each row).  A tile's 8192 keys are
// consecutive, so its output is one contiguous range: the kept entries are
// placed in LDS at their offsets in their tile's range and written out
// coalesced (lane-scattered stores wrote ~64 cache lines an instruction:
// 300 us at k = 2^24).  A window whose output exceeds the stage is written
// directly.  The next window's row records are loaded while this one is
// placed and copied (the loop is a chain of dependent loads and barriers).
// output entries a workgroup stages: 4096 (24 KiB of LDS) for k <= n / 32,
// 6144 (36 KiB) above (a window of 64 Ki keys then holds ~k / n * 64 Ki outputs)
// (round 6: 6144 instead of 8192 for the large stage, 36.9 instead of 49.3 KiB
// of LDS: 4 workgroups a CU instead of 3; k_tk5_write at k = 2^26 404 -> 372
// us, whole call -1.8 %; a window of 64 Ki keys holds ~k / n * 64 Ki <= 4096
// outputs on the staged path, profiles/r6_topk_seg_store_ab.txt)
#ifndef KTH_TK5_STAGE_LARGE
#define KTH_TK5_STAGE_LARGE 6144
#endif
#ifndef KTH_TK5_STAGE_SMALL
#define KTH_TK5_STAGE_SMALL 4096
#endif
constexpr int TK5_STAGE_SMALL = KTH_TK5_STAGE_SMALL, TK5_STAGE_LARGE = KTH_TK5_STAGE_LARGE;
struct Tk5Rec {                  // one lane's row records of a window
    uint32_t c, tc;              // the wave-row's entries; the row's count word
    u64 off, b0, b1;             // toff[r], bbase[2 blk], bbase[2 blk + 1]
    uint4 wc;                    // the row's four wave-row words
};
__device__ __forceinline__ Tk5Rec tk5_rec(const uint32_t *__restrict__ ws, const uint32_t *__restrict__ wcnt,
                                          const uint32_t *__restrict__ tcnt, const u64 *__restrict__ toff,
                                          const u64 *__restrict__ bbase, u64 r, u64 j, bool valid) {
    Tk5Rec x{0u, 0u, 0ull, 0ull, 0ull, make_uint4(0u, 0u, 0u, 0u)};
    if (valid) {
        const u64 blk = r / TK_TILES_PER_BLOCK;
        x.c = ws[j];
        x.tc = tcnt[r];
        x.off = toff[r];
        x.b0 = bbase[2 * blk];
        x.b1 = bbase[2 * blk + 1];
        x.wc = *reinterpret_cast<const uint4 *>(wcnt + r * (TK_BLOCK / WAVE));
    }
    return x;
}
template <int TK5_STAGE>
__global__ __launch_bounds__(TK_BLOCK) void k_tk5_write(const int32_t *__restrict__ segv,
                                                        const uint8_t *__restrict__ segp, u64 seg_cap,
                                                        const uint32_t *__restrict__ wstart, uint32_t nwin, u64 G,
                                                        const uint32_t *__restrict__ tflags, u64 nfull,
                                                        const int32_t *__restrict__ d_v, uint32_t flip,
                                                        const uint32_t *__restrict__ wcnt,
                                                        const uint32_t *__restrict__ tcnt,
                                                        const u64 *__restrict__ toff, const u64 *__restrict__ bbase,
                                                        const u64 *__restrict__ meta, int32_t *__restrict__ vals,
                                                        int64_t *__restrict__ idx) {
    __shared__ int32_t s_val[TK5_STAGE];
    __shared__ uint16_t s_loc[TK5_STAGE];  // key index within its tile: u << 10 | w << 8 | position
    __shared__ u64 s_lo[8];                // tile i of the window: its first output slot
    __shared__ uint32_t s_off[9];          // and its first stage entry (s_off[8]: the window's total)
    if (!tk5_ok(tflags, d_v) || meta[1]) return;  // grid-uniform
    const u64 need = meta[0];
    const int32_t v = d_v[0];
    const int lane = threadIdx.x & (WAVE - 1), w = threadIdx.x / WAVE;
    const Tk5Part P = tk5_part(nfull, G);
    const u64 b = P.b, m = P.m;  // m: a multiple of 8, whole tiles
    const u64 sbase = (b * (TK_BLOCK / WAVE) + w) * seg_cap;
    static_assert(MAIN_UNROLL == 8 && WAVE / MAIN_UNROLL == 8 && TK5_WIN_TILES * MAIN_UNROLL == WAVE,
                  "a window of 64 rows is 8 tiles");
    auto row_of = [&](u64 j) { return (b + (j / MAIN_UNROLL) * G) * MAIN_UNROLL + j % MAIN_UNROLL; };
    auto from = [](u64 x, int l) {  // x of lane l (per-lane l: bpermute)
        return ((u64)(uint32_t)__shfl((int)(uint32_t)(x >> 32), l, WAVE) << 32) |
               (uint32_t)__shfl((int)(uint32_t)x, l, WAVE);
    };
    const uint32_t *ws = tflags + TF_W0 + (b * (TK_BLOCK / WAVE) + w) * rw_seg_words(nfull, G);  // this wave's row words
    Tk5Rec nx = tk5_rec(ws, wcnt, tcnt, toff, bbase, row_of(P.w_lo * WAVE + lane), P.w_lo * WAVE + lane,
                        P.w_lo * WAVE + lane < m);
    for (u64 win = P.w_lo; win < P.w_hi; ++win) {  // same trip count in the 4 waves
        const u64 j0 = win * WAVE, j = j0 + lane;
        const bool valid = j < m;
        const u64 r = row_of(j);
        const Tk5Rec cur = nx;
        if (win + 1 < P.w_hi) nx = tk5_rec(ws, wcnt, tcnt, toff, bbase, row_of(j + WAVE), j + WAVE, j + WAVE < m);
        const uint32_t c = cur.c;
        const uint32_t wbase = tk5_wstart(wstart, nwin, b, w, win);  // the window's first entry
        const uint32_t start = wbase + wave_incl_scan32(c) - c;
        // this row's bases, and this wave-row's (after the earlier quarters' counts)
        const u64 rb = cur.b0 + (cur.off & 0xFFFFFFFFull), re = cur.b1 + (cur.off >> 32);
        u64 bb = rb, be = re;
        const uint32_t wcs[4] = {cur.wc.x, cur.wc.y, cur.wc.z, cur.wc.w};
#pragma unroll
        for (int q = 0; q < TK_BLOCK / WAVE; ++q)
            if (q < w) {
                bb += wcs[q] & 0xFFFFu;
                be += wcs[q] >> 16;
            }
        // each tile's output range (its first row's start to its last row's
        // end); every wave computes the same table, wave 0 publishes it
        const u64 lo = rb + (re < need ? re : need);
        const u64 e2 = re + tk_equal_of(cur.tc);
        const u64 hi = rb + tk_better_of(cur.tc) + (e2 < need ? e2 : need);
        const u64 tlo = from(lo, lane & ~7), thi = from(hi, lane | 7);
        const uint32_t len = (lane & 7) == 0 && valid ? (uint32_t)(thi - tlo) : 0u;
        const uint32_t li = wave_incl_scan32(len);  // lanes 0, 8, .., 56 hold the tiles' lengths
        const uint32_t total = (uint32_t)__builtin_amdgcn_readlane((int)li, WAVE - 1);
        const uint32_t toff_s = (uint32_t)__shfl((int)(li - len), lane & ~7, WAVE);  // this lane's tile's first entry
        if (w == 0 && (lane & 7) == 0) {
            s_lo[lane >> 3] = tlo;
            s_off[lane >> 3] = li - len;
        }
        if (w == 0 && lane == 0) s_off[8] = total;
        const bool staged = total <= (uint32_t)TK5_STAGE;  // block-uniform
        const uint16_t loc0 = (uint16_t)((lane & 7) << 10 | w << 8);
        const u64 i0 = r * TK_TILE + (u64)w * (TK_TILE / (TK_BLOCK / WAVE));  // the wave-row's first key
        auto place = [&](int32_t x, uint8_t p) __attribute__((always_inline)) {
            // (selects, not branches: with ++bb / ++be in branches the compiler
            // kept the pair in scratch and incremented it through a pointer)
            const bool isb = flip == 0u ? x < v : x > v, ise = x == v;
            const bool keep = isb || (ise && be < need);
            const u64 pos = bb + (be < need ? be : need);  // == bb + be for a kept equal entry
            bb += isb ? 1u : 0u;
            be += ise ? 1u : 0u;
            if (keep) {
                if (staged) {
                    const uint32_t s = toff_s + (uint32_t)(pos - tlo);
                    s_val[s] = x;
                    s_loc[s] = (uint16_t)(loc0 | p);
                } else {
                    if (vals) vals[pos] = x;
                    if (idx) idx[pos] = (int64_t)(i0 + p);
                }
            }
        };
        tk5_entries(segv + sbase + start, segp + sbase + start, c, place);
        if (staged) {  // coalesced copy-out, tile by tile
            __syncthreads();
            const u64 tile0 = (b + (j0 / MAIN_UNROLL) * G) * MAIN_UNROLL * TK_TILE;  // the window's first tile's first key
            for (uint32_t s = threadIdx.x; s < total; s += TK_BLOCK) {
                int i = 0;
#pragma unroll
                for (int q = 1; q < 8; ++q) i += s >= s_off[q] ? 1 : 0;
                const u64 gp = s_lo[i] + (s - s_off[i]);
                if (vals) vals[gp] = s_val[s];
                if (idx) idx[gp] = (int64_t)(tile0 + (u64)i * G * MAIN_UNROLL * TK_TILE + s_loc[s]);
            }
        }
        __syncthreads();  // the stage and the tile table are reused by the next window
    }
}

}  // namespace kth
