// gs_render.hip — front-to-back blend (forward), back-to-front gradient
// replay (backward) and the apply_weights back-projection, for gfx950.
//
// Reference: renderCUDA fwd (forward.cu:261-379), renderCUDA bwd
// (backward.cu:399-557), renderCUDA_apply_weights (apply_weights.cu:239-356).
// The per-pixel arithmetic, thresholds and the (1-based) contributor
// bookkeeping are the reference's; the work decomposition is not:
//
//  * one 64-lane wave owns one 8x8 quadrant of a 16x16 tile (lane = pixel).
//    Tile lists stay the reference's 16x16 bins, but each wave streams the
//    list in batches of 64, tests every entry against its quadrant with a
//    conservative analytic bound (cull_keep: min of the conic quadratic over
//    the quadrant box vs. the alpha >= 1/255 level), and compacts survivors
//    into LDS with a ballot/popcount prefix.  Skipped entries could not pass
//    the reference's `power > 0` / `alpha < 1/255` tests for any pixel of the
//    quadrant, so the output (including n_contrib) is unchanged;
//  * the forward waves are independent workgroups (no block barrier, a wave
//    retires as soon as its 64 pixels saturate);
//  * the backward also runs one independent wave per quadrant, starting at
//    the quadrant's largest n_contrib instead of the list end; it factors the
//    reference's per-pixel gradient terms into nine per-pixel sums,
//    reduce-scatters them across the wave four entries at a time with the
//    gfx950 lane swaps, and writes ONE 48-byte record per (kept entry,
//    quadrant) with plain stores.  No float atomics: the per-Gaussian sum
//    happens in gs_backward.hip in a fixed order, so the backward is bitwise
//    reproducible.
#include <string.h>

#include "gs_common.h"
#include "gs_internal.h"

namespace gs {

// =====================================================================
// forward: one wave per 8x8 quadrant
// =====================================================================
// exp used by the blend loops: gs_exp (gs_common.h), the fixed IEEE sequence the
// oracle evaluates bit for bit, so every alpha and blend decision is the oracle's
__device__ __forceinline__ float blend_exp(float x) { return gs_exp(x); }

// test hook (gs_blend_exp): the blend exp over an array, four-wide as the blend loops use it
__global__ __launch_bounds__(256) void k_blend_exp(long long n, const float* __restrict__ x, float* __restrict__ y) {
    const long long i = 4 * ((long long)blockIdx.x * 256 + threadIdx.x);
    if (i + 3 < n) {
        const f4v r = gs_exp4(f4v{x[i], x[i + 1], x[i + 2], x[i + 3]});
        y[i] = r.x;
        y[i + 1] = r.y;
        y[i + 2] = r.z;
        y[i + 3] = r.w;
    } else {
        for (long long k = i; k < n; ++k) y[k] = gs_exp(x[k]);
    }
}

// The per-(pixel, Gaussian) test shared by the forward, the backward replay
// and apply_weights: identical code (contraction pinned), hence identical
// skip decisions (forward.cu:336-348, backward.cu:491-501).  Branch-free:
// G and alpha are always defined; the result is false where the reference
// skips (`power > 0` or `alpha < 1/255`; NaN compares as the reference's).
__device__ __forceinline__ bool pixel_alpha(float2 xy, float4 co, float pfx, float pfy, float& dx, float& dy,
                                            float& G, float& alpha) {
#pragma clang fp contract(off)
    dx = xy.x - pfx;
    dy = xy.y - pfy;
    const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
    G = blend_exp(power);
    alpha = fminf(0.99f, co.w * G);
    return !(power > 0.0f) && !(alpha < 1.0f / 255.0f);
}

// (diagnostics) where this wave runs: HW_ID (wave slot, SIMD, CU, SH, SE) | XCC_ID << 32
__device__ __forceinline__ uint64_t wave_location() {
    const uint32_t hw = __builtin_amdgcn_s_getreg(4 | (31 << 11));   // HW_REG_HW_ID, bits [31:0]
    const uint32_t xcc = __builtin_amdgcn_s_getreg(20 | (15 << 11)); // HW_REG_XCC_ID, bits [15:0]
    return (uint64_t)xcc << 32 | hw;
}

constexpr int kRound = kBlendRound;  // list entries per round: 4 per lane

constexpr int kGroup = 4;    // blend entries per unrolled step (LDS is padded to a multiple)
constexpr int kFcmpOGT = 2;  // llvm::CmpInst::FCMP_OGT, the predicate of __builtin_amdgcn_fcmpf

// One list entry as gathered from the geometry buffer.
struct Entry {
    float2 xy;
    float4 co;
    float4 f;  // rgb + depth
};

__device__ __forceinline__ Entry gather_entry(const Splat* splat, uint32_t id) {
    const Splat* sp = splat + id;
    Entry e;
    e.xy = sp->xy;
    e.co = sp->co;
    e.f = sp->rgbd;
    return e;
}

// pixel_alpha for four consecutive entries: two packed streams (f4v ops split
// into pairs of v_pk_* instructions), bit-identical to four pixel_alpha calls.
// Operands arrive pre-negated where a subtraction would otherwise not pack
// (v_pk_add_f32 has no subtract form): (nca, ncb, ncc) = -conic, (npx, npy) = -pixel, and
//   x + npx == x - px,   0.5 ((nca dx) dx + (ncc dy) dy) + (ncb dx) dy == -0.5 (a dx^2 + c dy^2) - (b dx) dy
// exactly (negation is exact and commutes with rounding, a - b == a + (-b) in IEEE arithmetic; the
// one sign difference, +0 for -0 when a dx^2 == -c dy^2, gives the same G and the same tests).  With
// +conic.x/z the compiler turned -0.5 * s + t into t - 0.5 * s: four unpacked subtractions per group.
__device__ __forceinline__ void pixel_alpha4(f4v x, f4v y, f4v ncx, f4v ncy, f4v ncz, f4v op, float npx, float npy,
                                             f4v& dx, f4v& dy, f4v& G, f4v& alpha, bool (&ok)[4]) {
#pragma clang fp contract(off)
    dx = x + npx;
    dy = y + npy;
    const f4v power = 0.5f * (ncx * dx * dx + ncz * dy * dy) + ncy * dx * dy;
    G = gs_exp4(power);
    const f4v oG = op * G;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        alpha[u] = fminf(0.99f, oG[u]);
        ok[u] = !(power[u] > 0.0f) && !(alpha[u] < 1.0f / 255.0f);
    }
}

// The sequential part of blend_step once the entry's alpha test is done, on a
// signed transmittance: Ts = T while the pixel is live, Ts = -T once it has
// saturated (the reference's `done`), so the whole per-entry chain is VALU:
//   a' = ok ? alpha : 0                 (a skipped entry multiplies T by 1, exactly)
//   tT = Ts * (1 - a')                  (<= 0 once saturated: 1 - a' >= 0.01)
//   use-or-skip <=> tT >= 1e-4          (live and !stop, forward.cu:350-354)
//   Ts = (tT >= 1e-4) ? tT : -|Ts|       (a stop keeps T and marks the pixel done)
//   Tw = (tT >= 1e-4) ? Ts : 0          (the T a use blends with; 0 for stop/done)
// and the sums in the reference's association, `C += f * alpha * T` as nvcc's
// default fmad contracts it (forward.cu:355-357): C = fma(f * a', Tw, C), two
// packed pairs (C0, C1), (C2, D) against the entry's (r, g), (b, depth); the
// same products go into the segment-local sums (L01, L2) of the checkpoints.  A
// skipped entry adds (f * 0) * T = 0, a stopped or saturated one f a' * 0.
// T, the sums and `last` are bit-identical to the oracle's.  Returns
// w = a' Tw, > 0 exactly when the entry is blended (the caller's vote).
// AUX: the aux grey m in {0, 1} (m_on: m = 1, wave-uniform) composited the same way — a recolor blend with
// colour (m, m, m) computes fma(m a', Tw, C) on each channel, which is fma(a', Tw, C) for m = 1 and C for
// m = 0 (C + (+0) Tw, C >= +0) — so Cm + T bg is that render's image, bit for bit.
template <bool SEG = true, bool AUX = false>
__device__ __forceinline__ float blend_chain(float a, float4 fe, uint32_t pos, float& Ts, f2v& C01, f2v& C2D,
                                           f2v& L01, float& L2, uint32_t& last, bool m_on = false,
                                           float* Cm = nullptr) {
#pragma clang fp contract(off)
    const float tT = Ts * (1.0f - a);
    const bool go = tT >= 0.0001f;
    const float Tw = go ? Ts : 0.0f;
    Ts = go ? tT : -fabsf(Ts);
    const f2v a2 = {a, a}, T2 = {Tw, Tw};
    const f2v fa01 = f2v{fe.x, fe.y} * a2, fa2d = f2v{fe.z, fe.w} * a2;
    C01 = __builtin_elementwise_fma(fa01, T2, C01);
    C2D = __builtin_elementwise_fma(fa2d, T2, C2D);
    if constexpr (AUX) *Cm = m_on ? __builtin_fmaf(a, Tw, *Cm) : *Cm;
    if constexpr (SEG) {
        L01 = __builtin_elementwise_fma(fa01, T2, L01);  // the segment's own colour sum (backward start)
        L2 = __builtin_fmaf(fa2d.x, Tw, L2);
    }
    const float w = a * Tw;
    last = w > 0.0f ? pos : last;
    return w;
}

// Dispatch order of the blend: tiles by list length, longest first (coarse
// log-scale classes; the order inside a class is whatever the LDS atomics give
// — it only decides placement).  The longest lists are then dealt first, one
// per SIMD, instead of landing next to each other (they cluster in the image).
__global__ __launch_bounds__(1024) void k_tile_order(const uint2* __restrict__ ranges, int tiles,
                                                     uint32_t* __restrict__ order) {
    constexpr int kClasses = 64;
    __shared__ uint32_t cnt[kClasses];
    const int tid = threadIdx.x;
    if (tid < kClasses) cnt[tid] = 0u;
    __syncthreads();
    auto cls = [](uint32_t len) { return min(kClasses - 1, (int)(__log2f((float)len + 1.0f) * 3.0f)); };
    // (each thread's ranges loaded at once: grids up to 16 x 1024 tiles in one round trip)
    constexpr int kPer = 16;
    uint32_t len[kPer];
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int t = tid + 1024 * i;
        const uint2 r = t < tiles ? ranges[t] : make_uint2(0u, 0u);
        len[i] = r.y - r.x;
    }
    for (int t = tid + 1024 * kPer; t < tiles; t += 1024) {  // (larger grids)
        const uint2 r = ranges[t];
        atomicAdd(&cnt[cls(r.y - r.x)], 1u);
    }
#pragma unroll
    for (int i = 0; i < kPer; ++i)
        if (tid + 1024 * i < tiles) atomicAdd(&cnt[cls(len[i])], 1u);
    __syncthreads();
    if (tid == 0) {  // start of each class, longest class first
        uint32_t run = 0;
        for (int c = kClasses - 1; c >= 0; --c) {
            const uint32_t n = cnt[c];
            cnt[c] = run;
            run += n;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kPer; ++i) {
        const int t = tid + 1024 * i;
        if (t < tiles) order[atomicAdd(&cnt[cls(len[i])], 1u)] = (uint32_t)t;
    }
    for (int t = tid + 1024 * kPer; t < tiles; t += 1024) {
        const uint2 r = ranges[t];
        order[atomicAdd(&cnt[cls(r.y - r.x)], 1u)] = (uint32_t)t;
    }
}

// The replay's work items of a quadrant: one per 128-position segment of its window, all in the class
// of the quadrant's kept entries per segment (heaviest class first: the hardware dispatches
// workgroups in order, so the longest items start first and the short ones fill the end).  One atomic
// per wave, each class's counter on its own cache line (same-address atomics serialise).
__device__ __forceinline__ int item_class(uint32_t kept) { return kept >= 64 ? 0 : kept >= 40 ? 1 : kept >= 20 ? 2 : 3; }
// List x (the forward's XCD group, rank & 7) keeps a tile's four quadrants together (see kItemXcds).
__device__ __forceinline__ void emit_items(const RenderArgs& a, int tile, int quad, int x, uint32_t nseg,
                                           uint32_t nkept, int lane) {
    const int c = item_class(nkept / nseg);
    uint32_t base = 0;
    if (lane == 0) {
        base = atomicAdd(&a.bwd_count[item_count_at(c, x)], nseg);
        atomicMax(&a.bwd_count[item_max_at(c)], base + nseg);
    }
    base = __shfl(base, 0);
    uint2* list = a.bwd_items + (size_t)(c * kItemXcds + x) * a.item_cap;
    for (uint32_t k = lane; k < nseg; k += 64) list[base + k] = make_uint2((uint32_t)tile, (k << 2) | (uint32_t)quad);
}

// BWD: the backward's bookkeeping (checkpoints, blended bits, touched bytes, the replay's work list);
// a forward no backward follows (gs_params.forward_only) runs without it.  AUX (with BWD): the aux grey
// composited beside the colour (gs_params.aux_mask) into aux_out.  Without BWD, a recolor render whose
// colours are its source forward's aux grey (*aux_match == 0) composes its image from that forward's sums.
template <bool BWD, bool AUX = false>
__global__ __launch_bounds__(64, 3) void k_render_fwd(RenderArgs a) {
    // XCD-aware: blocks b, b+8, b+16, b+24 (one XCD under the round-robin dealing) take the four
    // quadrants of one tile, so the tile's list and its Splat gathers are fetched into one L2;
    // tiles in k_tile_order's order, longest list first
    const int x8 = blockIdx.x & 7, j8 = blockIdx.x >> 3;
    const int quad = j8 & 3, rank = (j8 >> 2) * 8 + x8;
    if (rank >= a.gx * a.gy) return;
    const int tile = (int)a.tile_order[rank];
    const int qidx = 4 * tile + quad;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int lane = threadIdx.x;
    const int bx0 = tx * kTile + (quad & 1) * kQuad, by0 = ty * kTile + (quad >> 1) * kQuad;
    const int px = bx0 + (lane & 7), py = by0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;
    if constexpr (!BWD) {
        if (a.aux_match && *a.aux_match == 0u) {  // (one flag for the whole grid: a uniform branch)
            if (inside) {  // the bits the blend below would produce (forward.cu:376, as at the end)
                const size_t pix = (size_t)a.W * py + px;
                const size_t HW = (size_t)a.W * a.H;
                const float T = a.final_T_src[pix];
                const float2 av = a.aux_src[pix];
                const float bg0 = a.bg[0], bg1 = a.bg[1], bg2 = a.bg[2];  // (all three before the stores)
                a.out_color[pix] = __builtin_fmaf(T, bg0, av.x);
                a.out_color[HW + pix] = __builtin_fmaf(T, bg1, av.x);
                a.out_color[2 * HW + pix] = __builtin_fmaf(T, bg2, av.x);
                a.out_depth[pix] = av.y;
            }
            return;
        }
    }

    // the round's kept entries, one array per field: a pair of consecutive entries' field is one
    // 16-B read, the operands of two packed instructions (pixel_alpha4)
    // (kRoundLds: the round's kept entries, the <= 7 pad slots that start its second segment on a
    // whole blend step, the end padding and the prefetch's overshoot)
    constexpr int kRoundLds = kRound + 4 * kGroup;
    __shared__ __attribute__((aligned(16))) float s_x[kRoundLds], s_y[kRoundLds];
    __shared__ __attribute__((aligned(16))) float s_cx[kRoundLds], s_cy[kRoundLds], s_cz[kRoundLds], s_op[kRoundLds];
    __shared__ float4 s_rgbd[kRoundLds];
    // (AUX) kept entries' aux bit: the sign of the gathered depth (Splat), no load of its own
    __shared__ __attribute__((aligned(16))) uint8_t s_mb[AUX ? kRoundLds : 4];
    __shared__ __attribute__((aligned(16))) uint32_t s_pos[kRoundLds];
    __shared__ uint32_t s_gused[kRoundLds / kGroup];  // per blend group: bit u = entry u was blended
    __shared__ uint32_t s_id[kRoundLds];              // the kept entries' Gaussians (the touched bytes)

    const uint2 range = a.ranges[tile];
    uint64_t* used = a.used + (size_t)used_base(range.x, tile) * 4 + quad;
    float Ts = inside ? 1.0f : -1.0f;  // signed transmittance (blend_chain): < 0 once done
    f2v C01 = {0.f, 0.f}, C2D = {0.f, 0.f};  // (C0, C1), (C2, depth)
    f2v L01 = {0.f, 0.f};                    // this segment's own colour sum (C0, C1), C2
    float L2 = 0.f;
    float Cm = 0.f;  // (AUX) the aux grey sum
    uint32_t last = 0;
    const uint64_t t_start = a.diag ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint64_t c_start = a.diag ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t c_blend = 0;
    uint32_t diag_kept = 0, diag_rounds = 0;

    // Software pipeline over rounds of 256 entries: the ids run two rounds
    // ahead and the geometry gathers one round ahead of the blend, so a
    // round's loads are in flight while the previous round blends.
    // Out-of-range slots load the list's last entry and are dropped by the cull
    // (unconditional loads, clamped into the list: the compiler can then count them in vmcnt
    // waits instead of draining every outstanding access).
    const uint32_t k_last = range.y > range.x ? range.y - 1 : 0u;
    // (an empty list reads nothing: its slot of the binning buffer need not hold a valid id; Gaussian 0
    // is gathered instead, P > 0 whenever the blend runs)
    const bool list_empty = range.y <= range.x;
    auto load_ids = [&](uint32_t b, uint32_t (&ids)[4]) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t k = b + 64 * i + lane;
            const uint32_t kc = k < range.y ? k : k_last;
            // (id-only lists come from forward-only binnings: only the !BWD blend reads them)
            if constexpr (BWD) ids[i] = list_empty ? 0u : a.point_pairs[kc].x;
            else ids[i] = list_empty ? 0u : a.point_ids ? a.point_ids[kc] : a.point_pairs[kc].x;
        }
    };
    uint32_t ids[4], cid[4];  // cid: the ids of the entries in `cur` (the touched bytes at the round's end)
    Entry cur[4];
    // (gs_render_recolor: a forward-only blend over another render's binning with its own colours)
    const auto gather = [&](uint32_t id) {
        Entry e = gather_entry(a.splat, id);
        if constexpr (!BWD) {
            if (a.colors) {
                e.f.x = a.colors[3 * (size_t)id];
                e.f.y = a.colors[3 * (size_t)id + 1];
                e.f.z = a.colors[3 * (size_t)id + 2];
            }
        }
        return e;
    };
    load_ids(range.x, ids);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        cur[i] = gather(ids[i]);
        cid[i] = ids[i];
    }
    load_ids(range.x + kRound, ids);

    // checkpoint of segment k of this quadrant: slot ckpt_base + k, quadrant `quad`: (T after it, its own
    // colour sum)
    float4* ckpt = a.ckpt + ((size_t)ckpt_base(range.x, tile) * 4 + quad) * 64 + lane;
    const auto put_ckpt = [&](int k) {
        if constexpr (BWD) {
            ckpt[(size_t)k * 256] = make_float4(fabsf(Ts), L01.x, L01.y, L2);
            L01 = f2v{0.f, 0.f};
            L2 = 0.f;
        }
    };
    int seg_done = -1;  // last segment whose checkpoint is pending (the round just blended)
    uint64_t c_cull = 0;
    // The round's global stores (checkpoint, the previous round's blended bits) are issued after
    // the next round's gathers: stores count in vmcnt, and one issued just before the cull would
    // make the cull's wait for the gathers wait for the store too.
    uint64_t pend_word = 0;    // lane i < 4: word i of the previous round's blended bits
    int pend_rel = -1;         // that round's first list position (-1: none)
    auto store_words = [&]() {
        if (BWD && pend_rel >= 0 && lane < kRound / 64 && pend_rel + 64 * lane < (int)(range.y - range.x))
            used[(size_t)(pend_rel / 64 + lane) * 4] = pend_word;  // (the list's own words only)
    };
    for (uint32_t b = range.x; b < range.y; b += kRound) {
        if (!__any(Ts > 0.0f)) break;
        const uint64_t r0 = a.diag ? __builtin_amdgcn_s_memtime() : 0;
        // cull against the quadrant, compact survivors in list order (i-major, lane-minor); the
        // round's second segment (positions kSegLen..) starts at slot n_mid, on a whole group, behind
        // <= 3 pad slots that blend nothing — the checkpoint between the two segments is taken between
        // the blend loops over them
        int nk = 0, n_mid = 0;
        int kslot[4];  // compacted slot of this lane's entry i (-1: culled)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            if (i == kSegLen / 64) {
                n_mid = (nk + kGroup - 1) & ~(kGroup - 1);
                if (lane < n_mid - nk) {
                    const int slot = nk + lane;
                    s_x[slot] = 0.f;
                    s_y[slot] = 0.f;
                    s_cx[slot] = 0.f;
                    s_cy[slot] = 0.f;
                    s_cz[slot] = 0.f;
                    s_op[slot] = 0.f;
                    s_rgbd[slot] = make_float4(0.f, 0.f, 0.f, 0.f);
                    if constexpr (AUX) s_mb[slot] = 0;
                    s_pos[slot] = 0u;
                }
                nk = n_mid;
            }
            const uint32_t k = b + 64 * i + lane;
            const bool keep = k < range.y && cull_keep(cur[i].xy, cur[i].co, (float)bx0, (float)by0);
            const uint64_t km = __ballot(keep);
            kslot[i] = keep ? nk + __popcll(km & lanemask_lt()) : -1;
            if (keep) {
                const int slot = kslot[i];
                s_x[slot] = cur[i].xy.x;
                s_y[slot] = cur[i].xy.y;
                s_cx[slot] = -cur[i].co.x;  // (negated: pixel_alpha4)
                s_cy[slot] = -cur[i].co.y;  // (negated: pixel_alpha4)
                s_cz[slot] = -cur[i].co.z;
                s_op[slot] = cur[i].co.w;
                // (|depth|: the sign is the aux bit, Splat; every variant strips it — a recolor may blend
                // the lists of a forward that had an aux mask)
                s_rgbd[slot] = make_float4(cur[i].f.x, cur[i].f.y, cur[i].f.z, fabsf(cur[i].f.w));
                if constexpr (AUX) s_mb[slot] = cur[i].f.w < 0.0f ? 1 : 0;
                s_pos[slot] = k - range.x + 1;  // 1-based contributor index (forward.cu:331)
                s_id[slot] = cid[i];
            }
            nk += __popcll(km);
        }
        // pad to a whole group with entries that fail alpha >= 1/255 everywhere
        if (lane < kGroup) {
            s_x[nk + lane] = 0.f;
            s_y[nk + lane] = 0.f;
            s_cx[nk + lane] = 0.f;
            s_cy[nk + lane] = 0.f;
            s_cz[nk + lane] = 0.f;
            s_op[nk + lane] = 0.f;
            s_rgbd[nk + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
            if constexpr (AUX) s_mb[nk + lane] = 0;
            s_pos[nk + lane] = 0u;
        }
        diag_kept += nk;
        diag_rounds += 1;
        if (a.diag) c_cull += __builtin_amdgcn_s_memtime() - r0;
        // next round's gathers and the round after's ids, in flight during the blend
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            cur[i] = gather(ids[i]);
            cid[i] = ids[i];
        }
        load_ids(b + 2 * kRound, ids);
        if (seg_done >= 0) put_ckpt(seg_done);  // the previous segment's: the replay's start
        seg_done = (int)((b - range.x) / kSegLen);  // the round's first segment
        // the round's second segment exists: its checkpoint follows the first one's at n_mid (-1: none,
        // or taken)
        const int n_mid_slot = n_mid;
        if (range.y - b <= (uint32_t)kSegLen) n_mid = -1;
        const auto take_mid = [&]() {
            put_ckpt(seg_done);
            ++seg_done;
            n_mid = -1;
        };
        store_words();
        if (BWD) {
            s_gused[lane] = 0u;  // (groups past an early exit stay 0)
            if (lane < kRoundLds / kGroup - 64) s_gused[64 + lane] = 0u;
        }
        __syncthreads();

        const uint64_t c0 = a.diag ? __builtin_amdgcn_s_memtime() : 0;
        // The alpha-test operands of a group are read one group ahead (ping-pong A/B, no register
        // copies), so their LDS latency overlaps the previous group's blend.  A group's colour and
        // position reads are issued before the next group's prefetch: LDS reads retire in order, so
        // waiting for them does not wait for the prefetch.  Reads past nk land in the padding or
        // stale slots (index < kRound + kGroup) and are never used.
        struct AlphaOps { f4v x, y, cx, cy, cz, op; };
        // (AUX: mb, the group's four aux bits, read with the colours — before the next group's alpha
        // prefetch, so the wait for it is the colours' wait and does not drain the prefetch)
        struct ColourOps { float4 rgbd[kGroup]; uint32_t pos[kGroup]; uint32_t mb; };
        const auto load_alpha = [&](int j, AlphaOps& g) {
            const auto ld4 = [&](const float* f) { return *reinterpret_cast<const f4v*>(f + j); };
            g.x = ld4(s_x);
            g.y = ld4(s_y);
            g.cx = ld4(s_cx);
            g.cy = ld4(s_cy);
            g.cz = ld4(s_cz);
            g.op = ld4(s_op);
        };
        const auto load_colour = [&](int j, ColourOps& c) {
            // (mb first: the first entry's chain needs it, and LDS reads retire in order)
            if constexpr (AUX) c.mb = *reinterpret_cast<const uint32_t*>(s_mb + j);
#pragma unroll
            for (int u = 0; u < kGroup; ++u) {
                c.rgbd[u] = s_rgbd[j + u];
                c.pos[u] = s_pos[j + u];
            }
        };
        const auto blend_group = [&](int j, const AlphaOps& g, const ColourOps& c) {
            f4v dx4, dy4, G4, al;
            bool ok[4];
            // (AUX: the group's four aux bits, the same for every lane: one scalar word)
            uint32_t mb = 0u;
            if constexpr (AUX) mb = __builtin_amdgcn_readfirstlane(c.mb);
            pixel_alpha4(g.x, g.y, g.cx, g.cy, g.cz, g.op, -pfx, -pfy, dx4, dy4, G4, al, ok);
            uint64_t vm[kGroup];  // per entry: the lanes that blended it (uniform masks, SALU)
#pragma unroll
            for (int u = 0; u < kGroup; ++u) {
                const float w = blend_chain<BWD, AUX>(ok[u] ? al[u] : 0.0f, c.rgbd[u], c.pos[u], Ts, C01, C2D, L01,
                                                      L2, last, ((mb >> (8 * u)) & 1u) != 0u, &Cm);
                if (BWD) vm[u] = __builtin_amdgcn_fcmpf(w, 0.0f, kFcmpOGT);
            }
            if (BWD) {
                const uint32_t gm = (vm[0] ? 1u : 0u) | (vm[1] ? 2u : 0u) | (vm[2] ? 4u : 0u) | (vm[3] ? 8u : 0u);
                s_gused[j / kGroup] = __builtin_amdgcn_readfirstlane(gm);
            }
        };
        AlphaOps ga, gb;
        ColourOps cc;
        // lgkmcnt(0) only (vmcnt 63, expcnt 7: the next round's gathers stay in flight): at the loop
        // head nothing is outstanding in LDS, so the compiler's waits inside count the colour reads
        // exactly instead of draining the prefetch (its loop-carried state is conservative)
        constexpr unsigned kWaitLds = 0xC07F;
        // (scheduling barriers keep the compiler from merging or reordering the reads across them)
        const auto blend_range = [&](int j0, int j1) {
            load_alpha(j0, ga);
            __builtin_amdgcn_s_waitcnt(kWaitLds);
            for (int j = j0; j < j1; j += 2 * kGroup) {
                if (!__any(Ts > 0.0f)) break;
                load_colour(j, cc);
                __builtin_amdgcn_sched_barrier(0);
                load_alpha(j + kGroup, gb);
                __builtin_amdgcn_sched_barrier(0);
                blend_group(j, ga, cc);
                __builtin_amdgcn_sched_barrier(0);
                if (j + kGroup >= j1 || !__any(Ts > 0.0f)) break;
                load_colour(j + kGroup, cc);
                __builtin_amdgcn_sched_barrier(0);
                load_alpha(j + 2 * kGroup, ga);
                __builtin_amdgcn_sched_barrier(0);
                blend_group(j + kGroup, gb, cc);
                __builtin_amdgcn_sched_barrier(0);
                __builtin_amdgcn_s_waitcnt(kWaitLds);  // (the prefetch of ga: issued a whole group ago)
            }
        };
        // the round's first segment, its checkpoint, the second segment: two copies of the loop, so the
        // checkpoint costs nothing inside it (an early exit leaves the state at the first segment's end)
        blend_range(0, n_mid >= 0 ? n_mid : nk);
        if (n_mid >= 0) {
            take_mid();
            blend_range(n_mid_slot, nk);
        }
        if (a.diag) c_blend += __builtin_amdgcn_s_memtime() - c0;
        __syncthreads();
        if (BWD) {
            // the round's blended bits in list order, one ballot per word (words of rounds the wave
            // never reaches stay unwritten: past every pixel's last contributor, outside every replay)
    #pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int sl = kslot[i];
                const bool blended = sl >= 0 && ((s_gused[sl / kGroup] >> (sl % kGroup)) & 1u);
                const uint64_t wd = __ballot(blended);
                pend_word = lane == i ? wd : pend_word;
                if (blended) a.touched[s_id[sl]] = 1;  // (same-value byte stores: no atomics needed)
            }
        }
        pend_rel = (int)(b - range.x);
    }
    store_words();

    // the last blended segment's checkpoint (an empty tile's range is (0, 0): no slot, no replay)
    const float T = fabsf(Ts);
    if (seg_done >= 0) put_ckpt(seg_done);
    if (inside) {
        const size_t pix = (size_t)a.W * py + px;
        const size_t HW = (size_t)a.W * a.H;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last;
        // forward.cu:376 `C + T * bg`, contracted (as the oracle): fma(T, bg, C)
        // (the background read before the first store: loaded between the stores, each load waited, the
        // compiler unable to tell out_color from bg — three round trips at every wave's end)
        const float bg0 = a.bg[0], bg1 = a.bg[1], bg2 = a.bg[2];
        a.out_color[pix] = __builtin_fmaf(T, bg0, C01.x);
        a.out_color[HW + pix] = __builtin_fmaf(T, bg1, C01.y);
        a.out_color[2 * HW + pix] = __builtin_fmaf(T, bg2, C2D.x);
        a.out_depth[pix] = C2D.y;
        if constexpr (AUX) a.aux_out[pix] = make_float2(Cm, C2D.y);
    }
    const uint32_t m = wave_max_u32(inside ? last : 0u);
    // (item class from the entries the cull kept — the diagnostics' count, live anyway: a blended-entry
    // count here pushed the kernel into spilling)
    if (BWD && m) emit_items(a, tile, quad, x8, (m + kSegLen - 1) / kSegLen, diag_kept, lane);
    if (lane == 0) {
        a.quad_last[qidx] = m;
        if (m) atomicMax(&a.tile_last[tile], m);
        if (a.diag) {
            uint64_t* d = a.diag + kDiagWords * (size_t)qidx;
            d[0] = t_start;
            d[1] = __builtin_amdgcn_s_memrealtime();
            d[2] = diag_kept;
            d[3] = diag_rounds;
            d[4] = c_blend;
            d[5] = __builtin_amdgcn_s_memtime() - c_start;
            d[6] = c_cull;
            d[7] = wave_location();
        }
    }
}

void launch_render_forward(const RenderArgs& a, hipStream_t s) {
    const int tiles = a.gx * a.gy;
    if (tiles <= 0) return;
    if (!a.order_ready) hipLaunchKernelGGL(k_tile_order, dim3(1), dim3(1024), 0, s, a.ranges, tiles, a.tile_order);
    if (a.bwd && a.aux_out)
        hipLaunchKernelGGL((k_render_fwd<true, true>), dim3(div_up(tiles, 8) * 32), dim3(64), 0, s, a);
    else if (a.bwd)
        hipLaunchKernelGGL((k_render_fwd<true, false>), dim3(div_up(tiles, 8) * 32), dim3(64), 0, s, a);
    else
        hipLaunchKernelGGL((k_render_fwd<false, false>), dim3(div_up(tiles, 8) * 32), dim3(64), 0, s, a);
}

// Whether a recolor's colours are its source forward's aux grey: flag[0] |= 1 on any difference
// (bits compared: the blend of equal bits gives equal bits); flag zeroed by the caller
__global__ __launch_bounds__(256) void k_aux_match(int P, const float* __restrict__ colors,
                                                   const uint8_t* __restrict__ aux_mask, uint32_t* __restrict__ flag) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    bool diff = false;
    if (i < P) {
        const uint32_t m = aux_mask[i] ? __float_as_uint(1.0f) : 0u;
        diff = __float_as_uint(colors[3 * (size_t)i]) != m || __float_as_uint(colors[3 * (size_t)i + 1]) != m ||
               __float_as_uint(colors[3 * (size_t)i + 2]) != m;
    }
    if (__any(diff) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);  // (a vector atomic, rare: only on difference)
}

void launch_aux_match(int P, const float* colors, const uint8_t* aux_mask, uint32_t* flag, hipStream_t s) {
    if (P <= 0) return;
    hipLaunchKernelGGL(k_aux_match, dim3(div_up(P, 256)), dim3(256), 0, s, P, colors, aux_mask, flag);
}

// =====================================================================
// apply_weights: same traversal, per blended pair add image weights
// =====================================================================
__global__ __launch_bounds__(64) void k_render_apply_weights(ApplyWeightsArgs a) {
    const int quad = blockIdx.x & 3, tile = blockIdx.x >> 2;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int lane = threadIdx.x;
    const int bx0 = tx * kTile + (quad & 1) * kQuad, by0 = ty * kTile + (quad >> 1) * kQuad;
    const int px = bx0 + (lane & 7), py = by0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;

    __shared__ float2 s_xy[64];
    __shared__ float4 s_co[64];
    __shared__ uint32_t s_id[64];

    const size_t HW = (size_t)a.W * a.H;
    const size_t pix = inside ? (size_t)a.W * py + px : 0;
    float Cw[3] = {0.f, 0.f, 0.f};
    if (inside)
        for (int ch = 0; ch < a.C; ++ch) Cw[ch] = a.image_weights[ch * HW + pix];

    const uint2 range = a.ranges[tile];
    float T = 1.0f;
    bool done = !inside;
    for (uint32_t b = range.x; b < range.y; b += 64) {
        if (!__any(!done)) break;
        const uint32_t k = b + lane;
        bool keep = false;
        float2 xy = make_float2(0.f, 0.f);
        float4 co = make_float4(0.f, 0.f, 0.f, 0.f);
        uint32_t id = 0;
        if (k < range.y) {
            id = a.point_pairs[k].x;
            xy = a.splat[id].xy;
            co = a.splat[id].co;
            keep = cull_keep(xy, co, (float)bx0, (float)by0);
        }
        const uint64_t km = __ballot(keep);
        if (keep) {
            const int slot = __popcll(km & lanemask_lt());
            s_xy[slot] = xy;
            s_co[slot] = co;
            s_id[slot] = id;
        }
        __syncthreads();
        const int nk = __popcll(km);
        for (int j = 0; j < nk; ++j) {
            if (!__any(!done)) break;
            bool blend = false;
            float dx, dy, G, alpha;
            if (!done && pixel_alpha(s_xy[j], s_co[j], pfx, pfy, dx, dy, G, alpha)) {
                const float test_T = T * (1 - alpha);
                if (test_T < 0.0001f) {
                    done = true;
                } else {
                    T = test_T;
                    blend = true;
                }
            }
            const uint64_t bm = __ballot(blend);
            if (bm) {
                // apply_weights.cu:331-335: weights += C[ch]; cnt += 1 once per channel
                const uint32_t gid = s_id[j];
                for (int ch = 0; ch < a.C; ++ch) {
                    const float v = wave_sum_to_lane63(blend ? Cw[ch] : 0.f);
                    if (lane == 63) atomicAdd(&a.weights[(size_t)gid * a.C + ch], v);
                }
                if (lane == 63) atomicAdd(&a.cnt[gid], (int)__popcll(bm) * a.C);
            }
        }
        __syncthreads();
    }
}

void launch_blend_exp(long long n, const float* x, float* y, hipStream_t s) {
    const long long quads = (n + 3) / 4;
    hipLaunchKernelGGL(k_blend_exp, dim3((unsigned)((quads + 255) / 256)), dim3(256), 0, s, n, x, y);
}

void launch_render_apply_weights(const ApplyWeightsArgs& a, hipStream_t s) {
    const int tiles = a.gx * a.gy;
    if (tiles <= 0) return;
    hipLaunchKernelGGL(k_render_apply_weights, dim3(tiles * 4), dim3(64), 0, s, a);
}

// =====================================================================
// backward: 4 quadrant waves per tile, records per instance
// =====================================================================
// One entry of the back-to-front replay for one pixel, branch-free
// (backward.cu:448-545).  State: T (transmittance in front of the entry) and
// D, the colour composited behind the current position.  The reference's
// accum_rec / last_alpha / last_color recurrence
//     accum = last_alpha*last_color + (1-last_alpha)*accum;  last_* = (alpha, c)
// hands every hit the value D had before it, with D <- alpha*c + (1-alpha)*D
// after it; written as D += ae*(c - D) with ae = 0 for a skipped pixel, the
// update is an exact no-op there and needs no select.  T is recovered with
// v_rcp_f32 (<= 1 ulp per hit instead of the IEEE quotient's 0.5).
// Instead of the reference's nine per-pixel gradient terms it emits the nine
// per-pixel sums they factor into, with u = G * dL/dalpha:
//   g = (u dx, u dy, u dx^2, u dx dy, u dy^2, u, aT dp0, aT dp1, aT dp2)
// — the entry's conic, opacity and the ndc scale are constant over pixels
// and are applied once per entry after the reduction (finish_record).
//
// Four consecutive entries of the replay: the alpha tests packed (pixel_alpha4),
// the back-to-front chain (T, D) entry by entry (bwd_chain), the per-pixel
// products of the nine sums packed again.
__device__ __forceinline__ float bwd_chain(bool hit, float alpha, float G, float4 c, float dp0, float dp1, float dp2,
                                           float nbg, float& T, float& D0, float& D1, float& D2, float& wc) {
    const float ae = hit ? alpha : 0.f;
    const float d = 1.f - ae;
    const float r = __builtin_amdgcn_rcpf(d);
    // T / d: the reciprocal's product plus one Newton step on the quotient (q + (T - q d) r), within about half
    // an ulp like the reference's IEEE division (backward.cu:503) — T * rcp alone carries v_rcp_f32's ulp into
    // every step of the back-to-front chain, and those errors add up in sums that cancel (round 6, the fp64-truth
    // bar: the dL/dcolor sums of a few Gaussians 14x further from the truth than the reference's own arithmetic)
    const float q = T * r;
    T = hit ? __builtin_fmaf(__builtin_fmaf(-q, d, T), r, q) : T;
    const float t0 = c.x - D0, t1 = c.y - D1, t2 = c.z - D2;
    float dL_dalpha = t0 * dp0;
    dL_dalpha += t1 * dp1;
    dL_dalpha += t2 * dp2;
    dL_dalpha = dL_dalpha * T + nbg * r;
    wc = ae * T;
    D0 += ae * t0;
    D1 += ae * t1;
    D2 += ae * t2;
    return hit ? G * dL_dalpha : 0.f;
}

__device__ __forceinline__ void bwd_quad(f4v x, f4v y, f4v cx, f4v ncy, f4v cz, f4v op, const float4 (&c)[4],
                                         const bool (&in)[4], float pfx, float pfy, float dp0, float dp1, float dp2,
                                         float nbg, float& T, float& D0, float& D1, float& D2, float (&g)[4][9]) {
    f4v dx, dy, G, alpha;
    bool ok[4];
    pixel_alpha4(x, y, cx, ncy, cz, op, -pfx, -pfy, dx, dy, G, alpha, ok);
    f4v u, wc;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        float w;
        u[e] = bwd_chain(ok[e] && in[e], alpha[e], G[e], c[e], dp0, dp1, dp2, nbg, T, D0, D1, D2, w);
        wc[e] = w;
    }
    const f4v udx = u * dx, udy = u * dy;
    const f4v gxx = udx * dx, gxy = udx * dy, gyy = udy * dy;
    const f4v w0 = wc * dp0, w1 = wc * dp1, w2 = wc * dp2;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
        g[e][0] = udx[e];
        g[e][1] = udy[e];
        g[e][2] = gxx[e];
        g[e][3] = gxy[e];
        g[e][4] = gyy[e];
        g[e][5] = u[e];
        g[e][6] = w0[e];
        g[e][7] = w1[e];
        g[e][8] = w2[e];
    }
}

// The entry's record from the quadrant sums S: the reference's per-pixel
// terms (backward.cu:524-545) with the per-entry constants factored out:
//   dL/dmean2D = -(ddelx_dx, ddely_dy) * o * (a Sx + b Sy, c Sy + b Sx),
//   dL/dconic  = -o/2 (Sxx, Sxy, Syy), dL/dopacity = Su, dL/dcolor = Sc.
__device__ __forceinline__ void finish_record(float4 co, const float (&S)[9], float ddelx_dx, float ddely_dy,
                                              float4* rec) {
    const float h = -0.5f * co.w;
    rec[0] = make_float4(-(co.x * S[0] + co.y * S[1]) * co.w * ddelx_dx,
                         -(co.z * S[1] + co.y * S[0]) * co.w * ddely_dy, h * S[2], h * S[3]);
    rec[1] = make_float4(h * S[4], S[5], S[6], S[7]);
    rec[2] = make_float4(S[8], 0.f, 0.f, 0.f);
}

constexpr int kBwdGroup = 4;            // entries replayed between two reduce-scatters
constexpr int kBwdHalf = 128;           // list positions per LDS staging unit
constexpr int kBwdNI = kSegLen / 64;    // list positions per lane
static_assert(kSegLen % kBwdHalf == 0, "whole staging units per segment");

// 5 waves per SIMD: the 128-position items need <= 96 VGPRs (no spill)
#ifndef GS_BWD_WAVES
#define GS_BWD_WAVES 5
#endif
// One wave per work item = (8x8 quadrant, segment of its window), independent
// 64-thread workgroups.  A segment is at most kSegLen = 128 list positions: the
// wave loads their (Gaussian, slot) pairs and the forward's blended bits (2 per
// lane), gathers the Splats of the blended ones, and replays the segment back
// to front in units of 128 positions staged through LDS (6.9 KB: with
// <= 128 VGPRs, 4 waves per SIMD), each in groups of four entries whose nine
// sums are reduce-scattered across the wave (quad_reduce).  Each kept entry gets
// one record at 4*slot + quadrant (slot: the binning slot, so k_gauss_bwd reads
// a Gaussian's records contiguously) and a flag.
// qi: the block's place in this view's grid of `grid` blocks (k_render_bwd: blockIdx.x, gridDim.x)
__device__ __forceinline__ void render_bwd_block(const RenderBwdArgs& a, const uint32_t qi, const uint32_t grid) {
    // kept entries of a half-segment, compacted back to front, + a group of padding
    // (one array per field: four consecutive entries' field is one 16-B read, see bwd_quad)
    __shared__ __attribute__((aligned(16))) float s_x[kBwdHalf + kBwdGroup], s_y[kBwdHalf + kBwdGroup];
    __shared__ __attribute__((aligned(16))) float s_cx[kBwdHalf + kBwdGroup], s_cy[kBwdHalf + kBwdGroup],
        s_cz[kBwdHalf + kBwdGroup],
        s_op[kBwdHalf + kBwdGroup];
    __shared__ float4 s_rgb[kBwdHalf + kBwdGroup];
    __shared__ uint32_t s_pos[kBwdHalf + kBwdGroup];
    __shared__ uint2 s_pair[kBwdHalf + kBwdGroup];  // (Gaussian, slot) of the kept entries: the record writes
    const int lane = threadIdx.x;
    // block -> work item (quadrant, segment) of the forward's lists, heaviest class first.  Class c's
    // region is 8 x (its longest XCD list) blocks; block b of it (b & 7 = its XCD under the round-robin
    // dealing) takes item b >> 3 of list (c, b & 7), so a tile's quadrants replay on one XCD and share
    // its L2.  Should the regions outgrow the grid (lists far out of balance; the grid bounds only their
    // total), the blocks take the lists one after another instead.  Blocks past the end exit (they
    // dispatch after every real item; see launch_render_backward for the grid).  (A persistent-wave
    // work queue measured slower than the hardware dispatcher here.)
    uint32_t region[kItemClasses], need = 0;
#pragma unroll
    for (int c = 0; c < kItemClasses; ++c) {
        region[c] = kItemXcds * a.bwd_count[item_max_at(c)];
        need += region[c];
    }
    int list;
    uint32_t idx;
    if (need <= grid) {
        if (qi >= need) return;
        uint32_t o = qi;
        int c = 0;
#pragma unroll
        for (int k = 0; k < kItemClasses - 1; ++k)
            if (c == k && o >= region[k]) {
                o -= region[k];
                c = k + 1;
            }
        const int x = (int)(o % kItemXcds);
        idx = o / kItemXcds;
        if (idx >= a.bwd_count[item_count_at(c, x)]) return;
        list = c * kItemXcds + x;
    } else {
        // (lane c * 8 + x loads count (c, x); readlane(nl, l) is list l's count: a block-uniform lane
        // select, no indexed array)
        const uint32_t nl =
            lane < kItemClasses * kItemXcds ? a.bwd_count[item_count_at(lane / kItemXcds, lane % kItemXcds)] : 0u;
        uint32_t o = qi;
        list = -1;
        idx = 0;
#pragma unroll
        for (int l = 0; l < kItemClasses * kItemXcds; ++l) {
            const uint32_t v = (uint32_t)__builtin_amdgcn_readlane((int)nl, l);
            if (list < 0 && o < v) {
                list = l;
                idx = o;
            }
            if (list < 0) o -= v;
        }
        if (list < 0) return;
    }
    const uint2 item = a.bwd_items[(size_t)list * a.item_cap + idx];
    const int tile = (int)item.x, quad = (int)(item.y & 3u), seg = (int)(item.y >> 2);
    const int qidx = 4 * tile + quad;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int bx0 = tx * kTile + (quad & 1) * kQuad, by0 = ty * kTile + (quad >> 1) * kQuad;
    const int px = bx0 + (lane & 7), py = by0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;

    const uint2 range = a.ranges[tile];
    const int window = (int)a.quad_last[qidx];  // the quadrant's last contributor (1-based)
    const int nseg_q = (window + kSegLen - 1) / kSegLen;
    // this wave's segment [lo, limit) of the window; the last segment ends at the window
    const int lo = seg * kSegLen;
    const int limit = seg == nseg_q - 1 ? window : lo + kSegLen;
    const int n = limit - lo;

    // (Gaussian, slot) and the forward's blended bit of the segment's entries (entry lo + 64 i + lane).
    // An entry no pixel of the quadrant blended has an all-zero gradient: the bit is the exact cull
    // (the forward's `use` is the replay's `hit && pos < n_contrib`).
    const uint32_t* used32 = reinterpret_cast<const uint32_t*>(a.used + (size_t)used_base(range.x, tile) * 4 + quad);
    uint2 pairs[kBwdNI];
    uint32_t kb = 0u;
#pragma unroll
    for (int i = 0; i < kBwdNI; ++i) {
        const int j = 64 * i + lane, k = lo + j;
        const bool in = j < n;
        pairs[i] = in ? a.point_pairs[range.x + k] : make_uint2(0u, 0u);
        const uint32_t ub = in ? used32[(size_t)(k >> 6) * 8 + ((k >> 5) & 1)] : 0u;
        kb |= ((ub >> (k & 31)) & 1u) << i;
    }
    Entry cur[kBwdNI];
#pragma unroll
    for (int i = 0; i < kBwdNI; ++i)  // (dropped entries gather Gaussian 0: one shared line)
        cur[i] = gather_entry(a.splat, (kb >> i) & 1u ? pairs[i].x : 0u);

    const size_t HW = (size_t)a.W * a.H;
    const size_t pix = inside ? (size_t)a.W * py + px : 0;
    const float T_final = inside ? a.final_T[pix] : 0.f;
    const uint32_t last_contributor = inside ? a.n_contrib[pix] : 0u;
    float dp0 = 0.f, dp1 = 0.f, dp2 = 0.f;
    if (inside) {
        dp0 = a.dL_dpix[pix];
        dp1 = a.dL_dpix[HW + pix];
        dp2 = a.dL_dpix[2 * HW + pix];
    }
    const float nbg = -T_final * (a.bg[0] * dp0 + a.bg[1] * dp1 + a.bg[2] * dp2);
    float T = T_final, D0 = 0.f, D1 = 0.f, D2 = 0.f;
    if (limit < window) {
        // start inside the window: T after this segment (its checkpoint) and the colour composited
        // behind position `limit`, D = (S_{seg+1} + ... + S_last) / T from the later segments' own
        // colour sums (summed back to front: the rounding stays relative to D itself; round 3 measured a
        // prefix difference (C_last - C_seg) in its place for the early segments: +17 MB of checkpoint
        // writes in the forward, no faster replay — these reads are a small part of its traffic)
        const float4* ck = a.ckpt + ((size_t)ckpt_base(range.x, tile) * 4 + quad) * 64 + lane;
        T = ck[(size_t)seg * 256].x;
        float B0 = 0.f, B1 = 0.f, B2 = 0.f;
        for (int k = nseg_q - 1; k > seg; --k) {
            const float4 c = ck[(size_t)k * 256];
            B0 += c.y;
            B1 += c.z;
            B2 += c.w;
        }
        const float inv = 1.0f / T;
        D0 = B0 * inv;
        D1 = B1 * inv;
        D2 = B2 * inv;
    }
    const float ddelx_dx = (float)(0.5 * a.W), ddely_dy = (float)(0.5 * a.H);
    const uint64_t t_start = a.diag ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint64_t c_start = a.diag ? __builtin_amdgcn_s_memtime() : 0;
    uint64_t c_replay = 0;
    uint32_t diag_kept = 0;

    // the lane-row -> entry map of quad_reduce's result (row r holds entry e0 + r)
    const int row = lane >> 4;
    const int row_entry = row;
    const bool row_writer = (lane & 15) == 0;

#pragma unroll
    for (int h = kSegLen / kBwdHalf - 1; h >= 0; --h) {  // back unit first
        // compact the forward's blended entries of this half back to front
        int nk = 0;
#pragma unroll
        for (int i = 2 * h + 1; i >= 2 * h; --i) {
            const int j = 64 * i + lane;
            const bool keep = j < n && ((kb >> i) & 1u);
            const uint64_t km = __ballot(keep);
            if (keep) {
                const int slot = nk + __popcll(km & ~lanemask_lt() & ~(1ull << lane));
                s_x[slot] = cur[i].xy.x;
                s_y[slot] = cur[i].xy.y;
                s_cx[slot] = -cur[i].co.x;  // (negated: pixel_alpha4)
                s_cy[slot] = -cur[i].co.y;  // (finish_record negates the three back)
                s_cz[slot] = -cur[i].co.z;
                s_op[slot] = cur[i].co.w;
                s_rgb[slot] = cur[i].f;
                s_pos[slot] = (uint32_t)(lo + j);
                s_pair[slot] = pairs[i];
            }
            nk += __popcll(km);
        }
        if (lane < kBwdGroup) {  // padding: alpha = 0 everywhere, never in a pixel's list
            s_x[nk + lane] = 0.f;
            s_y[nk + lane] = 0.f;
            s_cx[nk + lane] = 0.f;
            s_cy[nk + lane] = 0.f;
            s_cz[nk + lane] = 0.f;
            s_op[nk + lane] = 0.f;
            s_rgb[nk + lane] = make_float4(0.f, 0.f, 0.f, 0.f);
            s_pos[nk + lane] = 0xFFFFFFFFu;
        }
        diag_kept += nk;
        __syncthreads();

        const uint64_t c0 = a.diag ? __builtin_amdgcn_s_memtime() : 0;
        for (int k = 0; k < nk; k += kBwdGroup) {
            float g[kBwdGroup][9];
            {
                const auto ld4 = [&](const float* f) { return *reinterpret_cast<const f4v*>(f + k); };
                const float4 c4[4] = {s_rgb[k], s_rgb[k + 1], s_rgb[k + 2], s_rgb[k + 3]};
                const bool in4[4] = {s_pos[k] < last_contributor, s_pos[k + 1] < last_contributor,
                                     s_pos[k + 2] < last_contributor, s_pos[k + 3] < last_contributor};
                bwd_quad(ld4(s_x), ld4(s_y), ld4(s_cx), ld4(s_cy), ld4(s_cz), ld4(s_op), c4, in4, pfx, pfy, dp0, dp1,
                         dp2, nbg, T, D0, D1, D2, g);
            }
            __builtin_amdgcn_sched_barrier(0);  // (every product first: the lane swaps clobber their operands)
            float S[9];
#pragma unroll
            // (entries 0 and 2, 1 and 3 swapped together: the operands of each lane swap then sit in
            // different register pairs of the packed products — no copy before the swap — and row r
            // holds entry r; the per-entry sums are the same adds in the same order)
            for (int f = 0; f < 9; ++f) S[f] = quad_reduce_rows(g[0][f], g[2][f], g[1][f], g[3][f]);
            row_sum16_x9(S);
            __builtin_amdgcn_sched_barrier(0);
            const int kw = k + row_entry;
            if (row_writer && kw < nk) {
                const uint2 pr = s_pair[kw];
                const size_t rec = 4 * (size_t)pr.y + quad;
                finish_record(make_float4(-s_cx[kw], -s_cy[kw], -s_cz[kw], s_op[kw]), S, ddelx_dx, ddely_dy,
                              a.records + 3 * rec);
                a.rec_flags[rec] = 1;
            }
        }
        if (a.diag) c_replay += __builtin_amdgcn_s_memtime() - c0;
        __syncthreads();
    }
    if (a.diag && lane == 0) {
        uint64_t* d = a.diag + kDiagWords * (size_t)qi;
        d[0] = t_start;
        d[1] = __builtin_amdgcn_s_memrealtime();
        d[2] = diag_kept;
        d[3] = 1;
        d[4] = c_replay;
        d[5] = __builtin_amdgcn_s_memtime() - c_start;
        d[6] = (uint64_t)seg << 32 | (uint32_t)qidx;
        d[7] = wave_location();
    }
}

__global__ __launch_bounds__(64, GS_BWD_WAVES) void k_render_bwd(RenderBwdArgs a) {
    render_bwd_block(a, blockIdx.x, gridDim.x);
}

// Several views' replays in one launch (one stream: no fork to the views' streams and no join back
// before the per-Gaussian pass — each such cross-stream hop cost ~10 us of queue time on the box,
// tools/probes/queue_gap.hip).  The views' grids are interleaved in runs of 8 blocks: block b is block
// 8 i + (b & 7) of view (b >> 3) % n, i = (b >> 3) / n — so b & 7, the XCD under the round-robin dealing
// that each view's item lists are grouped by, is the block's XCD in its own view's grid too, and every
// view's heaviest items dispatch first.  A view's grid is m.grid[v] blocks (a multiple of 8), not its
// item bound: the bound (~7x the real items at c2) dealt from ONE queue made the surplus workgroups'
// dispatch outlast the replay (3 x 147k blocks: the step +43 us against three launches on three
// queues); a block takes items qi, qi + grid, ... below the lists' need (once at c2), so any count is
// replayed.
__global__ __launch_bounds__(64, 4) void k_render_bwd_views(RenderBwdViews m) {  // (4: the item loop spilled at 96 VGPRs)
    const uint32_t u = blockIdx.x >> 3, v = u % (uint32_t)m.n;
    const RenderBwdArgs& a = m.v[v];
    const uint32_t grid = m.grid[v];
    const uint32_t q0 = (u / (uint32_t)m.n) * 8 + (blockIdx.x & 7u);
    if (q0 >= grid) return;
    uint32_t need = 0;
#pragma unroll
    for (int c = 0; c < kItemClasses; ++c) need += kItemXcds * a.bwd_count[item_max_at(c)];
    const uint32_t lim = need < a.item_cap ? need : a.item_cap;  // (past it every block exits at once)
    for (uint32_t qi = q0; qi < lim; qi += grid) render_bwd_block(a, qi, a.item_cap);
}

// One workgroup per possible item (the bound, 4 x checkpoint slots, is ~7x the c2 count): the surplus
// workgroups exit at once and cost nothing measurable (render_bwd 104 us either way).
void launch_render_backward(const RenderBwdArgs& a, hipStream_t s) {
    const int tiles = a.gx * a.gy;
    if (tiles <= 0 || a.item_cap == 0) return;
    hipLaunchKernelGGL(k_render_bwd, dim3(a.item_cap), dim3(64), 0, s, a);
}

void launch_render_backward_views(const RenderBwdArgs* a, int n, uint32_t grid_div, hipStream_t s) {
    if (grid_div < 1) grid_div = 1;
    for (int v0 = 0; v0 < n; v0 += kMaxReplayViews) {
        RenderBwdViews m;
        m.n = std::min(kMaxReplayViews, n - v0);
        uint32_t runs = 0;  // the longest view grid, in runs of 8 blocks
        for (int v = 0; v < m.n; ++v) {
            m.v[v] = a[v0 + v];
            const uint32_t cap = a[v0 + v].item_cap;
            m.grid[v] = 8 * ((cap / grid_div + 7) / 8);
            if (m.grid[v] == 0 && cap > 0) m.grid[v] = 8;
            runs = std::max(runs, m.grid[v] / 8);
        }
        if (runs == 0) continue;
        hipLaunchKernelGGL(k_render_bwd_views, dim3(8 * m.n * runs), dim3(64), 0, s, m);
    }
}

}  // namespace gs
