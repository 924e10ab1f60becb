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
//  * the backward keeps the 4 quadrant waves of a tile in one workgroup,
//    starts at the tile's largest n_contrib instead of the list end, reduces
//    each entry's 9 gradient terms across the wave with DPP, combines the 4
//    waves in LDS and writes ONE 48-byte record per (Gaussian, tile) instance
//    with plain stores.  No float atomics: the per-Gaussian sum happens in
//    gs_backward.hip in a fixed order, so the backward is bitwise
//    reproducible.
#include "gs_common.h"
#include "gs_internal.h"

namespace gs {

// Conservative test: can Gaussian (xy, conic, opacity) reach alpha >= 1/255
// at any pixel of the box [bx0,bx0+7] x [by0,by0+7]?  alpha = min(.99, o*G),
// G = exp(-q/2), q = a dx^2 + 2 b dx dy + c dy^2, d = xy - pixel.
__device__ __forceinline__ bool cull_keep(float2 xy, float4 co, float bx0, float by0) {
    const float o = co.w;
    if (o < 1.0f / 255.0f) return false;  // alpha <= o*G <= o   (NaN falls through: keep)
    const float a = co.x, b = co.y, c = co.z;
    if (!(a > 0.f && c > 0.f && a * c - b * b > 0.f)) return true;  // not positive definite: no bound
    const float thr = 2.0f * __logf(255.0f * o);  // the slack below absorbs __logf's error
    const float X0 = xy.x - (bx0 + 7.0f), X1 = xy.x - bx0;
    const float Y0 = xy.y - (by0 + 7.0f), Y1 = xy.y - by0;
    if (X0 <= 0.f && X1 >= 0.f && Y0 <= 0.f && Y1 >= 0.f) return true;
    const float slack = 2e-3f * (1.0f + fabsf(thr));
    bool keep = false;
    // edges dx = X: minimise over dy
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const float X = e ? X1 : X0;
        const float dy = fminf(Y1, fmaxf(Y0, __fdividef(-b * X, c)));
        const float t1 = a * X * X, t2 = 2.f * b * X * dy, t3 = c * dy * dy;
        keep |= (t1 + t2 + t3) - 1e-5f * (t1 + fabsf(t2) + t3) <= thr + slack;
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const float Y = e ? Y1 : Y0;
        const float dx = fminf(X1, fmaxf(X0, __fdividef(-b * Y, a)));
        const float t1 = a * dx * dx, t2 = 2.f * b * dx * Y, t3 = c * Y * Y;
        keep |= (t1 + t2 + t3) - 1e-5f * (t1 + fabsf(t2) + t3) <= thr + slack;
    }
    return keep;
}

// =====================================================================
// forward: one wave per 8x8 quadrant
// =====================================================================
// exp used by the blend loops: v_exp_f32 on the pre-scaled argument
// (|rel. err| ~1e-7 over the live range power in [-5.6, 0], same order as
// the CUDA expf the reference compiles to; see DESIGN.md §5 for the parity bar)
__device__ __forceinline__ float blend_exp(float x) { return __expf(x); }

// The per-(pixel, Gaussian) test shared by the forward, the backward replay
// and apply_weights: identical code, hence identical skip decisions
// (forward.cu:336-348, backward.cu:491-501).  Returns false when skipped.
__device__ __forceinline__ bool pixel_alpha(float2 xy, float4 co, float pfx, float pfy, float& dx, float& dy,
                                            float& G, float& alpha) {
    dx = xy.x - pfx;
    dy = xy.y - pfy;
    const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
    if (power > 0.0f) return false;
    G = blend_exp(power);
    alpha = fminf(0.99f, co.w * G);
    return alpha >= 1.0f / 255.0f;
}

constexpr int kRound = 256;  // list entries per round: 4 per lane, all loads in flight together

__global__ __launch_bounds__(64) void k_render_fwd(RenderArgs a) {
    const int quad = blockIdx.x & 3, tile = blockIdx.x >> 2;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int lane = threadIdx.x;
    const int bx0 = tx * kTile + (quad & 1) * kQuad, by0 = ty * kTile + (quad >> 1) * kQuad;
    const int px = bx0 + (lane & 7), py = by0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;

    __shared__ float2 s_xy[kRound];
    __shared__ float4 s_co[kRound];
    __shared__ float4 s_rgbd[kRound];
    __shared__ uint32_t s_pos[kRound];

    const uint2 range = a.ranges[tile];
    float T = 1.0f, C0 = 0.f, C1 = 0.f, C2 = 0.f, D = 0.f;
    uint32_t last = 0;
    bool done = !inside;
    const uint64_t t_start = a.diag ? __builtin_amdgcn_s_memrealtime() : 0;
    uint32_t diag_kept = 0, diag_rounds = 0;

    // prefetch the first round's ids
    uint32_t ids[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t k = range.x + 64 * i + lane;
        ids[i] = k < range.y ? a.point_list[k] : 0u;
    }
    for (uint32_t b = range.x; b < range.y; b += kRound) {
        if (!__any(!done)) break;
        float2 xy[4];
        float4 co[4], f[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t k = b + 64 * i + lane;
            if (k < range.y) {
                xy[i] = a.means2D[ids[i]];
                co[i] = a.conic_opacity[ids[i]];
                f[i] = a.rgbd[ids[i]];
            }
        }
        // next round's ids, in flight during this round's blend
        uint32_t nids[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t k = b + kRound + 64 * i + lane;
            nids[i] = k < range.y ? a.point_list[k] : 0u;
        }
        // cull against the quadrant, compact survivors in list order (i-major, lane-minor)
        int nk = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t k = b + 64 * i + lane;
            const bool keep = k < range.y && cull_keep(xy[i], co[i], (float)bx0, (float)by0);
            const uint64_t km = __ballot(keep);
            if (keep) {
                const int slot = nk + __popcll(km & lanemask_lt());
                s_xy[slot] = xy[i];
                s_co[slot] = co[i];
                s_rgbd[slot] = f[i];
                s_pos[slot] = k - range.x + 1;  // 1-based contributor index (forward.cu:331)
            }
            nk += __popcll(km);
        }
        diag_kept += nk;
        diag_rounds += 1;
        __syncthreads();
        for (int j = 0; j < nk; ++j) {
            if (!__any(!done)) break;
            float dx, dy, G, alpha;
            if (!done && pixel_alpha(s_xy[j], s_co[j], pfx, pfy, dx, dy, G, alpha)) {
                const float test_T = T * (1 - alpha);
                if (test_T < 0.0001f) {
                    done = true;
                } else {
                    const float4 fe = s_rgbd[j];
                    const float w = alpha * T;
                    C0 += fe.x * w;
                    C1 += fe.y * w;
                    C2 += fe.z * w;
                    D += fe.w * w;
                    T = test_T;
                    last = s_pos[j];
                }
            }
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 4; ++i) ids[i] = nids[i];
    }

    if (inside) {
        const size_t pix = (size_t)a.W * py + px;
        const size_t HW = (size_t)a.W * a.H;
        a.final_T[pix] = T;
        a.n_contrib[pix] = last;
        a.out_color[pix] = C0 + T * a.bg[0];
        a.out_color[HW + pix] = C1 + T * a.bg[1];
        a.out_color[2 * HW + pix] = C2 + T * a.bg[2];
        a.out_depth[pix] = D;
    }
    const uint32_t m = wave_max_u32(inside ? last : 0u);
    if (lane == 0) {
        a.quad_last[blockIdx.x] = m;
        if (m) atomicMax(&a.tile_last[tile], m);
        if (a.diag) {
            uint64_t* d = a.diag + 4 * (size_t)blockIdx.x;
            d[0] = t_start;
            d[1] = __builtin_amdgcn_s_memrealtime();
            d[2] = diag_kept;
            d[3] = diag_rounds;
        }
    }
}

void launch_render_forward(const RenderArgs& a, hipStream_t s) {
    const int tiles = a.gx * a.gy;
    if (tiles <= 0) return;
    hipLaunchKernelGGL(k_render_fwd, dim3(tiles * 4), dim3(64), 0, s, a);
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
            id = a.point_list[k];
            xy = a.means2D[id];
            co = a.conic_opacity[id];
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

void launch_render_apply_weights(const ApplyWeightsArgs& a, hipStream_t s) {
    const int tiles = a.gx * a.gy;
    if (tiles <= 0) return;
    hipLaunchKernelGGL(k_render_apply_weights, dim3(tiles * 4), dim3(64), 0, s, a);
}

// =====================================================================
// backward: 4 quadrant waves per tile, records per instance
// =====================================================================
__global__ __launch_bounds__(256) void k_render_bwd(RenderBwdArgs a) {
    const int tile = blockIdx.x;
    const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
    const int tx = tile % a.gx, ty = tile / a.gx;
    const int bx0 = tx * kTile + (w & 1) * kQuad, by0 = ty * kTile + (w >> 1) * kQuad;
    const int px = bx0 + (lane & 7), py = by0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pfx = (float)px, pfy = (float)py;

    __shared__ float2 s_xy[64];
    __shared__ float4 s_co[64];
    __shared__ float4 s_rgb[64];
    __shared__ float s_part[4][9][64];

    const uint2 range = a.ranges[tile];
    const uint32_t limit = a.tile_last[tile];
    const size_t HW = (size_t)a.W * a.H;
    const size_t pix = inside ? (size_t)a.W * py + px : 0;

    const float T_final = inside ? a.final_T[pix] : 0.f;
    float T = T_final;
    const uint32_t last_contributor = inside ? a.n_contrib[pix] : 0u;
    float dp0 = 0.f, dp1 = 0.f, dp2 = 0.f;
    if (inside) {
        dp0 = a.dL_dpix[pix];
        dp1 = a.dL_dpix[HW + pix];
        dp2 = a.dL_dpix[2 * HW + pix];
    }
    const float bg_dot = a.bg[0] * dp0 + a.bg[1] * dp1 + a.bg[2] * dp2;
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f;     // accum_rec
    float lc0 = 0.f, lc1 = 0.f, lc2 = 0.f;        // last_color
    float last_alpha = 0.f;
    const float ddelx_dx = (float)(0.5 * a.W), ddely_dy = (float)(0.5 * a.H);
    const uint32_t wave_last = wave_max_u32(last_contributor);
    const uint64_t t_start = a.diag ? __builtin_amdgcn_s_memrealtime() : 0;
    uint32_t diag_kept = 0, diag_rounds = 0;

    for (int hi = (int)limit; hi > 0; hi -= 64) {
        const int lo = hi > 64 ? hi - 64 : 0;
        const int n = hi - lo;
        if (tid < n) {
            const uint32_t id = a.point_list[range.x + lo + tid];
            s_xy[tid] = a.means2D[id];
            s_co[tid] = a.conic_opacity[id];
            s_rgb[tid] = a.rgbd[id];
        }
#pragma unroll
        for (int f = 0; f < 9; ++f) s_part[w][f][lane] = 0.f;
        __syncthreads();

        bool keep = false;
        if (lane < n && (uint32_t)(lo + lane) < wave_last) keep = cull_keep(s_xy[lane], s_co[lane], (float)bx0, (float)by0);
        uint64_t km = __ballot(keep);
        diag_kept += __popcll(km);
        diag_rounds += 1;
        while (km) {
            const int j = 63 - __clzll(km);
            km &= ~(1ull << j);
            const uint32_t contributor = (uint32_t)(lo + j);  // 0-based position in the tile list
            float g0 = 0.f, g1 = 0.f, g2 = 0.f, g3 = 0.f, g4 = 0.f, g5 = 0.f, g6 = 0.f, g7 = 0.f, g8 = 0.f;
            bool hit = false;
            float dx, dy, G, alpha;
            const float4 co = s_co[j];
            if (contributor < last_contributor && pixel_alpha(s_xy[j], co, pfx, pfy, dx, dy, G, alpha)) {
                {
                    {
                        hit = true;
                        T = T / (1.f - alpha);
                        const float dchannel_dcolor = alpha * T;
                        const float4 c = s_rgb[j];
                        float dL_dalpha = 0.0f;
                        acc0 = last_alpha * lc0 + (1.f - last_alpha) * acc0;
                        lc0 = c.x;
                        dL_dalpha += (c.x - acc0) * dp0;
                        g6 = dchannel_dcolor * dp0;
                        acc1 = last_alpha * lc1 + (1.f - last_alpha) * acc1;
                        lc1 = c.y;
                        dL_dalpha += (c.y - acc1) * dp1;
                        g7 = dchannel_dcolor * dp1;
                        acc2 = last_alpha * lc2 + (1.f - last_alpha) * acc2;
                        lc2 = c.z;
                        dL_dalpha += (c.z - acc2) * dp2;
                        g8 = dchannel_dcolor * dp2;
                        dL_dalpha *= T;
                        last_alpha = alpha;
                        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
                        const float dL_dG = co.w * dL_dalpha;
                        const float gdx = G * dx, gdy = G * dy;
                        const float dG_ddelx = -gdx * co.x - gdy * co.y;
                        const float dG_ddely = -gdy * co.z - gdx * co.y;
                        g0 = dL_dG * dG_ddelx * ddelx_dx;
                        g1 = dL_dG * dG_ddely * ddely_dy;
                        g2 = -0.5f * gdx * dx * dL_dG;
                        g3 = -0.5f * gdx * dy * dL_dG;
                        g4 = -0.5f * gdy * dy * dL_dG;
                        g5 = G * dL_dalpha;
                    }
                }
            }
            if (__any(hit)) {
                g0 = wave_sum_to_lane63(g0);
                g1 = wave_sum_to_lane63(g1);
                g2 = wave_sum_to_lane63(g2);
                g3 = wave_sum_to_lane63(g3);
                g4 = wave_sum_to_lane63(g4);
                g5 = wave_sum_to_lane63(g5);
                g6 = wave_sum_to_lane63(g6);
                g7 = wave_sum_to_lane63(g7);
                g8 = wave_sum_to_lane63(g8);
                if (lane == 63) {
                    s_part[w][0][j] = g0; s_part[w][1][j] = g1; s_part[w][2][j] = g2;
                    s_part[w][3][j] = g3; s_part[w][4][j] = g4; s_part[w][5][j] = g5;
                    s_part[w][6][j] = g6; s_part[w][7][j] = g7; s_part[w][8][j] = g8;
                }
            }
        }
        __syncthreads();
        if (tid < 3 * 64) {
            const int q = tid >> 6, j = tid & 63;
            if (j < n) {
                float4 r;
                const int f0 = 4 * q;
                r.x = (s_part[0][f0][j] + s_part[1][f0][j]) + (s_part[2][f0][j] + s_part[3][f0][j]);
                if (q < 2) {
                    r.y = (s_part[0][f0 + 1][j] + s_part[1][f0 + 1][j]) + (s_part[2][f0 + 1][j] + s_part[3][f0 + 1][j]);
                    r.z = (s_part[0][f0 + 2][j] + s_part[1][f0 + 2][j]) + (s_part[2][f0 + 2][j] + s_part[3][f0 + 2][j]);
                    r.w = (s_part[0][f0 + 3][j] + s_part[1][f0 + 3][j]) + (s_part[2][f0 + 3][j] + s_part[3][f0 + 3][j]);
                } else {
                    r.y = r.z = r.w = 0.f;
                }
                a.records[3 * ((size_t)range.x + lo + j) + q] = r;
            }
        }
        __syncthreads();
    }
    if (a.diag) {
        __shared__ uint32_t s_kept[4];
        if (lane == 0) s_kept[w] = diag_kept;
        __syncthreads();
        if (tid == 0) {
            uint64_t* d = a.diag + 4 * (size_t)tile;
            d[0] = t_start;
            d[1] = __builtin_amdgcn_s_memrealtime();
            d[2] = (uint64_t)s_kept[0] + s_kept[1] + s_kept[2] + s_kept[3];
            d[3] = diag_rounds;
        }
    }
}

void launch_render_backward(const RenderBwdArgs& a, hipStream_t s) {
    const int tiles = a.gx * a.gy;
    if (tiles <= 0) return;
    hipLaunchKernelGGL(k_render_bwd, dim3(tiles), dim3(256), 0, s, a);
}

}  // namespace gs
