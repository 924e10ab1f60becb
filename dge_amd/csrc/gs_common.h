// gs_common.h — device-side building blocks shared by the gfx950 kernels.
//
// The per-Gaussian math restates the reference rasterizer
// (gaussiansplatting/submodules/diff-gaussian-rasterization/cuda_rasterizer/
//  forward.cu, backward.cu, auxiliary.h); every helper cites the lines whose
// numerics it must reproduce.  Matrices are the reference's float[16]
// (column-major transforms, auxiliary.h:58-97).
#pragma once

#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace gs {

constexpr int kTile = 16;             // BLOCK_X = BLOCK_Y (config.h:15-16)
constexpr int kTilePixels = kTile * kTile;
constexpr int kWave = 64;             // CDNA wavefront
constexpr int kQuad = 8;              // a wave rasterises one 8x8 quadrant of a tile

// auxiliary.h:22-39
__device__ constexpr float kSH_C0 = 0.28209479177387814f;
__device__ constexpr float kSH_C1 = 0.4886025119029199f;
__device__ constexpr float kSH_C2_0 = 1.0925484305920792f;
__device__ constexpr float kSH_C2_1 = -1.0925484305920792f;
__device__ constexpr float kSH_C2_2 = 0.31539156525252005f;
__device__ constexpr float kSH_C2_3 = -1.0925484305920792f;
__device__ constexpr float kSH_C2_4 = 0.5462742152960396f;
__device__ constexpr float kSH_C3_0 = -0.5900435899266435f;
__device__ constexpr float kSH_C3_1 = 2.890611442640554f;
__device__ constexpr float kSH_C3_2 = -0.4570457994644658f;
__device__ constexpr float kSH_C3_3 = 0.3731763325901154f;
__device__ constexpr float kSH_C3_4 = -0.4570457994644658f;
__device__ constexpr float kSH_C3_5 = 1.445305721320277f;
__device__ constexpr float kSH_C3_6 = -0.5900435899266435f;

struct f3 {
    float x, y, z;
};
__device__ __forceinline__ f3 mk3(float x, float y, float z) { return f3{x, y, z}; }
__device__ __forceinline__ f3 operator+(f3 a, f3 b) { return mk3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ f3 operator-(f3 a, f3 b) { return mk3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ f3 operator*(f3 a, float s) { return mk3(a.x * s, a.y * s, a.z * s); }
__device__ __forceinline__ float dot3(f3 a, f3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ f3 ld3(const float* p) { return mk3(p[0], p[1], p[2]); }

// Camera constants, read once per thread from device memory (uniform ->
// scalar loads).
struct Camera {
    float v[16];  // viewmatrix
    float p[16];  // projmatrix
};

__device__ __forceinline__ void load_camera(const float* __restrict__ view, const float* __restrict__ proj, Camera& c) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        c.v[i] = view[i];
        c.p[i] = proj[i];
    }
}

// auxiliary.h:58-66
__device__ __forceinline__ f3 view_point(const float* m, f3 p) {
    return mk3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
               m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
// auxiliary.h:68-77
__device__ __forceinline__ float4 proj_point(const float* m, f3 p) {
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12], m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14], m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}

// auxiliary.h:41-44 — the 1.0 literals make the reference evaluate in double.
__device__ __forceinline__ float ndc_to_pixel(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

// auxiliary.h:46-56 (float arithmetic, truncation toward zero, clamp to grid)
struct Rect {
    int x0, y0, x1, y1;
};
__device__ __forceinline__ Rect tile_rect(float px, float py, int r, int gx, int gy) {
    Rect q;
    q.x0 = min(gx, max(0, (int)((px - (float)r) / (float)kTile)));
    q.y0 = min(gy, max(0, (int)((py - (float)r) / (float)kTile)));
    q.x1 = min(gx, max(0, (int)((((px + (float)r) + (float)kTile) - 1.0f) / (float)kTile)));
    q.y1 = min(gy, max(0, (int)((((py + (float)r) + (float)kTile) - 1.0f) / (float)kTile)));
    return q;
}

// forward.cu:118-152 — Sigma = (S R)^T (S R) with R from the UNnormalised
// quaternion (w,x,y,z).  Output: upper triangle [00,01,02,11,12,22].
__device__ __forceinline__ void cov3d_from_scale_rot(f3 scale, float mod, float4 q, float cov[6]) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    // rows of the rotation matrix in the reference's (column-major) layout:
    // Rg[c][r] below is glm's R[c][r]
    const float R00 = 1.f - 2.f * (y * y + z * z), R01 = 2.f * (x * y - r * z), R02 = 2.f * (x * z + r * y);
    const float R10 = 2.f * (x * y + r * z), R11 = 1.f - 2.f * (x * x + z * z), R12 = 2.f * (y * z - r * x);
    const float R20 = 2.f * (x * z - r * y), R21 = 2.f * (y * z + r * x), R22 = 1.f - 2.f * (x * x + y * y);
    const float sx = mod * scale.x, sy = mod * scale.y, sz = mod * scale.z;
    // M[c][r] = s_r * R[c][r]; Sigma[c][r] = sum_k M[r][k] * M[c][k]
    const float M00 = sx * R00, M01 = sy * R01, M02 = sz * R02;
    const float M10 = sx * R10, M11 = sy * R11, M12 = sz * R12;
    const float M20 = sx * R20, M21 = sy * R21, M22 = sz * R22;
    cov[0] = M00 * M00 + M01 * M01 + M02 * M02;
    cov[1] = M10 * M00 + M11 * M01 + M12 * M02;
    cov[2] = M20 * M00 + M21 * M01 + M22 * M02;
    cov[3] = M10 * M10 + M11 * M11 + M12 * M12;
    cov[4] = M20 * M10 + M21 * M11 + M22 * M12;
    cov[5] = M20 * M20 + M21 * M21 + M22 * M22;
}

// The EWA projection of forward.cu:74-113 / backward.cu:160-199.
// T holds the two non-zero rows of (J * W_rot) as T[i][j], i in {0,1}
// (= glm T[i][j] in the reference); V is the symmetric 3D covariance.
struct Ewa {
    f3 t;                    // clamped camera-space mean
    float txtz, tytz, limx, limy;
    float J00, J02, J11, J12;
    float T[2][3];
    float V[3][3];
};

__device__ __forceinline__ void ewa_setup(f3 mean, float fx, float fy, float tanfovx, float tanfovy,
                                          const float cov3D[6], const float* v, Ewa& e) {
    f3 t = view_point(v, mean);
    e.limx = 1.3f * tanfovx;
    e.limy = 1.3f * tanfovy;
    e.txtz = t.x / t.z;
    e.tytz = t.y / t.z;
    t.x = fminf(e.limx, fmaxf(-e.limx, e.txtz)) * t.z;
    t.y = fminf(e.limy, fmaxf(-e.limy, e.tytz)) * t.z;
    e.t = t;
    e.J00 = fx / t.z;
    e.J02 = -(fx * t.x) / (t.z * t.z);
    e.J11 = fy / t.z;
    e.J12 = -(fy * t.y) / (t.z * t.z);
    // W (glm) = mat3(v0,v4,v8, v1,v5,v9, v2,v6,v10): W[k][r] = v[k + 4r]
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        e.T[0][j] = v[4 * j] * e.J00 + v[4 * j + 2] * e.J02;
        e.T[1][j] = v[4 * j + 1] * e.J11 + v[4 * j + 2] * e.J12;
    }
    e.V[0][0] = cov3D[0]; e.V[0][1] = cov3D[1]; e.V[0][2] = cov3D[2];
    e.V[1][0] = cov3D[1]; e.V[1][1] = cov3D[3]; e.V[1][2] = cov3D[4];
    e.V[2][0] = cov3D[2]; e.V[2][1] = cov3D[4]; e.V[2][2] = cov3D[5];
}

// (T V)_i,k = sum_m T[i][m] V[k][m]
__device__ __forceinline__ float tv(const Ewa& e, int i, int k) {
    return e.T[i][0] * e.V[k][0] + e.T[i][1] * e.V[k][1] + e.T[i][2] * e.V[k][2];
}

// forward.cu:106-112: filtered 2D covariance (a, b, c)
__device__ __forceinline__ void ewa_cov2d(const Ewa& e, float& a, float& b, float& c) {
    const float B00 = tv(e, 0, 0), B01 = tv(e, 0, 1), B02 = tv(e, 0, 2);
    const float B10 = tv(e, 1, 0), B11 = tv(e, 1, 1), B12 = tv(e, 1, 2);
    a = (B00 * e.T[0][0] + B01 * e.T[0][1] + B02 * e.T[0][2]) + 0.3f;
    b = B10 * e.T[0][0] + B11 * e.T[0][1] + B12 * e.T[0][2];
    c = (B10 * e.T[1][0] + B11 * e.T[1][1] + B12 * e.T[1][2]) + 0.3f;
}

// ---------------------------------------------------------------------
// The blend's exp (forward.cu:345 `exp(power)`, backward.cu:495).
// The reference compiles CUDA's expf (<= 2 ulp, not reproducible off an
// NVIDIA GPU); the skip / stop decisions of the blend (alpha >= 1/255,
// T (1 - alpha) >= 1e-4) and therefore n_contrib, the per-pixel lists and the
// whole T chain depend on the last bit of every G.  So the exp here is a fixed
// sequence of IEEE single operations that the CPU oracle (oracle/gs_oracle.c
// gs_expf) evaluates identically: G, alpha, T and every blend decision are
// bit-identical between the two.
//   u = fma(x, log2e, S)        S = 1.5 * 2^23: u = S + rint(x log2e), the product unrounded (round 5:
//                               one fma where a multiply and an add were: 2 VALU less per group of four)
//   u = clamp(u, S - 120, S + 120)
//   n = u - S;  r = fma(n, -ln2, x)            (|r| <= ln2 / 2 for |x log2e| <= 120)
//   p = degree-7 Taylor/Horner in fma;  result = p * 2^n  (2^n from u's bits)
// Accuracy: <= 0.86 ulp against exp on [-6, 0] (every float), <= 0.97 ulp on [-10, 1].  NaN -> NaN (r is
// NaN: the reference then blends the entry at alpha = min(0.99, NaN) = 0.99, and so do we); -inf and
// x << -83 (u clamped, r huge and negative) give p -> -inf or a negative value (odd degree), alpha < 1/255:
// skipped, as exp's 0 is.  The clamp keeps 2^n a normal number, so p * 2^n is exact.
// Why not a 2^(j/64) table + a short polynomial (round-4 verdict): the Horner steps are packed (v_pk_fma_f32:
// half an instruction per entry each), so a degree-3 polynomial saves 2 VALU per entry while the table costs
// the index arithmetic (2), an LDS read per entry in a loop already bound by LDS reads of its operands, and a
// second reduction constant (2 fma: |n| grows 64x) — no fewer instructions, and a longer dependency chain.
// A degree-6 minimax polynomial (one packed step less) loses the odd-degree sign for x << -83.
// ---------------------------------------------------------------------
typedef float f2v __attribute__((ext_vector_type(2)));  // two entries per packed instruction

constexpr float kExpLog2e = 1.44269504f;
constexpr float kExpShifter = 12582912.0f;  // 1.5 * 2^23: x log2e + S rounds to S + an integer (ties to even)
constexpr float kExpLo = kExpShifter - 120.0f, kExpHi = kExpShifter + 120.0f;
constexpr float kExpLn2 = 0.693147182f;
constexpr float kExpC7 = 1.98412698e-4f, kExpC6 = 1.38888889e-3f, kExpC5 = 8.33333377e-3f,
                kExpC4 = 4.16666679e-2f, kExpC3 = 1.66666672e-1f;

__device__ __forceinline__ float exp_scale(float u) {  // 2^n from the shifter sum u = S + n
    return __uint_as_float((__float_as_uint(u) << 23) + 0x3F800000u);
}

#ifdef GS_HW_EXP
// (A/B measurement only, tools/probes/exp_flips.py: the hardware v_exp_f32 on x log2e, __expf's sequence — not
// reproducible on the CPU, so the oracle's blend decisions become flips)
__device__ __forceinline__ float gs_exp(float x) { return __builtin_amdgcn_exp2f(x * kExpLog2e); }
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4v gs_exp4(f4v x) {
    return f4v{gs_exp(x.x), gs_exp(x.y), gs_exp(x.z), gs_exp(x.w)};
}
#else
__device__ __forceinline__ float gs_exp(float x) {
#pragma clang fp contract(off)
    float u = __builtin_fmaf(x, kExpLog2e, kExpShifter);
    u = fminf(fmaxf(u, kExpLo), kExpHi);
    const float n = u - kExpShifter;
    const float r = __builtin_fmaf(n, -kExpLn2, x);
    float p = __builtin_fmaf(kExpC7, r, kExpC6);
    p = __builtin_fmaf(p, r, kExpC5);
    p = __builtin_fmaf(p, r, kExpC4);
    p = __builtin_fmaf(p, r, kExpC3);
    p = __builtin_fmaf(p, r, 0.5f);
    p = __builtin_fmaf(p, r, 1.0f);
    p = __builtin_fmaf(p, r, 1.0f);
    return p * exp_scale(u);
}

// gs_exp of four values: two independent packed streams, so each dependent
// v_pk_fma of one stream issues behind the other's (no hazard nops between the
// Horner steps, which a single packed chain needs on gfx950)
typedef float f4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4v gs_exp4(f4v x) {
#pragma clang fp contract(off)
    const f4v c = {1.0f, 1.0f, 1.0f, 1.0f};
    f4v u = __builtin_elementwise_fma(x, kExpLog2e * c, kExpShifter * c);
    u.x = fminf(fmaxf(u.x, kExpLo), kExpHi);
    u.y = fminf(fmaxf(u.y, kExpLo), kExpHi);
    u.z = fminf(fmaxf(u.z, kExpLo), kExpHi);
    u.w = fminf(fmaxf(u.w, kExpLo), kExpHi);
    const f4v n = u - kExpShifter;
    const f4v r = __builtin_elementwise_fma(n, -kExpLn2 * c, x);
    f4v p = __builtin_elementwise_fma(kExpC7 * c, r, kExpC6 * c);
    p = __builtin_elementwise_fma(p, r, kExpC5 * c);
    p = __builtin_elementwise_fma(p, r, kExpC4 * c);
    p = __builtin_elementwise_fma(p, r, kExpC3 * c);
    p = __builtin_elementwise_fma(p, r, 0.5f * c);
    p = __builtin_elementwise_fma(p, r, c);
    p = __builtin_elementwise_fma(p, r, c);
    return p * f4v{exp_scale(u.x), exp_scale(u.y), exp_scale(u.z), exp_scale(u.w)};
}
#endif

// GaussianModel activations (gaussian_model.py:42-57): sigmoid, exp,
// F.normalize(q, dim=1, eps=1e-12) and their derivatives (what torch's
// autograd applies to the getters in the reference's render()).
__device__ __forceinline__ float act_sigmoid(float x) { return 1.0f / (1.0f + expf(-x)); }
__device__ __forceinline__ float4 act_normalize(float4 q, float& norm_out) {
    const float len = sqrtf(q.x * q.x + q.y * q.y + q.z * q.z + q.w * q.w);
    const float n = fmaxf(len, 1e-12f);
    norm_out = len;
    return make_float4(q.x / n, q.y / n, q.z / n, q.w / n);
}
// d(q / max(|q|, eps)) / dq applied to g, given y = normalized q
__device__ __forceinline__ float4 act_normalize_bwd(float4 y, float len, float4 g) {
    if (len > 1e-12f) {
        const float d = y.x * g.x + y.y * g.y + y.z * g.z + y.w * g.w;
        return make_float4((g.x - y.x * d) / len, (g.y - y.y * d) / len, (g.z - y.z * d) / len, (g.w - y.w * d) / len);
    }
    return make_float4(g.x / 1e-12f, g.y / 1e-12f, g.z / 1e-12f, g.w / 1e-12f);
}

// ---------------------------------------------------------------------
// wave-level primitives (64 lanes)
// ---------------------------------------------------------------------
__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ uint64_t lanemask_lt() { return (1ull << lane_id()) - 1ull; }

// Conservative test: can Gaussian (xy, conic, opacity) reach alpha >= 1/255
// at any pixel of the box [bx0,bx0+7] x [by0,by0+7]?  alpha = min(.99, o*G),
// G = exp(-q/2), q = a dx^2 + 2 b dx dy + c dy^2, d = xy - pixel.
// Shared by the blend kernels and k_gauss_bwd (which re-derives from it which
// quadrant records exist), so contraction is pinned: every caller evaluates
// the identical instruction sequence and takes the identical decision.
__device__ __forceinline__ bool cull_keep(float2 xy, float4 co, float bx0, float by0) {
#pragma clang fp contract(off)
    const float o = co.w;
    if (o < 1.0f / 255.0f) return false;  // alpha <= o*G <= o   (NaN falls through: keep)
    const float a = co.x, b = co.y, c = co.z;
    if (!(a > 0.f && c > 0.f && a * c - b * b > 0.f)) return true;  // not positive definite: no bound
    // (v_log_f32: 255 o >= 1 here, no denormal; the slack below absorbs its ~1-ulp error)
    const float thr = (2.0f * 0.693147182f) * __builtin_amdgcn_logf(255.0f * o);
    const float X0 = xy.x - (bx0 + 7.0f), X1 = xy.x - bx0;
    const float Y0 = xy.y - (by0 + 7.0f), Y1 = xy.y - by0;
    if (X0 <= 0.f && X1 >= 0.f && Y0 <= 0.f && Y1 >= 0.f) return true;
    const float slack = 2e-3f * (1.0f + fabsf(thr));
    // the minimisers below only choose WHERE the quadratic is evaluated: a 1-ulp reciprocal moves them by
    // ~1e-7 relative, which changes the evaluated value at second order, far inside the slack (an IEEE
    // division here was ~40 of the cull's ~136 VALU per 64 list positions)
    const float rc = __builtin_amdgcn_rcpf(c), ra = __builtin_amdgcn_rcpf(a);
    // the smallest of the four edge minima against the level (fminf drops a NaN edge, which could
    // not pass its own comparison either)
    float qmin;
    // edges dx = X: minimise over dy
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const float X = e ? X1 : X0;
        const float dy = fminf(Y1, fmaxf(Y0, (-b * X) * rc));
        const float t1 = a * X * X, t2 = 2.f * b * X * dy, t3 = c * dy * dy;
        const float q = (t1 + t2 + t3) - 1e-5f * (t1 + fabsf(t2) + t3);
        qmin = e ? fminf(qmin, q) : q;
    }
#pragma unroll
    for (int e = 0; e < 2; ++e) {
        const float Y = e ? Y1 : Y0;
        const float dx = fminf(X1, fmaxf(X0, (-b * Y) * ra));
        const float t1 = a * dx * dx, t2 = 2.f * b * dx * Y, t3 = c * Y * Y;
        qmin = fminf(qmin, (t1 + t2 + t3) - 1e-5f * (t1 + fabsf(t2) + t3));
    }
    return qmin <= thr + slack;
}

// =====================================================================
// SH coefficient rows staged through LDS (k_preprocess, k_gauss_bwd):
// coalesced block-wide global transfers instead of 45 strided dword
// accesses per lane.  NT = threads (= Gaussians) per block.
// =====================================================================
// Output store: out = v, or out += v when the output's GS_ACC_* bit is set
// (fused gradient accumulation into an existing .grad buffer).
__device__ __forceinline__ void put_out(float* p, size_t i, float v, bool acc) { p[i] = acc ? p[i] + v : v; }

constexpr int kShPitch = 45;  // LDS floats per Gaussian row: (16-1)*3, odd -> conflict-free row access

// Coalesced block transfer of the SH "rest" rows of Gaussians [idx0, idx0+nrow)
// between global rows of `stride` floats and LDS rows of kShPitch floats;
// only the first ncol floats of each row are moved (the tail of an
// interleaved [P,16,3] row is the next Gaussian's DC term: never touched).
// When the block's region is 16-B aligned (contiguous [P,15,3] parameters)
// the global side moves float4s; every load of a thread is issued before
// its first LDS store, so ~12 x 16 B per lane are in flight at once.
__device__ __forceinline__ void sh_element_to_lds(float* __restrict__ lds, int e, float v, float inv, int stride,
                                                  int ncol) {
    const int row = (int)(((float)e + 0.5f) * inv);  // exact: e < 2^16, margin 0.5/stride
    const int col = e - row * stride;
    if (col < ncol) lds[row * kShPitch + col] = v;
}

// Dense rows: does float4 i of the block's region hold a float of a live row?
// (a float4 spans at most two rows of 45 floats)
__device__ __forceinline__ bool dense_f4_live(const uint8_t* live, int i) {
    return !live || (live[(4 * i) / kShPitch] | live[(4 * i + 3) / kShPitch]);
}

// `live` (LDS, one byte per row, nullable): rows whose Gaussian needs its SH;
// the dense path skips the loads of the other rows (their LDS rows are left
// undefined: the caller does not read them).
template <int NT>
__device__ __forceinline__ void sh_rows_load(const float* __restrict__ g, int stride, float* __restrict__ lds,
                                             int nrow, int ncol, const uint8_t* live = nullptr) {
    const int total = (nrow - 1) * stride + ncol;
    const float inv = 1.0f / (float)stride;
    if (stride == kShPitch && ncol == kShPitch && (reinterpret_cast<uintptr_t>(g) & 15) == 0) {
        // dense [P,15,3] rows (the raw-parameter path): the LDS image is the global one
        constexpr int kV = 12;
        const float4* g4 = reinterpret_cast<const float4*>(g);
        float4* l4 = reinterpret_cast<float4*>(lds);
        const int n4 = total >> 2;
        for (int b = 0; b < n4; b += kV * NT) {
            float4 v[kV];
#pragma unroll
            for (int u = 0; u < kV; ++u) {
                const int i = b + u * NT + (int)threadIdx.x;
                v[u] = i < n4 && dense_f4_live(live, i) ? g4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < kV; ++u) {
                const int i = b + u * NT + (int)threadIdx.x;
                if (i < n4) l4[i] = v[u];
            }
        }
        for (int e = 4 * n4 + (int)threadIdx.x; e < total; e += NT) lds[e] = g[e];
    } else if ((reinterpret_cast<uintptr_t>(g) & 15) == 0) {
        constexpr int kV = 12;  // float4 per lane per batch: 256 x 45 floats = 2880 float4
        const float4* g4 = reinterpret_cast<const float4*>(g);
        const int n4 = total >> 2;
        for (int b = 0; b < n4; b += kV * NT) {
            float4 v[kV];
#pragma unroll
            for (int u = 0; u < kV; ++u) {
                const int i = b + u * NT + (int)threadIdx.x;
                v[u] = i < n4 ? g4[i] : make_float4(0.f, 0.f, 0.f, 0.f);
            }
#pragma unroll
            for (int u = 0; u < kV; ++u) {
                const int i = b + u * NT + (int)threadIdx.x;
                if (i < n4) {
                    sh_element_to_lds(lds, 4 * i, v[u].x, inv, stride, ncol);
                    sh_element_to_lds(lds, 4 * i + 1, v[u].y, inv, stride, ncol);
                    sh_element_to_lds(lds, 4 * i + 2, v[u].z, inv, stride, ncol);
                    sh_element_to_lds(lds, 4 * i + 3, v[u].w, inv, stride, ncol);
                }
            }
        }
        for (int e = 4 * n4 + (int)threadIdx.x; e < total; e += NT) sh_element_to_lds(lds, e, g[e], inv, stride, ncol);
    } else {
        constexpr int kV = 16;
        for (int b = 0; b < total; b += kV * NT) {
            float v[kV];
#pragma unroll
            for (int u = 0; u < kV; ++u) {
                const int e = b + u * NT + (int)threadIdx.x;
                v[u] = e < total ? g[e] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < kV; ++u) {
                const int e = b + u * NT + (int)threadIdx.x;
                if (e < total) sh_element_to_lds(lds, e, v[u], inv, stride, ncol);
            }
        }
    }
}

// With `accumulate`, the dense path skips float4s of rows that are not `live`
// (their gradient is zero: adding it is a no-op).
// fp16 SH rows (the local-edit path's storage): the same block transfer with
// 2-byte elements, upcast to fp32 in LDS.  Consecutive lanes read consecutive
// halves (128 B per wave instruction); a thread's loads are all issued first.
template <int NT>
__device__ __forceinline__ void sh_rows_load_half(const __half* __restrict__ g, int stride, float* __restrict__ lds,
                                                  int nrow, int ncol, const uint8_t* live = nullptr) {
    const int total = (nrow - 1) * stride + ncol;
    const float inv = 1.0f / (float)stride;
    constexpr int kV = 16;
    for (int b = 0; b < total; b += kV * NT) {
        __half v[kV];
#pragma unroll
        for (int u = 0; u < kV; ++u) {
            const int e = b + u * NT + (int)threadIdx.x;
            const int row = (int)(((float)e + 0.5f) * inv);
            v[u] = e < total && (!live || live[row]) ? g[e] : __float2half(0.f);
        }
#pragma unroll
        for (int u = 0; u < kV; ++u) {
            const int e = b + u * NT + (int)threadIdx.x;
            if (e < total) sh_element_to_lds(lds, e, __half2float(v[u]), inv, stride, ncol);
        }
    }
}

// coefficient 0 (3 values) of an SH row, fp32 or fp16
__device__ __forceinline__ f3 sh_dc3(const float* dc, int half, size_t off) {
    if (half) {
        const __half* h = reinterpret_cast<const __half*>(dc) + off;
        return mk3(__half2float(h[0]), __half2float(h[1]), __half2float(h[2]));
    }
    return ld3(dc + off);
}

template <int NT>
__device__ __forceinline__ void sh_rows_store(float* __restrict__ g, int stride, const float* __restrict__ lds,
                                              int nrow, int ncol, bool accumulate, const uint8_t* live = nullptr) {
    const int total = (nrow - 1) * stride + ncol;
    const float inv = 1.0f / (float)stride;
    auto at = [&](int e, float& v) {
        const int row = (int)(((float)e + 0.5f) * inv);
        const int col = e - row * stride;
        v = col < ncol ? lds[row * kShPitch + col] : 0.f;
        return col < ncol;
    };
    if (stride == kShPitch && ncol == kShPitch && (reinterpret_cast<uintptr_t>(g) & 15) == 0) {
        // dense [P,15,3] rows: the LDS image is the global one
        float4* g4 = reinterpret_cast<float4*>(g);
        const float4* l4 = reinterpret_cast<const float4*>(lds);
        const int n4 = total >> 2;
        for (int i = threadIdx.x; i < n4; i += NT) {
            if (accumulate && !dense_f4_live(live, i)) continue;
            float4 v = l4[i];
            if (accumulate) {
                const float4 o = g4[i];
                v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
            }
            g4[i] = v;
        }
        for (int e = 4 * n4 + (int)threadIdx.x; e < total; e += NT) put_out(g, e, lds[e], accumulate);
    } else if ((reinterpret_cast<uintptr_t>(g) & 15) == 0 && stride == ncol) {  // dense rows: float4 stores
        float4* g4 = reinterpret_cast<float4*>(g);
        const int n4 = total >> 2;
        for (int i = threadIdx.x; i < n4; i += NT) {
            float4 v;
            at(4 * i, v.x);
            at(4 * i + 1, v.y);
            at(4 * i + 2, v.z);
            at(4 * i + 3, v.w);
            if (accumulate) {
                const float4 o = g4[i];
                v = make_float4(o.x + v.x, o.y + v.y, o.z + v.z, o.w + v.w);
            }
            g4[i] = v;
        }
        for (int e = 4 * n4 + (int)threadIdx.x; e < total; e += NT) {
            float v;
            at(e, v);
            put_out(g, e, v, accumulate);
        }
    } else {
        for (int e = threadIdx.x; e < total; e += NT) {
            float v;
            if (at(e, v)) put_out(g, e, v, accumulate);
        }
    }
}

// Sum over the 64 lanes with DPP row ops; the total lands in lane 63.
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ float dpp_mov(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, ROW_MASK, 0xF, false));
}
__device__ __forceinline__ float wave_sum_to_lane63(float v) {
    v += dpp_mov<0xB1, 0xF>(v);   // quad_perm [1,0,3,2]
    v += dpp_mov<0x4E, 0xF>(v);   // quad_perm [2,3,0,1]
    v += dpp_mov<0x141, 0xF>(v);  // row_half_mirror
    v += dpp_mov<0x140, 0xF>(v);  // row_mirror
    v += dpp_mov<0x142, 0xA>(v);  // row_bcast:15 into rows 1,3
    v += dpp_mov<0x143, 0xC>(v);  // row_bcast:31 into rows 2,3
    return v;
}

// Sum over the 16 lanes of each row; every lane of the row gets the total.
// (every lane has a source in these patterns, so no `old` value is needed
// and each step folds into one v_add_f32_dpp)
template <int CTRL>
__device__ __forceinline__ float dpp_row(float v) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
__device__ __forceinline__ float row_sum16(float v) {
    v += dpp_row<0xB1>(v);   // quad_perm [1,0,3,2]
    v += dpp_row<0x4E>(v);   // quad_perm [2,3,0,1]
    v += dpp_row<0x141>(v);  // row_half_mirror
    v += dpp_row<0x140>(v);  // row_mirror
    return v;
}

// Reduce-scatter of four per-lane values over the 64 lanes with the gfx950
// lane swaps (v_permlane32_swap / v_permlane16_swap) and one row reduction:
// 3 swaps + 3 adds + 4 DPP adds for four sums instead of 4 x 6 DPP adds.
// Result: every lane of row 0 holds sum(a), row 1 sum(c), row 2 sum(b),
// row 3 sum(d).  Fixed summation order (deterministic).
__device__ __forceinline__ float quad_reduce_rows(float a, float b, float c, float d) {  // before the row sum
    const auto p = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    const float ab = __uint_as_float(p[0]) + __uint_as_float(p[1]);  // lanes 0-31: a, 32-63: b
    const auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(c), __float_as_uint(d), false, false);
    const float cd = __uint_as_float(q[0]) + __uint_as_float(q[1]);  // lanes 0-31: c, 32-63: d
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(ab), __float_as_uint(cd), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);  // rows: a, c, b, d (each still to be summed)
}
__device__ __forceinline__ float quad_reduce(float a, float b, float c, float d) {
    return row_sum16(quad_reduce_rows(a, b, c, d));
}

// row_sum16 of nine values at once, each step one v_add_f32_dpp.  (Written out: the compiler pairs the row
// sums' adds of two values into one v_pk_add_f32, which takes no DPP operand, so each step became a
// v_mov_b32_dpp per value plus half a packed add — 36 + 9 instructions where 36 do.)  Same adds in the same
// order as row_sum16 on each value, so the sums are bitwise row_sum16's.  A DPP read of a VGPR needs two wait
// states after the VALU write of it (the s_nop for the inputs); inside, a value is read again nine
// instructions after its write.
__device__ __forceinline__ void row_sum16_x9(float (&v)[9]) {
#define GS_DPP9(CTRL)                                                                                  \
    "v_add_f32_dpp %0, %0, %0 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                 \
    "v_add_f32_dpp %1, %1, %1 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                 \
    "v_add_f32_dpp %2, %2, %2 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                 \
    "v_add_f32_dpp %3, %3, %3 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                 \
    "v_add_f32_dpp %4, %4, %4 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                 \
    "v_add_f32_dpp %5, %5, %5 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                 \
    "v_add_f32_dpp %6, %6, %6 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                 \
    "v_add_f32_dpp %7, %7, %7 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"                 \
    "v_add_f32_dpp %8, %8, %8 " CTRL " row_mask:0xf bank_mask:0xf bound_ctrl:1\n\t"
    asm("s_nop 1\n\t" GS_DPP9("quad_perm:[1,0,3,2]") GS_DPP9("quad_perm:[2,3,0,1]") GS_DPP9("row_half_mirror")
            GS_DPP9("row_mirror")
        : "+v"(v[0]), "+v"(v[1]), "+v"(v[2]), "+v"(v[3]), "+v"(v[4]), "+v"(v[5]), "+v"(v[6]), "+v"(v[7]),
          "+v"(v[8]));
#undef GS_DPP9
}

__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o));
    return v;
}

}  // namespace gs
