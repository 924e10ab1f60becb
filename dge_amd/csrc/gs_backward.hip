// gs_backward.hip — per-Gaussian backward for gfx950, one thread per Gaussian.
//
// Fuses what the reference runs as three steps plus a memset:
//   * torch::zeros of the 9 gradient tensors (rasterize_points.cu:120-128):
//     not needed, every output element is written here;
//   * the sum of the per-pixel atomics of renderCUDA bwd (backward.cu:523-554):
//     here the sum of this Gaussian's per-tile records, read in tile order
//     (deterministic);
//   * computeCov2DCUDA (backward.cu:144-274) and preprocessCUDA bwd
//     (backward.cu:346-396) with computeColorFromSH bwd (:20-139) and
//     computeCov3D bwd (:278-341).
// The 3D covariance is recomputed from (scale, rotation) with the forward's
// own helper instead of being stored in the geometry buffer (-48 B/Gaussian
// of HBM traffic).
// Exact IEEE single-precision operations in the order written (no FMA
// contraction): the per-Gaussian geometry, depth keys, radii and tile rects
// then match the CPU restatement bit for bit, so the discrete outputs
// (num_rendered, radii, sorted tile lists) are identical, not just close.
// These kernels are HBM-bound; the extra multiplies cost nothing measurable.
#pragma clang fp contract(off)
#include "gs_common.h"
#include "gs_internal.h"
#include "gs_raster.h"  // GS_ACC_*

namespace gs {

// backward.cu:20-139 — the mean gradient through the normalised view direction
// (return value) and dL_dsh of the (deg+1)^2 used coefficients, times `msk`
// (the grad mask, 1 when none): coefficient 0 into ddc, coefficients 1..
// written over the input row r in place (after every read of it; ncol floats,
// zeros beyond the degree) — no 48-float register array.
// r: SH coefficients 1.. of this Gaussian (coefficient 0 has no direction term).
__device__ __forceinline__ f3 sh_backward(int deg, f3 pos, f3 campos, float* r, int ncol, uint8_t clamp_bits,
                                          f3 dL_dcolor, float msk, float (&ddc)[3]) {
    const f3 dir_orig = pos - campos;
    const float len = sqrtf(dot3(dir_orig, dir_orig));
    const f3 dir = mk3(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
    const f3 g = mk3(dL_dcolor.x * ((clamp_bits & 1) ? 0.f : 1.f), dL_dcolor.y * ((clamp_bits & 2) ? 0.f : 1.f),
                     dL_dcolor.z * ((clamp_bits & 4) ? 0.f : 1.f));
    // coefficient k >= 1 of the input
#define SHK(k) ld3(r + 3 * ((k) - 1))
    f3 dx = mk3(0, 0, 0), dy = mk3(0, 0, 0), dz = mk3(0, 0, 0);
    const float x = dir.x, y = dir.y, z = dir.z;
    if (deg > 0) {
        dx = SHK(3) * (-kSH_C1);
        dy = SHK(1) * (-kSH_C1);
        dz = SHK(2) * kSH_C1;
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            dx = dx + (SHK(4) * (kSH_C2_0 * y) + SHK(6) * (kSH_C2_2 * 2.f * -x) + SHK(7) * (kSH_C2_3 * z) +
                       SHK(8) * (kSH_C2_4 * 2.f * x));
            dy = dy + (SHK(4) * (kSH_C2_0 * x) + SHK(5) * (kSH_C2_1 * z) + SHK(6) * (kSH_C2_2 * 2.f * -y) +
                       SHK(8) * (kSH_C2_4 * 2.f * -y));
            dz = dz + (SHK(5) * (kSH_C2_1 * y) + SHK(6) * (kSH_C2_2 * 2.f * 2.f * z) + SHK(7) * (kSH_C2_3 * x));
            if (deg > 2) {
                dx = dx + (SHK(9) * (kSH_C3_0 * 3.f * 2.f * xy) + SHK(10) * (kSH_C3_1 * yz) +
                           SHK(11) * (kSH_C3_2 * -2.f * xy) + SHK(12) * (kSH_C3_3 * -3.f * 2.f * xz) +
                           SHK(13) * (kSH_C3_4 * (-3.f * xx + 4.f * zz - yy)) + SHK(14) * (kSH_C3_5 * 2.f * xz) +
                           SHK(15) * (kSH_C3_6 * 3.f * (xx - yy)));
                dy = dy + (SHK(9) * (kSH_C3_0 * 3.f * (xx - yy)) + SHK(10) * (kSH_C3_1 * xz) +
                           SHK(11) * (kSH_C3_2 * (-3.f * yy + 4.f * zz - xx)) + SHK(12) * (kSH_C3_3 * -3.f * 2.f * yz) +
                           SHK(13) * (kSH_C3_4 * -2.f * xy) + SHK(14) * (kSH_C3_5 * -2.f * yz) +
                           SHK(15) * (kSH_C3_6 * -3.f * 2.f * xy));
                dz = dz + (SHK(10) * (kSH_C3_1 * xy) + SHK(11) * (kSH_C3_2 * 4.f * 2.f * yz) +
                           SHK(12) * (kSH_C3_3 * 3.f * (2.f * zz - xx - yy)) + SHK(13) * (kSH_C3_4 * 4.f * 2.f * xz) +
                           SHK(14) * (kSH_C3_5 * (xx - yy)));
            }
        }
    }
#undef SHK
    // every read of r is done: the coefficient gradients overwrite it
    auto put = [&](int k, f3 v) {
        v = v * msk;
        if (k == 0) {
            ddc[0] = v.x;
            ddc[1] = v.y;
            ddc[2] = v.z;
            return;
        }
        const int c = 3 * (k - 1);
        if (c < ncol) r[c] = v.x;
        if (c + 1 < ncol) r[c + 1] = v.y;
        if (c + 2 < ncol) r[c + 2] = v.z;
    };
    const f3 zero = mk3(0.f, 0.f, 0.f);
    put(0, g * kSH_C0);
    put(1, deg > 0 ? g * (-kSH_C1 * y) : zero);
    put(2, deg > 0 ? g * (kSH_C1 * z) : zero);
    put(3, deg > 0 ? g * (-kSH_C1 * x) : zero);
    {
        const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
        put(4, deg > 1 ? g * (kSH_C2_0 * xy) : zero);
        put(5, deg > 1 ? g * (kSH_C2_1 * yz) : zero);
        put(6, deg > 1 ? g * (kSH_C2_2 * (2.f * zz - xx - yy)) : zero);
        put(7, deg > 1 ? g * (kSH_C2_3 * xz) : zero);
        put(8, deg > 1 ? g * (kSH_C2_4 * (xx - yy)) : zero);
        put(9, deg > 2 ? g * (kSH_C3_0 * y * (3.f * xx - yy)) : zero);
        put(10, deg > 2 ? g * (kSH_C3_1 * xy * z) : zero);
        put(11, deg > 2 ? g * (kSH_C3_2 * y * (4.f * zz - xx - yy)) : zero);
        put(12, deg > 2 ? g * (kSH_C3_3 * z * (2.f * zz - 3.f * xx - 3.f * yy)) : zero);
        put(13, deg > 2 ? g * (kSH_C3_4 * x * (4.f * zz - xx - yy)) : zero);
        put(14, deg > 2 ? g * (kSH_C3_5 * z * (xx - yy)) : zero);
        put(15, deg > 2 ? g * (kSH_C3_6 * x * (xx - 3.f * yy)) : zero);
    }
    const f3 dL_ddir = mk3(dot3(dx, g), dot3(dy, g), dot3(dz, g));
    // dnormvdv (auxiliary.h:107-117)
    const f3 v = dir_orig;
    const float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    const float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    return mk3(((+sum2 - v.x * v.x) * dL_ddir.x - v.y * v.x * dL_ddir.y - v.z * v.x * dL_ddir.z) * invsum32,
               (-v.x * v.y * dL_ddir.x + (sum2 - v.y * v.y) * dL_ddir.y - v.z * v.y * dL_ddir.z) * invsum32,
               (-v.x * v.z * dL_ddir.x - v.y * v.z * dL_ddir.y + (sum2 - v.z * v.z) * dL_ddir.z) * invsum32);
}

// backward.cu:278-341 (gradient w.r.t. mod*scale and the unnormalised quaternion)
__device__ __forceinline__ void cov3d_backward(f3 scale, float mod, float4 q, const float dc[6], float* dscale,
                                               float* drot) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    float R[3][3];  // glm R[c][r]
    R[0][0] = 1.f - 2.f * (y * y + z * z); R[0][1] = 2.f * (x * y - r * z); R[0][2] = 2.f * (x * z + r * y);
    R[1][0] = 2.f * (x * y + r * z); R[1][1] = 1.f - 2.f * (x * x + z * z); R[1][2] = 2.f * (y * z - r * x);
    R[2][0] = 2.f * (x * z - r * y); R[2][1] = 2.f * (y * z + r * x); R[2][2] = 1.f - 2.f * (x * x + y * y);
    const float s[3] = {mod * scale.x, mod * scale.y, mod * scale.z};
    float S2M[3][3];  // (2 * M)[c][r] with M = S * R  ->  M[c][r] = s_r R[c][r]
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) S2M[c][rr] = 2.0f * (s[rr] * R[c][rr]);
    float dS[3][3];  // dL_dSigma, glm column-major, symmetric
    dS[0][0] = dc[0]; dS[0][1] = 0.5f * dc[1]; dS[0][2] = 0.5f * dc[2];
    dS[1][0] = 0.5f * dc[1]; dS[1][1] = dc[3]; dS[1][2] = 0.5f * dc[4];
    dS[2][0] = 0.5f * dc[2]; dS[2][1] = 0.5f * dc[4]; dS[2][2] = dc[5];
    float dM[3][3];  // glm product (2M) * dSigma
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int rr = 0; rr < 3; ++rr)
            dM[c][rr] = S2M[0][rr] * dS[c][0] + S2M[1][rr] * dS[c][1] + S2M[2][rr] * dS[c][2];
    // dL_dscale[i] = dot(Rt[i], dMt[i]) = sum_r R[r][i] dM[r][i]
#pragma unroll
    for (int i = 0; i < 3; ++i) dscale[i] = R[0][i] * dM[0][i] + R[1][i] * dM[1][i] + R[2][i] * dM[2][i];
    float D[3][3];  // dMt[c][r] * s_c = dM[r][c] * s_c
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int rr = 0; rr < 3; ++rr) D[c][rr] = dM[rr][c] * s[c];
    drot[0] = 2 * z * (D[0][1] - D[1][0]) + 2 * y * (D[2][0] - D[0][2]) + 2 * x * (D[1][2] - D[2][1]);
    drot[1] = 2 * y * (D[1][0] + D[0][1]) + 2 * z * (D[2][0] + D[0][2]) + 2 * r * (D[1][2] - D[2][1]) - 4 * x * (D[2][2] + D[1][1]);
    drot[2] = 2 * x * (D[1][0] + D[0][1]) + 2 * r * (D[2][0] - D[0][2]) + 2 * z * (D[1][2] + D[2][1]) - 4 * y * (D[2][2] + D[0][0]);
    drot[3] = 2 * r * (D[0][1] - D[1][0]) + 2 * x * (D[2][0] + D[0][2]) + 2 * y * (D[1][2] + D[2][1]) - 4 * z * (D[1][1] + D[0][0]);
}

constexpr int kGB = 256;  // Gaussians per block

// Per-Gaussian inputs, loaded at kernel entry so their latency overlaps the
// SH staging and the record sums.
struct GaussIn {
    f3 m;
    f3 scale;
    float4 rot;
    float cov[6];
    float opacity;
    uint8_t clamped;
};

// idx: the Gaussian in the render (its clamp bits); src: its parameter row (gs_params.index)
__device__ __forceinline__ GaussIn load_gauss_in(const GaussBwdArgs& a, int idx, int src) {
    GaussIn g;
    g.m = ld3(a.means3D + 3 * (size_t)src);
    g.scale = mk3(0, 0, 0);
    g.rot = make_float4(0, 0, 0, 0);
#pragma unroll
    for (int k = 0; k < 6; ++k) g.cov[k] = 0.f;
    if (a.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; ++k) g.cov[k] = a.cov3D_precomp[6 * (size_t)src + k];
    } else {
        g.scale = ld3(a.scales + 3 * (size_t)src);
        g.rot = *reinterpret_cast<const float4*>(a.rotations + 4 * (size_t)src);
    }
    g.opacity = a.activation ? a.opacities[src] : 0.f;
    g.clamped = a.clamped[idx];
    return g;
}

// Gradients of one live Gaussian w.r.t. its inputs, in registers: they are
// committed afterwards with every load of an accumulated output issued before
// the first store (see commit_outputs).
struct GaussOut {
    f3 dmean;
    float dcov[6];
    float dscale[3];
    float4 drot;
};

// The per-Gaussian chain of a live Gaussian (geometry gradients into `o`,
// SH gradients into dsh, opacity gradient chained into dop).
__device__ __forceinline__ void gauss_bwd_visible(const GaussBwdArgs& a, const GaussIn& gin, const float (&acc)[9],
                                                  float& dop, float* my_sh, int ncol, float sh_msk, float (&ddc)[3],
                                                  GaussOut& o) {
    const float* v = a.view;
    const float* pm = a.proj;
    const f3 m = gin.m;
    float cov3[6];
    f3 scale = mk3(0, 0, 0);
    float4 rot = make_float4(0, 0, 0, 0), rot_raw = rot;
    float rot_len = 0.f;
    if (a.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; ++k) cov3[k] = gin.cov[k];
    } else {
        scale = gin.scale;
        rot = gin.rot;
        if (a.activation) {
            rot_raw = rot;
            rot = act_normalize(rot_raw, rot_len);
            scale = mk3(expf(scale.x), expf(scale.y), expf(scale.z));
        }
        cov3d_from_scale_rot(scale, a.scale_modifier, rot, cov3);
    }

    // ---- computeCov2DCUDA (backward.cu:144-274) ----
    Ewa e;
    ewa_setup(m, a.fx, a.fy, a.tanfovx, a.tanfovy, cov3, v, e);
    const float x_grad_mul = e.txtz < -e.limx || e.txtz > e.limx ? 0.f : 1.f;
    const float y_grad_mul = e.tytz < -e.limy || e.tytz > e.limy ? 0.f : 1.f;
    float ca, cb, cc;
    ewa_cov2d(e, ca, cb, cc);
    const float dcx = acc[2], dcy = acc[3], dcw = acc[4];  // dL_dconic x, y, w
    const float denom = ca * cc - cb * cb;
    float dL_da = 0.f, dL_db = 0.f, dL_dc = 0.f;
    const float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    float dcov[6];
    const float(&T)[2][3] = e.T;
    if (denom2inv != 0) {
        dL_da = denom2inv * (-cc * cc * dcx + 2 * cb * cc * dcy + (denom - ca * cc) * dcw);
        dL_dc = denom2inv * (-ca * ca * dcw + 2 * ca * cb * dcy + (denom - ca * cc) * dcx);
        dL_db = denom2inv * 2 * (cb * cc * dcx - (denom + 2 * cb * cb) * dcy + ca * cb * dcw);
        dcov[0] = (T[0][0] * T[0][0] * dL_da + T[0][0] * T[1][0] * dL_db + T[1][0] * T[1][0] * dL_dc);
        dcov[3] = (T[0][1] * T[0][1] * dL_da + T[0][1] * T[1][1] * dL_db + T[1][1] * T[1][1] * dL_dc);
        dcov[5] = (T[0][2] * T[0][2] * dL_da + T[0][2] * T[1][2] * dL_db + T[1][2] * T[1][2] * dL_dc);
        dcov[1] = 2 * T[0][0] * T[0][1] * dL_da + (T[0][0] * T[1][1] + T[0][1] * T[1][0]) * dL_db + 2 * T[1][0] * T[1][1] * dL_dc;
        dcov[2] = 2 * T[0][0] * T[0][2] * dL_da + (T[0][0] * T[1][2] + T[0][2] * T[1][0]) * dL_db + 2 * T[1][0] * T[1][2] * dL_dc;
        dcov[4] = 2 * T[0][2] * T[0][1] * dL_da + (T[0][1] * T[1][2] + T[0][2] * T[1][1]) * dL_db + 2 * T[1][1] * T[1][2] * dL_dc;
    } else {
#pragma unroll
        for (int k = 0; k < 6; ++k) dcov[k] = 0.f;
    }
    float dT[2][3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        dT[0][j] = 2 * tv(e, 0, j) * dL_da + tv(e, 1, j) * dL_db;
        dT[1][j] = 2 * tv(e, 1, j) * dL_dc + tv(e, 0, j) * dL_db;
    }
    // W[i][j] (glm) = v[i + 4j]
    const float dL_dJ00 = v[0] * dT[0][0] + v[4] * dT[0][1] + v[8] * dT[0][2];
    const float dL_dJ02 = v[2] * dT[0][0] + v[6] * dT[0][1] + v[10] * dT[0][2];
    const float dL_dJ11 = v[1] * dT[1][0] + v[5] * dT[1][1] + v[9] * dT[1][2];
    const float dL_dJ12 = v[2] * dT[1][0] + v[6] * dT[1][1] + v[10] * dT[1][2];
    const f3 t = e.t;
    const float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const float dL_dtx = x_grad_mul * -a.fx * tz2 * dL_dJ02;
    const float dL_dty = y_grad_mul * -a.fy * tz2 * dL_dJ12;
    const float dL_dtz = -a.fx * tz2 * dL_dJ00 - a.fy * tz2 * dL_dJ11 + (2 * a.fx * t.x) * tz3 * dL_dJ02 +
                         (2 * a.fy * t.y) * tz3 * dL_dJ12;
    // transformVec4x3Transpose (auxiliary.h:89-97)
    f3 dmean = mk3(v[0] * dL_dtx + v[1] * dL_dty + v[2] * dL_dtz, v[4] * dL_dtx + v[5] * dL_dty + v[6] * dL_dtz,
                   v[8] * dL_dtx + v[9] * dL_dty + v[10] * dL_dtz);

    // ---- preprocessCUDA bwd: projection of the 2D mean (backward.cu:370-387) ----
    {
        const float4 mh = proj_point(pm, m);
        const float m_w = 1.0f / (mh.w + 0.0000001f);
        const float mul1 = (pm[0] * m.x + pm[4] * m.y + pm[8] * m.z + pm[12]) * m_w * m_w;
        const float mul2 = (pm[1] * m.x + pm[5] * m.y + pm[9] * m.z + pm[13]) * m_w * m_w;
        const float gx2 = acc[0], gy2 = acc[1];
        const f3 d2 = mk3((pm[0] * m_w - pm[3] * mul1) * gx2 + (pm[1] * m_w - pm[3] * mul2) * gy2,
                          (pm[4] * m_w - pm[7] * mul1) * gx2 + (pm[5] * m_w - pm[7] * mul2) * gy2,
                          (pm[8] * m_w - pm[11] * mul1) * gx2 + (pm[9] * m_w - pm[11] * mul2) * gy2);
        dmean = dmean + d2;
    }
    // ---- SH -> RGB backward ----
    if (a.sh.dc)
        dmean = dmean + sh_backward(a.D, m, ld3(a.campos), my_sh, ncol, gin.clamped, mk3(acc[6], acc[7], acc[8]),
                                    sh_msk, ddc);
    o.dmean = dmean;
#pragma unroll
    for (int k = 0; k < 6; ++k) o.dcov[k] = dcov[k];
    if (a.activation) {  // opacity = sigmoid(raw): torch's sigmoid backward g * (1 - y) * y
        const float y = act_sigmoid(gin.opacity);
        dop = acc[5] * ((1.0f - y) * y);
    }
    // ---- scale / rotation ----
    if (a.scales) {
        float ds[3], dq[4];
        cov3d_backward(scale, a.scale_modifier, rot, dcov, ds, dq);
        float4 g4 = make_float4(dq[0], dq[1], dq[2], dq[3]);
        if (a.activation) {  // scale = exp(raw): g * y;  rotation = normalize(raw)
            ds[0] *= scale.x;
            ds[1] *= scale.y;
            ds[2] *= scale.z;
            g4 = act_normalize_bwd(rot, rot_len, g4);
        }
        o.dscale[0] = ds[0];
        o.dscale[1] = ds[1];
        o.dscale[2] = ds[2];
        o.drot = g4;
    } else {
        o.dscale[0] = o.dscale[1] = o.dscale[2] = 0.f;
        o.drot = make_float4(0.f, 0.f, 0.f, 0.f);
    }
}

// The grad-mask hooks of the reference's GaussianModel (gaussian_model.py:837-856:
// grad * mask[:, None] on _xyz, _features_dc, _features_rest, _opacity,
// _scaling — not _rotation), applied to the outputs named in mask_bits.
// (the SH part is applied inside sh_backward)
__device__ __forceinline__ void apply_grad_mask(const GaussBwdArgs& a, float m, float (&acc)[9], float& dop,
                                                GaussOut& o) {
    const uint32_t b = a.mask_bits;
    if (b & GS_ACC_MEANS2D) { acc[0] *= m; acc[1] *= m; }
    if (b & GS_ACC_COLORS) { acc[6] *= m; acc[7] *= m; acc[8] *= m; }
    if (b & GS_ACC_OPACITY) dop *= m;
    if (b & GS_ACC_MEANS3D) o.dmean = o.dmean * m;
    if (b & GS_ACC_COV3D)
#pragma unroll
        for (int k = 0; k < 6; ++k) o.dcov[k] *= m;
    if (b & GS_ACC_SCALES)
#pragma unroll
        for (int k = 0; k < 3; ++k) o.dscale[k] *= m;
    if (b & GS_ACC_ROTATIONS) o.drot = make_float4(o.drot.x * m, o.drot.y * m, o.drot.z * m, o.drot.w * m);
}

// Writes (or adds, per GS_ACC_* bit) one live Gaussian's per-Gaussian outputs:
// all loads of the accumulated ones first, then all stores, so the ~20
// scattered read-modify-writes overlap instead of forming a dependent chain.
// (means2D and colors are per rendered Gaussian `idx`; the parameter-shaped outputs go to row `src`)
// f: the GS_ACC_* bits this Gaussian's outputs are added into (a.acc, less gs_grads.zeroed's on its first write)
__device__ __forceinline__ void commit_outputs(const GaussBwdArgs& a, uint32_t f, int idx, int src,
                                               const float (&acc)[9], float dop, const float (&ddc)[3],
                                               const GaussOut& o) {
    const size_t i3 = 3 * (size_t)idx;
    float* const m3 = a.dL_dmeans3D + (size_t)src * a.pm3;
    float* const op1 = a.dL_dopacity + (size_t)src * a.pop;
    float* const sc3 = a.dL_dscales + (size_t)src * a.psc;
    float* d0 = a.dsh.dc ? a.dsh.dc + (size_t)src * a.dsh.dc_stride : nullptr;
    float4* r4 = reinterpret_cast<float4*>(a.dL_drot + (size_t)src * a.prot);
    float om2[2] = {0.f, 0.f}, oop = 0.f, ocol[3] = {0.f, 0.f, 0.f}, om3[3] = {0.f, 0.f, 0.f};
    float ocov[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, osc[3] = {0.f, 0.f, 0.f}, odc[3] = {0.f, 0.f, 0.f};
    float4 orot = make_float4(0.f, 0.f, 0.f, 0.f);
    if (a.dL_dconic)
#pragma unroll
        for (int k = 0; k < 3; ++k) a.dL_dconic[i3 + k] = acc[2 + k];
    if (f & GS_ACC_MEANS2D) { om2[0] = a.dL_dmeans2D[i3]; om2[1] = a.dL_dmeans2D[i3 + 1]; }
    if (f & GS_ACC_OPACITY) oop = *op1;
    if (a.dL_dcolors && (f & GS_ACC_COLORS))
#pragma unroll
        for (int k = 0; k < 3; ++k) ocol[k] = a.dL_dcolors[i3 + k];
    if (f & GS_ACC_MEANS3D)
#pragma unroll
        for (int k = 0; k < 3; ++k) om3[k] = m3[k];
    if (a.dL_dcov3D && (f & GS_ACC_COV3D))
#pragma unroll
        for (int k = 0; k < 6; ++k) ocov[k] = a.dL_dcov3D[6 * (size_t)src + k];
    if (f & GS_ACC_SCALES)
#pragma unroll
        for (int k = 0; k < 3; ++k) osc[k] = sc3[k];
    if (f & GS_ACC_ROTATIONS) orot = *r4;
    if (d0 && (f & GS_ACC_SH))
#pragma unroll
        for (int k = 0; k < 3; ++k) odc[k] = d0[k];

    a.dL_dmeans2D[i3] = om2[0] + acc[0];
    a.dL_dmeans2D[i3 + 1] = om2[1] + acc[1];
    if (!(f & GS_ACC_MEANS2D)) a.dL_dmeans2D[i3 + 2] = 0.f;
    *op1 = oop + dop;
    if (a.dL_dcolors)  // optional (the raw-parameter SH path does not need it)
#pragma unroll
        for (int k = 0; k < 3; ++k) a.dL_dcolors[i3 + k] = ocol[k] + acc[6 + k];
    m3[0] = om3[0] + o.dmean.x;
    m3[1] = om3[1] + o.dmean.y;
    m3[2] = om3[2] + o.dmean.z;
    if (a.dL_dcov3D)
#pragma unroll
        for (int k = 0; k < 6; ++k) a.dL_dcov3D[6 * (size_t)src + k] = ocov[k] + o.dcov[k];
#pragma unroll
    for (int k = 0; k < 3; ++k) sc3[k] = osc[k] + o.dscale[k];
    *r4 = make_float4(orot.x + o.drot.x, orot.y + o.drot.y, orot.z + o.drot.z, orot.w + o.drot.w);
    if (d0) {
#pragma unroll
        for (int k = 0; k < 3; ++k) d0[k] = odc[k] + ddc[k];
        // coefficients beyond the 16 a degree-3 evaluation uses get zero gradient
        if (!(f & GS_ACC_SH)) {
            float* dr = a.dsh.rest + (size_t)src * a.dsh.rest_stride;
            for (int k = kShPitch; k < (a.M - 1) * 3; ++k) dr[k] = 0.f;
        }
    }
}

// ---------------------------------------------------------------------
// Several views in one pass (gs_views_backward): the views of a batch share the
// parameters and their gradient outputs, view v >= 1 adding into them (GS_ACC_*
// set for every parameter-shaped output), so the per-Gaussian work of all views
// runs as ONE pass over the union of their live sets — each live Gaussian's
// parameters and SH row read once, its views' gradients added into the outputs
// in view order by the same thread (the later views' read-modify-writes hit L2),
// bitwise the sums of consecutive per-view passes — instead of one pass per view
// chained across the views' streams.  One view is the n = 1 case.
// ---------------------------------------------------------------------
constexpr int kMaxBwdViews = 4;
static_assert(kMaxBwdViews <= 4, "view masks live in the top 4 bits of a live-list entry");
constexpr uint32_t kLiveIdMask = 0x0FFFFFFFu;  // live-list entry: Gaussian | view mask << 28
struct GaussBwdViews {
    GaussBwdArgs v[kMaxBwdViews];
    int n;
};

// ---------------------------------------------------------------------
// Pass 1 (all P, coalesced): the live set = visible Gaussians with at least
// one gradient record, in some view.  Every other Gaussian has exactly zero
// gradients: its overwritten outputs get zeros here, its accumulated ones are
// left alone (the parameter-shaped outputs of a Gaussian dead in view 0 are
// zeroed per view 0's GS_ACC_* bits; a later view that has it live adds to the
// zero, as its own pass would).  Each 256-Gaussian block compacts its live
// entries in place (no atomics): live_list[256 b + i], i < live_count[b], in
// view 0's geometry buffer.
// ---------------------------------------------------------------------
__global__ __launch_bounds__(kGB) void k_gauss_live(GaussBwdViews m) {
    const GaussBwdArgs& a = m.v[0];
    __shared__ uint32_t s_wave[kGB / 64];
    __shared__ uint8_t s_live[kGB];  // view mask per Gaussian of the block
    const int idx0 = blockIdx.x * kGB;
    const int idx = idx0 + threadIdx.x;
    const int nrow = a.P - idx0 < kGB ? a.P - idx0 : kGB;
    const bool in = idx < a.P;
    // (every view's touched byte and radius loaded together, clamped; `a && b` per view loaded them one by
    // one, each waited for)
    const int ci = in ? idx : 0;
    uint32_t tb[kMaxBwdViews];
    int rv[kMaxBwdViews];
#pragma unroll
    for (int v = 0; v < kMaxBwdViews; ++v) {
        const GaussBwdArgs& b = m.v[v < m.n ? v : 0];
        tb[v] = b.touched[ci];
        rv[v] = b.radii[ci];
    }
    __builtin_amdgcn_sched_barrier(0);
    uint32_t mask = 0;
#pragma unroll
    for (int v = 0; v < kMaxBwdViews; ++v)
        if (v < m.n && in && tb[v] && rv[v] > 0) mask |= 1u << v;
    const bool live = mask != 0;
    s_live[threadIdx.x] = (uint8_t)mask;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const uint64_t bm = __ballot(live);
    if (lane == 0) s_wave[wave] = (uint32_t)__popcll(bm);
    __syncthreads();
    uint32_t off = 0, total = 0;
#pragma unroll
    for (int w = 0; w < kGB / 64; ++w) {
        off += w < wave ? s_wave[w] : 0u;
        total += s_wave[w];
    }
    if (live) a.live_list[idx0 + off + (uint32_t)__popcll(bm & lanemask_lt())] = (uint32_t)idx | mask << 28;
    if (threadIdx.x == 0) a.live_count[blockIdx.x] = total;

    // zeros for the overwritten outputs of the Gaussians dead in view 0 (parameter-shaped ones at row src)
    const uint32_t acc = a.acc;
    const int src = in && a.index ? a.index[idx] : idx;
    if (live && a.dirty) a.dirty[src] = 1;  // (the bucket row this pass may write: its next clear zeroes it)
    if (in && !(mask & 1u)) {
        if (!(acc & GS_ACC_OPACITY)) a.dL_dopacity[(size_t)src * a.pop] = 0.f;
        if (!(acc & GS_ACC_MEANS3D))
#pragma unroll
            for (int k = 0; k < 3; ++k) a.dL_dmeans3D[(size_t)src * a.pm3 + k] = 0.f;
        if (a.dL_dcov3D && !(acc & GS_ACC_COV3D))
#pragma unroll
            for (int k = 0; k < 6; ++k) a.dL_dcov3D[6 * (size_t)src + k] = 0.f;
        if (!(acc & GS_ACC_SCALES))
#pragma unroll
            for (int k = 0; k < 3; ++k) a.dL_dscales[(size_t)src * a.psc + k] = 0.f;
        if (!(acc & GS_ACC_ROTATIONS))
            *reinterpret_cast<float4*>(a.dL_drot + (size_t)src * a.prot) = make_float4(0.f, 0.f, 0.f, 0.f);
        if (a.dsh.dc && !(acc & GS_ACC_SH)) {
            float* d0 = a.dsh.dc + (size_t)src * a.dsh.dc_stride;
            d0[0] = 0.f; d0[1] = 0.f; d0[2] = 0.f;
            if (a.index && a.M > 1) {  // (scattered rows: per thread)
                float* dr = a.dsh.rest + (size_t)src * a.dsh.rest_stride;
                for (int k = 0; k < (a.M - 1) * 3; ++k) dr[k] = 0.f;
            }
        }
    }
    // each view's Gaussian-indexed 3-float outputs of its dead Gaussians, coalesced over the block's
    // region (one 4-B store per lane and element instead of three strided stores per Gaussian: PMC
    // write traffic of this kernel 60 -> ~15 MB at c2)
    __syncthreads();  // s_live
    for (int v = 0; v < m.n; ++v) {
        const GaussBwdArgs& b = m.v[v];
        float* z3[3] = {b.dL_dconic, !(b.acc & GS_ACC_MEANS2D) ? b.dL_dmeans2D : nullptr,
                        !(b.acc & GS_ACC_COLORS) ? b.dL_dcolors : nullptr};
#pragma unroll
        for (int t = 0; t < 3; ++t) {
            float* g = z3[t];
            if (!g) continue;
            g += 3 * (size_t)idx0;
            for (int e = threadIdx.x; e < 3 * nrow; e += kGB)
                if (!((s_live[e / 3] >> v) & 1u)) g[e] = 0.f;
        }
    }
    if (a.dsh.dc && !(acc & GS_ACC_SH) && a.M > 1 && !a.index) {
        // rest rows of the block's Gaussians dead in view 0, coalesced over the block's region
        const int ncol = (a.M - 1) * 3;
        const int stride = a.dsh.rest_stride;
        float* g = a.dsh.rest + (size_t)idx0 * stride;
        const int total_f = (nrow - 1) * stride + ncol;
        for (int e = threadIdx.x; e < total_f; e += kGB) {
            const int row = e / stride, col = e - row * stride;
            if (col < ncol && !(s_live[row] & 1u)) g[e] = 0.f;
        }
    }
}

// ---------------------------------------------------------------------
// Pass 2: the live Gaussians of `group` consecutive pass-1 blocks (group =
// ceil(blocks / 512), at most 8: about 512 workgroups whatever P is, so a small
// or densely visible scene is not funnelled through a few workgroups), one per
// thread, in batches of 256; per batch, each view in turn (a Gaussian's threads
// idle through the views it is dead in).  Their rows are scattered, so the SH
// rows move through LDS with a flat block-wide index (consecutive lanes touch
// consecutive floats of one or two rows) instead of one 180-B row per lane,
// and every read-modify-write batch issues its loads before its stores.
// ---------------------------------------------------------------------
constexpr int kLiveGroup = 8;    // most pass-1 blocks per workgroup
constexpr int kLiveGrid = 768;   // target workgroups (3 per CU: 166 VGPRs, 48 KB of LDS each)
constexpr uint32_t kNoRow = 0xFFFFFFFFu;

// One view's work on one batch of live Gaussians (every thread of the block calls it: it has
// barriers).  ok: this thread's Gaussian is live in the view; src: its parameter row; vfirst: no earlier
// view of the batch has it live (zeroed outputs are stored, not added, on its first write).
__device__ __forceinline__ void bwd_view_batch(const GaussBwdArgs& a, bool ok, int idx, int src, bool vfirst,
                                               uint32_t zeroed, int nrow, int ncol, float inv_ncol, float* s_sh,
                                               uint32_t* s_gid, uint8_t* s_shacc, uint64_t* st) {
    float* const my_sh = s_sh + threadIdx.x * kShPitch;
    const uint32_t facc = a.acc & ~(vfirst ? zeroed : 0u);
    s_gid[threadIdx.x] = ok ? (uint32_t)src : kNoRow;  // (SH rows are parameter rows)
    s_shacc[threadIdx.x] = (facc & GS_ACC_SH) ? 1 : 0;  // (the SH rows' read-modify-write, by row)
    // independent loads first: parameters (a later view's from L2), slot range, the first 8 record flags
    GaussIn gin{};
    if (ok) gin = load_gauss_in(a, idx, src);
    // (the grad-mask byte with the other inputs: read where it is used, it waited for itself alone)
    // (no branch: without a mask the load reads the means' bytes, a valid address, and is ignored)
    const uint32_t gmb_raw = (a.grad_mask ? a.grad_mask : reinterpret_cast<const uint8_t*>(a.means3D))[ok ? src : 0];
    uint32_t n = ok ? a.tiles_touched[idx] : 0u;
    const uint32_t first = ok ? a.first_slot[idx] : 0u;  // (a live Gaussian has slots)
    // (a speculative forward that overflowed its capacity is re-rendered; its slots stop at the capacity)
    n = first < a.slot_cap ? min(n, a.slot_cap - first) : 0u;
    const uint32_t* flags = reinterpret_cast<const uint32_t*>(a.rec_flags);
    uint32_t fl[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) fl[u] = (uint32_t)u < n ? flags[first + u] : 0u;
    __syncthreads();  // s_gid
    if (st) st[1] = __builtin_amdgcn_s_memrealtime();
    const int total = nrow * ncol;
    constexpr int kV = 12;
    if (a.sh.dc && ncol > 0 && !a.sh.half && ncol == kShPitch) {
        // fp32 rows of the full pitch: the LDS image is the flat index itself, so each wave-instruction's
        // 64 floats land contiguously — direct global->LDS loads (no registers, all in flight at once;
        // the barrier below waits for them)
        const uint32_t wave_base = __builtin_amdgcn_readfirstlane(threadIdx.x & ~63u);
        for (int b = 0; b < total; b += kGB) {
            const int e = b + (int)threadIdx.x;
            if (e < total) {
                const int row = (int)(((float)e + 0.5f) * inv_ncol), col = e - row * ncol;
                const float* src = a.sh.rest + (size_t)s_gid[row] * a.sh.rest_stride + col;
                __builtin_amdgcn_global_load_lds((__attribute__((address_space(1))) void*)src,
                                                 (__attribute__((address_space(3))) void*)(s_sh + b + wave_base), 4, 0, 0);
            }
        }
    } else if (a.sh.dc && ncol > 0) {
        // (raw bits first, converted once the batch's loads are all issued: a conversion beside its load made
        // each fp16 load wait in turn)
        const bool half = a.sh.half != 0;
        for (int b = 0; b < total; b += kV * kGB) {
            uint32_t v[kV];
#pragma unroll
            for (int u = 0; u < kV; ++u) {
                const int e = b + u * kGB + (int)threadIdx.x;
                const int row = (int)(((float)e + 0.5f) * inv_ncol), col = e - row * ncol;
                const uint32_t gid = e < total ? s_gid[row] : kNoRow;
                const size_t off = (size_t)gid * a.sh.rest_stride + col;
                v[u] = gid == kNoRow ? 0u
                       : half ? (uint32_t)reinterpret_cast<const uint16_t*>(a.sh.rest)[off]
                              : __float_as_uint(a.sh.rest[off]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int u = 0; u < kV; ++u) {
                const int e = b + u * kGB + (int)threadIdx.x;
                const int row = (int)(((float)e + 0.5f) * inv_ncol), col = e - row * ncol;
                if (e < total)
                    s_sh[row * kShPitch + col] = half ? __half2float(__ushort_as_half((unsigned short)v[u]))
                                                      : __uint_as_float(v[u]);
            }
        }
    }
    // sum of this Gaussian's records: one per (slot, quadrant) the backward
    // replay kept, flagged per slot; slots in emission order = tile order,
    // quadrants in order within a slot.  The flagged records are taken four at
    // a time from a bit mask (bit 4u + quadrant), all twelve loads of a batch
    // issued before its sums: one memory round trip per four records instead
    // of one per record (a batch's unused places re-read its first record and
    // add nothing; acc is never -0, so the skipped +0 changes no bit).
    float acc[9];
#pragma unroll
    for (int f = 0; f < 9; ++f) acc[f] = 0.f;
    for (uint32_t k0 = 0; k0 < n; k0 += 8) {
        if (k0) {
#pragma unroll
            for (int u = 0; u < 8; ++u) fl[u] = k0 + u < n ? flags[first + k0 + u] : 0u;
        }
        uint32_t m = 0;
#pragma unroll
        for (int u = 0; u < 8; ++u)
#pragma unroll
            for (int qd = 0; qd < 4; ++qd) m |= ((fl[u] >> (8 * qd)) & 0xFFu) ? 1u << (4 * u + qd) : 0u;
        const float4* recs = a.records + 3 * (4 * (size_t)(first + k0));
        while (m) {
            int bi[4];
            bool use[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                use[i] = m != 0u;
                bi[i] = use[i] ? __builtin_ctz(m) : bi[0];
                m &= m - 1u;
            }
            float4 r[4][3];
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int c = 0; c < 3; ++c) r[i][c] = recs[3 * bi[i] + c];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                if (use[i]) {
                    acc[0] += r[i][0].x; acc[1] += r[i][0].y; acc[2] += r[i][0].z; acc[3] += r[i][0].w;
                    acc[4] += r[i][1].x; acc[5] += r[i][1].y; acc[6] += r[i][1].z; acc[7] += r[i][1].w;
                    acc[8] += r[i][2].x;
                }
            }
        }
    }
    if (st) st[2] = __builtin_amdgcn_s_memrealtime();
    __syncthreads();  // SH staged
    if (st) st[3] = __builtin_amdgcn_s_memrealtime();

    float ddc[3] = {0.f, 0.f, 0.f};
    float dop = acc[5];  // w.r.t. opacity; chained through the sigmoid when activation = 1
    GaussOut o;
    if (ok) {
        const float gm = !a.grad_mask || gmb_raw ? 1.f : 0.f;
        // (each thread reads and then overwrites only its own LDS row: no barrier in between)
        gauss_bwd_visible(a, gin, acc, dop, my_sh, ncol, (a.mask_bits & GS_ACC_SH) ? gm : 1.f, ddc, o);
        if (a.grad_mask) apply_grad_mask(a, gm, acc, dop, o);
    }
    if (st) st[4] = __builtin_amdgcn_s_memrealtime();
    if (ok) commit_outputs(a, facc, idx, src, acc, dop, ddc, o);
    if (st) st[5] = __builtin_amdgcn_s_memrealtime();
    // dL_dsh rest rows: through LDS (in place), flat block-wide batches, loads before stores
    if (a.dsh.dc && ncol > 0) {
        __syncthreads();
        for (int b = 0; b < total; b += kV * kGB) {
            float old[kV];
#pragma unroll
            for (int u = 0; u < kV; ++u) {
                const int e = b + u * kGB + (int)threadIdx.x;
                const int row = (int)(((float)e + 0.5f) * inv_ncol), col = e - row * ncol;
                const uint32_t gid = e < total ? s_gid[row] : kNoRow;
                old[u] = gid != kNoRow && s_shacc[row] ? a.dsh.rest[(size_t)gid * a.dsh.rest_stride + col] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < kV; ++u) {
                const int e = b + u * kGB + (int)threadIdx.x;
                const int row = (int)(((float)e + 0.5f) * inv_ncol), col = e - row * ncol;
                const uint32_t gid = e < total ? s_gid[row] : kNoRow;
                if (gid != kNoRow) a.dsh.rest[(size_t)gid * a.dsh.rest_stride + col] = old[u] + s_sh[row * kShPitch + col];
            }
        }
    }
    __syncthreads();  // s_gid / s_sh reused by the next view or batch
}

__global__ __launch_bounds__(kGB) void k_gauss_bwd_live(GaussBwdViews m) {
    const GaussBwdArgs& a = m.v[0];
    __shared__ float s_sh[kGB * kShPitch];
    __shared__ uint32_t s_gid[kGB];
    __shared__ uint8_t s_shacc[kGB];
    __shared__ uint32_t s_pre[kLiveGroup + 1];
    __shared__ uint32_t s_vlist[2 * kGB];  // Gaussians live in the view being processed, compacted (+ a chunk's overflow)
    __shared__ uint32_t s_wave[kGB / 64];
    const int nsrc = (a.P + kGB - 1) / kGB;
    const int group = (nsrc + kLiveGrid - 1) / kLiveGrid < kLiveGroup ? (nsrc + kLiveGrid - 1) / kLiveGrid : kLiveGroup;
    const int sb0 = blockIdx.x * group;
    if (threadIdx.x < kLiveGroup)
        s_pre[threadIdx.x + 1] = (int)threadIdx.x < group && sb0 + (int)threadIdx.x < nsrc ? a.live_count[sb0 + threadIdx.x] : 0u;
    __syncthreads();
    if (threadIdx.x == 0) {
        s_pre[0] = 0;
#pragma unroll
        for (int g = 1; g <= kLiveGroup; ++g) s_pre[g] += s_pre[g - 1];
    }
    __syncthreads();
    const uint32_t count = s_pre[kLiveGroup];
    // (diagnostics) per wave, s_memrealtime at: start, the ids/params barrier, records summed, SH staged,
    // chain computed, outputs committed (view 0 of the first batch); then the workgroup's live count and the end
    uint64_t st[8] = {a.diag ? __builtin_amdgcn_s_memrealtime() : 0, 0, 0, 0, 0, 0, 0, 0};
    // rest floats staged per Gaussian: coefficients 1..15 (degree <= 3 never reads more)
    const int ncol = (a.M - 1) * 3 < kShPitch ? (a.M - 1) * 3 : kShPitch;
    const float inv_ncol = ncol > 0 ? 1.0f / (float)ncol : 0.f;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // view-major: for each view in turn, the workgroup's Gaussians live in it, compacted into batches of
    // up to 256 (a Gaussian's views one after another, in view order).  Most live Gaussians are live in
    // one view only, so a batch per (union batch, view) would run mostly idle threads through the pass's
    // latency-bound phases once per view; this runs each view's Gaussians of the whole workgroup together.
    bool first = true;
    // this thread's entry of chunk `base` (the union list with every view's bit: the same for all views)
    const auto load_entry = [&](uint32_t base) {
        const uint32_t j = base + threadIdx.x;
        int g = 0;
#pragma unroll
        for (int q = 1; q < kLiveGroup; ++q) g += j >= s_pre[q] ? 1 : 0;
        return j < count ? a.live_list[(size_t)(sb0 + g) * kGB + (j - s_pre[g])] : 0u;
    };
    // (chunk 0 loaded once for every view: most workgroups have one chunk, and each view's reload of it was a
    // round trip on the pass's latency-bound path)
    const uint32_t entry0 = load_entry(0);
#pragma unroll 1
    for (int v = 0; v < m.n; ++v) {
        uint32_t filled = 0;  // compacted entries pending in s_vlist (< kGB between batches)
        for (uint32_t base = 0; base < count; base += kGB) {
            const bool in = base + threadIdx.x < count;
            const uint32_t entry = base == 0 ? entry0 : load_entry(base);
            const bool has = in && ((entry >> (28 + v)) & 1u);
            const uint64_t bm = __ballot(has);
            if (lane == 0) s_wave[wave] = (uint32_t)__popcll(bm);
            __syncthreads();
            uint32_t off = 0, nv = 0;
#pragma unroll
            for (int w = 0; w < kGB / 64; ++w) {
                off += w < wave ? s_wave[w] : 0u;
                nv += s_wave[w];
            }
            if (has) s_vlist[filled + off + (uint32_t)__popcll(bm & lanemask_lt())] = entry;  // (with the view mask)
            filled += nv;
            __syncthreads();  // s_vlist (and s_wave, read by every thread, before its next write)
            if (filled < (uint32_t)kGB && base + kGB < count) continue;  // (fill the batch further)
            while (filled > 0) {
                const uint32_t nb = filled < (uint32_t)kGB ? filled : (uint32_t)kGB;
                const bool ok = threadIdx.x < nb;
                const uint32_t ent = ok ? s_vlist[threadIdx.x] : 0u;
                const int idx = (int)(ent & kLiveIdMask);
                const int src = ok && a.index ? a.index[idx] : idx;  // parameter row
                const bool vfirst = ((ent >> 28) & ((1u << v) - 1u)) == 0u;  // no earlier view has it live
                bwd_view_batch(m.v[v], ok, idx, src, vfirst, a.zeroed, (int)nb, ncol, inv_ncol, s_sh, s_gid, s_shacc,
                               a.diag && first ? st : nullptr);
                first = false;
                // (bwd_view_batch ends on a barrier: every thread has read its entry) the rest to the front
                const uint32_t rest = filled - nb;
                if (threadIdx.x < rest) s_vlist[threadIdx.x] = s_vlist[kGB + threadIdx.x];
                __syncthreads();
                filled = rest;
                if (base + kGB < count) break;  // (a partial batch waits for the next chunk)
            }
        }
    }
    if (a.diag && (threadIdx.x & 63) == 0) {
        st[7] = __builtin_amdgcn_s_memrealtime();
        st[6] = count;  // live Gaussians of the workgroup
        uint64_t* d = a.diag + kDiagWords * ((size_t)blockIdx.x * 4 + (threadIdx.x >> 6));
#pragma unroll
        for (int i = 0; i < 8; ++i) d[i] = st[i];
    }
}

static GaussBwdViews gauss_views(const GaussBwdArgs* views, int n) {
    GaussBwdViews m;
    m.n = n < kMaxBwdViews ? n : kMaxBwdViews;
    for (int v = 0; v < m.n; ++v) m.v[v] = views[v];
    return m;
}

// Pass 1 alone: it reads only what the forwards left (touched bytes, radii), so it may run before the
// views' gradient replays end (gs_views_backward: behind view 0's replay, beside the others')
// writes_after: the pass marks the gradient bucket's dirty rows (GaussBwdArgs::dirty) — after the bucket's clear,
// which zeroes the marked rows and resets the marks (a mark made before it would be lost, and the row never cleared)
void launch_gauss_live_views(const GaussBwdArgs* views, int n, hipStream_t s, hipEvent_t writes_after) {
    if (views[0].P <= 0 || n <= 0) return;
    if (writes_after && views[0].dirty) (void)hipStreamWaitEvent(s, writes_after, 0);
    hipLaunchKernelGGL(k_gauss_live, dim3(div_up(views[0].P, kGB)), dim3(kGB), 0, s, gauss_views(views, n));
}

// Pass 2 (after launch_gauss_live_views on an ordered stream, and after every view's replay)
void launch_gauss_bwd_live_views(const GaussBwdArgs* views, int n, hipStream_t s, hipEvent_t writes_after) {
    if (views[0].P <= 0 || n <= 0) return;
    // k_gauss_live writes only overwritten (per-call) outputs; the accumulated ones start here
    if (writes_after) (void)hipStreamWaitEvent(s, writes_after, 0);
    const int blocks = div_up(views[0].P, kGB);
    const int group = std::min(div_up(blocks, kLiveGrid), kLiveGroup);  // (the kernel derives the same)
    hipLaunchKernelGGL(k_gauss_bwd_live, dim3(div_up(blocks, group)), dim3(kGB), 0, s, gauss_views(views, n));
}

void launch_gauss_backward_views(const GaussBwdArgs* views, int n, hipStream_t s, hipEvent_t writes_after) {
    launch_gauss_live_views(views, n, s, writes_after);
    launch_gauss_bwd_live_views(views, n, s, views[0].dirty ? nullptr : writes_after);  // (same stream: waited)
}

void launch_gauss_backward(const GaussBwdArgs& a, hipStream_t s, hipEvent_t writes_after) {
    launch_gauss_backward_views(&a, 1, s, writes_after);
}

int gauss_backward_max_views() { return kMaxBwdViews; }

}  // namespace gs
