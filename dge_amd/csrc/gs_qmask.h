// gs_qmask.h — the per-instance quadrant mask: which 8x8 quadrants of a 16x16 tile a Gaussian can
// reach with alpha >= 1/255 (forward.cu:336-348's skip tests), computed ONCE per (Gaussian, tile) by
// the preprocess (a 64-bit word per Gaussian: each pixel-row band's range of quadrant columns, rects of up
// to 8 x 4 tiles; the emission bounds larger ones per instance)
// instead of by each of the four quadrant waves of the blend for every list position it walks (the
// blend's cull_keep: ~136 VALU per lane and position, 14-21% of the heaviest waves' cycles, plus the
// gathers of entries it then drops); the emission copies each instance's 4 bits into its list id.
//
// Host + device: the CPU suite checks the bound against the blend's own per-pixel test
// (tests/qmask_check.cpp, brute force over the 64 pixels of every quadrant).
//
// The test a pixel p passes is q(d) = a dx^2 + 2 b dx dy + c dy^2 <= thr, d = g - p (Gaussian centre
// minus pixel), thr = 2 ln(255 o) (o G >= 1/255 with G = exp(-q/2)).  The level set is an ellipse;
// a quadrant box [X0, X1] x [Y0, Y1] (in d) meets it iff the ellipse's x-extent inside the band
// Y0 <= dy <= Y1 meets [X0, X1].  For D = ac - b^2 > 0 that extent is exact in closed form:
//   at a fixed dy the ellipse spans dx = (-b dy -+ sqrt(a T - D dy^2)) / a, |dy| <= dyE = sqrt(a T / D);
//   its right end is concave in dy, maximal (dx = dxE = sqrt(c T / D)) at dy = yr = -b dxE / c, its
//   left end convex, minimal (-dxE) at -yr — so over a band the extreme is dxE when yr lies in it,
//   else the larger band-edge value (the smaller, on the left).
// Conservative on purpose: T = thr + (1 + thr) (4e-3 + 1e-5 ac / D) — the blend's exp is within an
// ulp of exp, and its float power -0.5 (a dx^2 + c dy^2) - b dx dy is off by a few ulp of
// a dx^2 + c dy^2 <= q / (1 - |b| / sqrt(ac)) ~ 2 q ac / D (cancellation in elongated ellipses) —
// and the band and the extent widened by 1e-3 of the ellipse's half-axes + 1e-3 px (the closed
// form's rounding is below 0.35e-3 of them with D from an exact split of b^2; 1e-3 px also covers
// the blend's rounding of dx = x - px at 2k-pixel coordinates); a non-positive-definite, NaN or
// degenerate (ac / D >= 1e6) conic keeps every quadrant; opacity < 1/255 keeps none (alpha <= o).
// A kept quadrant only costs the blend a test; a dropped one must never pass — the mask is a
// superset of the quadrants any pixel blends, so every output (n_contrib included: it counts list
// positions, not kept entries) is the same as with no cull at all.
#pragma once

#include <math.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define GS_QM_HD __host__ __device__
#else
#define GS_QM_HD
#endif

namespace gs {

// On the device the hardware's approximate square root, reciprocal and log2 (~1 ulp: far inside the
// 1e-3 margins below); the host check uses the libm forms
GS_QM_HD inline float qm_sqrt(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_sqrtf(x);
#else
    return sqrtf(x);
#endif
}
GS_QM_HD inline float qm_rcp(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(x);
#else
    return 1.0f / x;
#endif
}
GS_QM_HD inline float qm_ln(float x) {
#if defined(__HIP_DEVICE_COMPILE__)
    return 0.693147182f * __builtin_amdgcn_logf(x);
#else
    return logf(x);
#endif
}

// Gaussian ids in the per-tile lists carry the mask in their top bits (bit 28 + quadrant) when the
// scene has fewer than 2^28 Gaussians; id_mask() strips it
constexpr int kIdBits = 28;
constexpr uint32_t kIdMask = (1u << kIdBits) - 1u;

// The per-Gaussian part (a thread per Gaussian in the emission's round set-up)
struct QuadCull {
    float gx, gy;    // centre (pixels)
    float dxE, dyE;  // the ellipse's half-extents, widened; dyE < 0: reaches no pixel
    float yr;        // dy of the right end (the left end's is -yr)
    float bs, s;     // b / a, 1 / a
    float aT, D;     // a T, ac - b^2
    int all;         // 1: no bound (every quadrant kept)
};

GS_QM_HD inline QuadCull quad_cull_setup(float gx, float gy, float a, float b, float c, float o) {
    QuadCull q;
    q.gx = gx;
    q.gy = gy;
    q.all = 0;
    q.dxE = q.dyE = -1.0f;
    q.yr = q.bs = q.s = q.aT = q.D = 0.0f;
    if (o < 1.0f / 255.0f) return q;  // alpha <= o G <= o < 1/255 (power > 0 is skipped; NaN: below)
    // D = ac - b^2 with b^2 split exactly (fma): ~1 ulp of D however elongated the ellipse
    const float bb = b * b, bb_err = fmaf(b, b, -bb);
    const float D = fmaf(a, c, -bb) - bb_err;
    const float rD = qm_rcp(D);
    const float k = (a * c) * rD;  // conditioning (>= 1): the blend's own rounding of power grows with it
    const float thr = 2.0f * qm_ln(255.0f * o);
    const float T = thr + (1.0f + fabsf(thr)) * (4e-3f + 1e-5f * k);
    if (!(a > 0.0f && c > 0.0f && D > 0.0f && k < 1e6f && T >= 0.0f && T < 1e30f && fabsf(gx) < 1e7f &&
          fabsf(gy) < 1e7f)) {
        q.all = 1;  // not positive definite, degenerate, NaN or huge: no bound
        return q;
    }
    const float dxE = qm_sqrt(c * T * rD), dyE = qm_sqrt(a * T * rD);
    q.s = qm_rcp(a);
    q.bs = b * q.s;
    q.aT = a * T;
    q.D = D;
    q.yr = -b * dxE * qm_rcp(c);
    q.dxE = dxE + (1e-3f * dxE + 1e-3f);
    q.dyE = dyE + (1e-3f * dyE + 1e-3f);
    return q;
}

// Bits q = (qy << 1) | qx of the tile whose first pixel is (tx0, ty0) (k_render_fwd's quadrant
// numbering: box x0 = tx0 + 8 (q & 1), y0 = ty0 + 8 (q >> 1)) that the Gaussian may reach.
GS_QM_HD inline uint32_t quad_mask(const QuadCull& q, float tx0, float ty0) {
    if (q.all) return 0xFu;
    uint32_t m = 0u;
    const float mx = 1e-3f * q.dxE + 1e-3f, my = 1e-3f * q.dyE + 1e-3f;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
        // the band's pixel rows ty0 + 8j .. ty0 + 8j + 7, in d = gy - py, widened
        const float Y0 = (q.gy - (ty0 + (float)(8 * j + 7))) - my;
        const float Y1 = (q.gy - (ty0 + (float)(8 * j))) + my;
        const float lo = fmaxf(Y0, -q.dyE), hi = fminf(Y1, q.dyE);
        if (!(lo <= hi)) continue;  // the band misses the ellipse
        const float sl = qm_sqrt(fmaxf(0.0f, q.aT - q.D * lo * lo));
        const float sh = qm_sqrt(fmaxf(0.0f, q.aT - q.D * hi * hi));
        const float cl = -q.bs * lo, ch = -q.bs * hi;
        float xmax = fmaxf(cl + q.s * sl, ch + q.s * sh);
        float xmin = fminf(cl - q.s * sl, ch - q.s * sh);
        if (lo <= q.yr && q.yr <= hi) xmax = q.dxE;
        if (lo <= -q.yr && -q.yr <= hi) xmin = -q.dxE;
        xmax += mx;
        xmin -= mx;
#pragma unroll
        for (int i = 0; i < 2; ++i) {
            const float X0 = q.gx - (tx0 + (float)(8 * i + 7)), X1 = q.gx - (tx0 + (float)(8 * i));
            if (X0 <= xmax && X1 >= xmin) m |= 1u << (2 * j + i);
        }
    }
    return m;
}

// The bound of a Gaussian's whole tile rect [x0, x0 + w) x [y0, y0 + h) (w <= kBandMaxW, h <= kBandMaxH) in
// one 64-bit word: for each of its 2h pixel-row bands (band b: rows 16 y0 + 8 b .. + 7) the range of
// quadrant columns c (pixels 16 x0 + 8 c .. + 7, c < 2w) the ellipse reaches — contiguous, the ellipse
// being convex — as byte b = cmin << 4 | cmax (0xF0: none).  Each band is bounded once, not once per
// tile; band_inst_mask() gives the instance's 4 bits, equal to quad_mask's tile by tile.  Larger rects
// (huge footprints): the emission bounds each instance with quad_mask.
constexpr int kBandMaxW = 8, kBandMaxH = 4;
constexpr uint64_t kBandsAll = 0x0F0F0F0F0F0F0F0Full, kBandsNone = 0xF0F0F0F0F0F0F0F0ull;
GS_QM_HD inline bool band_rect_fits(int w, int h) { return w <= kBandMaxW && h <= kBandMaxH; }
GS_QM_HD inline uint64_t rect_band_ranges(const QuadCull& q, int x0, int y0, int w, int h) {
    if (q.all) return kBandsAll;
    uint64_t word = kBandsNone;
    const float mx = 1e-3f * q.dxE + 1e-3f, my = 1e-3f * q.dyE + 1e-3f;
    for (int j = 0; j < 2 * h; ++j) {
        const float py0 = (float)(16 * y0 + 8 * j);
        const float Y0 = (q.gy - (py0 + 7.0f)) - my, Y1 = (q.gy - py0) + my;
        const float lo = fmaxf(Y0, -q.dyE), hi = fminf(Y1, q.dyE);
        if (!(lo <= hi)) continue;
        const float sl = qm_sqrt(fmaxf(0.0f, q.aT - q.D * lo * lo));
        const float sh = qm_sqrt(fmaxf(0.0f, q.aT - q.D * hi * hi));
        const float cl = -q.bs * lo, ch = -q.bs * hi;
        float xmax = fmaxf(cl + q.s * sl, ch + q.s * sh);
        float xmin = fminf(cl - q.s * sl, ch - q.s * sh);
        if (lo <= q.yr && q.yr <= hi) xmax = q.dxE;
        if (lo <= -q.yr && -q.yr <= hi) xmin = -q.dxE;
        xmax += mx;
        xmin -= mx;
        int cmin = 15, cmax = -1;
        for (int c = 0; c < 2 * w; ++c) {
            const float px0 = (float)(16 * x0 + 8 * c);
            const float X0 = q.gx - (px0 + 7.0f), X1 = q.gx - px0;
            if (X0 <= xmax && X1 >= xmin) {
                cmin = c < cmin ? c : cmin;
                cmax = c;
            }
        }
        if (cmax >= 0) {
            word &= ~(0xFFull << (8 * j));
            word |= (uint64_t)(cmin << 4 | cmax) << (8 * j);
        }
    }
    return word;
}
// tile (x0 + i, y0 + j) of such a rect: its quadrant bits q = (qy << 1) | qx
GS_QM_HD inline uint32_t band_inst_mask(uint64_t word, int i, int j) {
    uint32_t m = 0u;
#pragma unroll
    for (int qy = 0; qy < 2; ++qy) {
        const uint32_t band = (uint32_t)(word >> (8 * (2 * j + qy))) & 0xFFu;
        const int cmin = (int)(band >> 4), cmax = (int)(band & 15u);
#pragma unroll
        for (int qx = 0; qx < 2; ++qx) {
            const int c = 2 * i + qx;
            if (cmin <= c && c <= cmax) m |= 1u << (2 * qy + qx);
        }
    }
    return m;
}

}  // namespace gs
