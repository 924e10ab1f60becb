/*
 * gs_truth.c — the backward evaluated in double: the "truth" a per-element gradient bar is measured against.
 *
 * TEST INFRASTRUCTURE ONLY (see gs_oracle.h).  Paths are relative to
 *   /root/reference/gaussiansplatting/submodules/diff-gaussian-rasterization/cuda_rasterizer/
 *
 * What "truth" means here: the reference's backward formulas (backward.cu:20-557, auxiliary.h:107-117)
 * evaluated in double at the float forward's state.  Every decision is the float forward's — which entries a
 * pixel blends (the forward's float dx, dy, power, G = the blend exp, alpha, n_contrib), radii > 0, the
 * clamped SH colours, the x/y Jacobian clamps — and every per-entry input the blend used (G, alpha, the
 * Gaussian's conic, opacity and colour) is taken as the float value it had; everything after that is double:
 * the transmittance T in front of an entry as the forward product of (1 - alpha) (not the back-division of
 * the rounded final T), the colour behind it, the per-pixel terms, their sums over pixels and the whole
 * per-Gaussian chain with its forward quantities (the camera-space mean, the EWA Jacobian, cov3D from scale
 * and rotation, the SH direction) recomputed in double from the float inputs.  The reference's float
 * constants (0.3f, 1.3f, 0.0000001f, the SH constants) keep their float values.
 *
 * Beside it, go_backward_truth gives the rasterizer sums as the reference's own float arithmetic forms them:
 * the oracle's float per-pixel terms (render_pixel_bwd, backward.cu:482-545) added one by one in float, the
 * way its float atomicAdds accumulate them (backward.cu:523-548), in several admissible arrival orders.  The
 * spread of those orders around the truth is the reference's own rounding; tests/helpers.py truth_bar holds
 * the GPU's gradients to a small multiple of it.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "gs_oracle.h"
#include "gs_oracle_internal.h"

/* auxiliary.h:22-39, the float values promoted */
static const double kD0 = 0.28209479177387814f;
static const double kD1 = 0.4886025119029199f;
static const double kD2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f, -1.0925484305920792f,
                              0.5462742152960396f};
static const double kD3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f, 0.3731763325901154f,
                              -0.4570457994644658f, 1.445305721320277f, -0.5900435899266435f};

/* ------------------------------------------------------------------ */
/* rasterizer sums in double, and in float in several arrival orders   */
/* ------------------------------------------------------------------ */
typedef struct {
    uint32_t k, id;   /* list position, Gaussian */
    double alpha, G, dx, dy, T;  /* the forward's float values; T the double transmittance in front */
} blended;

/* backward.cu:399-557 for one pixel in double (see the file comment); per-instance sums into rec [K,9] */
static void pixel_bwd_f64(const go_state *st, const float *colors, const float *bg, const float *dL_dpix, int tile,
                          int px, int py, blended *buf, double *rec) {
    const uint32_t r0 = st->ranges[2 * tile];
    const size_t pix = (size_t)st->W * py + px, HW = (size_t)st->W * st->H;
    const uint32_t last = st->n_contrib[pix];
    const float pfx = (float)px, pfy = (float)py;
    /* front to back over the positions the forward reached: its blended entries and T in front of each
     * (forward.cu:330-366: an entry up to n_contrib that passes the alpha test was blended) */
    int n = 0;
    double T = 1.0;
    for (uint32_t c = 0; c < last; ++c) {
        const uint32_t k = r0 + c, id = st->point_list[k];
        const float dx = st->means2D[2 * (size_t)id] - pfx, dy = st->means2D[2 * (size_t)id + 1] - pfy;
        float G, alpha;
        if (!go_pixel_alpha(st->conic_opacity + 4 * (size_t)id, dx, dy, &G, &alpha)) continue;
        blended *b = buf + n++;
        b->k = k; b->id = id; b->alpha = alpha; b->G = G; b->dx = dx; b->dy = dy; b->T = T;
        T *= 1.0 - (double)alpha;
    }
    const double T_final = T;
    double dp[3], bg_dot = 0;
    for (int ch = 0; ch < 3; ++ch) {
        dp[ch] = dL_dpix[ch * HW + pix];
        bg_dot += (double)bg[ch] * dp[ch];
    }
    const double ddelx_dx = 0.5 * st->W, ddely_dy = 0.5 * st->H;
    double accum[3] = {0, 0, 0}, last_color[3] = {0, 0, 0}, last_alpha = 0;
    for (int e = n - 1; e >= 0; --e) {  /* back to front (backward.cu:468-555) */
        const blended *b = buf + e;
        const float *co = st->conic_opacity + 4 * (size_t)b->id;
        double *r = rec + 9 * (size_t)b->k;
        const double dchannel_dcolor = b->alpha * b->T;
        double dL_dalpha = 0;
        for (int ch = 0; ch < 3; ++ch) {
            const double c = colors[3 * (size_t)b->id + ch];
            accum[ch] = last_alpha * last_color[ch] + (1.0 - last_alpha) * accum[ch];
            last_color[ch] = c;
            dL_dalpha += (c - accum[ch]) * dp[ch];
            r[6 + ch] += dchannel_dcolor * dp[ch];
        }
        dL_dalpha *= b->T;
        last_alpha = b->alpha;
        dL_dalpha += (-T_final / (1.0 - b->alpha)) * bg_dot;
        const double dL_dG = (double)co[3] * dL_dalpha;
        const double gdx = b->G * b->dx, gdy = b->G * b->dy;
        const double dG_ddelx = -gdx * co[0] - gdy * co[1];
        const double dG_ddely = -gdy * co[2] - gdx * co[1];
        r[0] += dL_dG * dG_ddelx * ddelx_dx;
        r[1] += dL_dG * dG_ddely * ddely_dy;
        r[2] += -0.5 * gdx * b->dx * dL_dG;
        r[3] += -0.5 * gdx * b->dy * dL_dG;
        r[4] += -0.5 * gdy * b->dy * dL_dG;
        r[5] += b->G * dL_dalpha;
    }
}

/* position of the i-th term of a Gaussian's n terms in arrival order o (0: tiles ascending, each tile's
 * pixels row-major, each pixel's entries back to front; 1: the reverse; 2: the even-numbered terms, then
 * the odd ones; 3: a pseudo-random permutation, seeded per Gaussian — see go_backward_truth) */
static size_t order_at(int o, size_t i, size_t n, const uint32_t *perm) {
    switch (o) {
    case 0: return i;
    case 1: return n - 1 - i;
    case 2: { const size_t h = (n + 1) / 2; return i < h ? 2 * i : 2 * (i - h) + 1; }
    default: return perm[i];
    }
}

int go_backward_truth(go_state *st, const go_settings *s, const go_inputs *in, const float *dL_dpix, int n_orders,
                      float *sums_f, double *sums_d) {
    const int P = in->P;
    if (n_orders < 0 || n_orders > 4) return GO_ERR_INVALID;
    if (n_orders) memset(sums_f, 0, (size_t)n_orders * P * 9 * sizeof(float));
    if (sums_d) memset(sums_d, 0, (size_t)P * 9 * sizeof(double));
    if (P == 0 || st->K == 0) return GO_OK;
    const size_t K = (size_t)st->K;
    const float *colors = in->colors_precomp ? in->colors_precomp : st->rgb;
    const int ntiles = st->gx * st->gy, W = st->W, H = st->H;
    double *rec = sums_d ? (double *)calloc(K * 9, sizeof(double)) : NULL;
    go_emit *em = (go_emit *)calloc((size_t)ntiles, sizeof(go_emit));
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < ntiles; ++t) {
        const uint32_t len = st->ranges[2 * t + 1] - st->ranges[2 * t];
        blended *buf = (blended *)malloc((len ? len : 1) * sizeof(blended));
        const int tx = t % st->gx, ty = t / st->gx;
        for (int yy = 0; yy < TILE_Y; ++yy)
            for (int xx = 0; xx < TILE_X; ++xx) {
                const int px = tx * TILE_X + xx, py = ty * TILE_Y + yy;
                if (px >= W || py >= H) continue;
                if (n_orders) go_render_pixel_terms(st, colors, s->bg, dL_dpix, t, px, py, em + t);
                if (rec) pixel_bwd_f64(st, colors, s->bg, dL_dpix, t, px, py, buf, rec);
            }
        free(buf);
    }
    for (size_t k = 0; rec && k < K; ++k) {  /* per Gaussian, its instances in list order (double: order immaterial) */
        double *a = sums_d + 9 * (size_t)st->point_list[k];
        for (int j = 0; j < 9; ++j) a[j] += rec[9 * k + j];
    }
    free(rec);
    if (!n_orders) {
        free(em);
        return GO_OK;
    }
    /* the float terms grouped by Gaussian in arrival order 0 */
    size_t *off = (size_t *)calloc((size_t)P + 1, sizeof(size_t));
    for (int t = 0; t < ntiles; ++t)
        for (size_t i = 0; i < em[t].n; ++i) off[em[t].ids[i] + 1]++;
    size_t nmax = 0;
    for (int g = 0; g < P; ++g) {
        if (off[g + 1] > nmax) nmax = off[g + 1];
        off[g + 1] += off[g];
    }
    float *terms = (float *)malloc((off[P] ? off[P] : 1) * 9 * sizeof(float));
    size_t *fill = (size_t *)malloc(((size_t)P ? (size_t)P : 1) * sizeof(size_t));
    memcpy(fill, off, (size_t)P * sizeof(size_t));
    for (int t = 0; t < ntiles; ++t) {
        for (size_t i = 0; i < em[t].n; ++i)
            memcpy(terms + 9 * fill[em[t].ids[i]]++, em[t].terms + 9 * i, 9 * sizeof(float));
        free(em[t].ids);
        free(em[t].terms);
    }
    free(em);
    free(fill);
#pragma omp parallel
    {
        uint32_t *perm = (uint32_t *)malloc((nmax ? nmax : 1) * sizeof(uint32_t));
#pragma omp for schedule(dynamic, 256)
        for (int g = 0; g < P; ++g) {
            const size_t n = off[g + 1] - off[g];
            if (!n) continue;
            const float *tg = terms + 9 * off[g];
            if (n_orders > 3) {  /* Fisher-Yates, 64-bit LCG seeded by the Gaussian */
                uint64_t x = 0x9E3779B97F4A7C15ull * ((uint64_t)g + 1);
                for (size_t i = 0; i < n; ++i) perm[i] = (uint32_t)i;
                for (size_t i = n - 1; i > 0; --i) {
                    x = x * 6364136223846793005ull + 1442695040888963407ull;
                    const size_t j = (size_t)((x >> 33) % (i + 1));
                    const uint32_t v = perm[i]; perm[i] = perm[j]; perm[j] = v;
                }
            }
            for (int o = 0; o < n_orders; ++o) {
                float acc[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
                for (size_t i = 0; i < n; ++i) {
                    const float *tm = tg + 9 * order_at(o, i, n, perm);
                    for (int j = 0; j < 9; ++j) acc[j] = acc[j] + tm[j];
                }
                memcpy(sums_f + ((size_t)o * P + g) * 9, acc, 9 * sizeof(float));
            }
        }
        free(perm);
    }
    free(terms);
    free(off);
    return GO_OK;
}

/* ------------------------------------------------------------------ */
/* the per-Gaussian chain in double (backward.cu:20-396)               */
/* ------------------------------------------------------------------ */
typedef struct { double x, y, z; } d3;
typedef struct { double c[3][3]; } dm3; /* c[col][row], like glm::mat3 */

static d3 d3make(double x, double y, double z) { d3 r = {x, y, z}; return r; }
static d3 d3add(d3 a, d3 b) { return d3make(a.x + b.x, a.y + b.y, a.z + b.z); }
static d3 d3scale(d3 a, double s) { return d3make(a.x * s, a.y * s, a.z * s); }
static double d3dot(d3 a, d3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static d3 d3ld(const float *p) { return d3make(p[0], p[1], p[2]); }
static dm3 dm3mul(const dm3 *A, const dm3 *B) {
    dm3 R;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r)
            R.c[c][r] = A->c[0][r] * B->c[c][0] + A->c[1][r] * B->c[c][1] + A->c[2][r] * B->c[c][2];
    return R;
}
static dm3 dm3T(const dm3 *A) {
    dm3 R;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) R.c[c][r] = A->c[r][c];
    return R;
}
static dm3 dm3cols(double a, double b, double c, double d, double e, double f, double g, double h, double i) {
    dm3 R;
    R.c[0][0] = a; R.c[0][1] = b; R.c[0][2] = c;
    R.c[1][0] = d; R.c[1][1] = e; R.c[1][2] = f;
    R.c[2][0] = g; R.c[2][1] = h; R.c[2][2] = i;
    return R;
}
static dm3 rot_matrix(double r, double x, double y, double z) { /* forward.cu:131-135, not normalised */
    return dm3cols(1.0 - 2.0 * (y * y + z * z), 2.0 * (x * y - r * z), 2.0 * (x * z + r * y),
                   2.0 * (x * y + r * z), 1.0 - 2.0 * (x * x + z * z), 2.0 * (y * z - r * x),
                   2.0 * (x * z - r * y), 2.0 * (y * z + r * x), 1.0 - 2.0 * (x * x + y * y));
}

/* forward.cu:118-152 in double */
static void cov3d_f64(const float *scale, float mod, const float *rot, double out[6]) {
    dm3 S = dm3cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    for (int k = 0; k < 3; ++k) S.c[k][k] = (double)mod * scale[k];
    dm3 R = rot_matrix(rot[0], rot[1], rot[2], rot[3]);
    dm3 M = dm3mul(&S, &R), Mt = dm3T(&M);
    dm3 Sig = dm3mul(&Mt, &M);
    out[0] = Sig.c[0][0]; out[1] = Sig.c[0][1]; out[2] = Sig.c[0][2];
    out[3] = Sig.c[1][1]; out[4] = Sig.c[1][2]; out[5] = Sig.c[2][2];
}

GO_EXACT static void clamp_decisions(const float *m, float tanfovx, float tanfovy, const float *view, int *xclamp,
                                     int *yclamp, float *limx, float *limy, float *txtz, float *tytz) {
    GO_EXACT_BODY
    const float tfx = view[0] * m[0] + view[4] * m[1] + view[8] * m[2] + view[12];
    const float tfy = view[1] * m[0] + view[5] * m[1] + view[9] * m[2] + view[13];
    const float tfz = view[2] * m[0] + view[6] * m[1] + view[10] * m[2] + view[14];
    *limx = 1.3f * tanfovx;
    *limy = 1.3f * tanfovy;
    *txtz = tfx / tfz;
    *tytz = tfy / tfz;
    *xclamp = *txtz < -*limx || *txtz > *limx;
    *yclamp = *tytz < -*limy || *tytz > *limy;
}

/* backward.cu:144-274 in double; the x/y clamps (forward.cu:87-90, backward.cu:163-170) as the float
 * forward decided them.  Writes dL_dcov (6), returns the cov-path mean gradient. */
static d3 cov2d_bwd_f64(const float *meanf, float fx, float fy, float tanfovx, float tanfovy, const double cov3D[6],
                        const float *view, const double dL_dconic[3], double dL_dcov[6]) {
    /* the float forward's decisions (gs_oracle.c ewa_setup, same operations) */
    int xclamp, yclamp;
    float limxf, limyf, txtzf, tytzf;
    clamp_decisions(meanf, tanfovx, tanfovy, view, &xclamp, &yclamp, &limxf, &limyf, &txtzf, &tytzf);
    const float mx = meanf[0], my = meanf[1], mz = meanf[2];
    /* camera-space mean in double, clamped where the forward clamped */
    const double vx = (double)view[0] * mx + (double)view[4] * my + (double)view[8] * mz + view[12];
    const double vy = (double)view[1] * mx + (double)view[5] * my + (double)view[9] * mz + view[13];
    const double vz = (double)view[2] * mx + (double)view[6] * my + (double)view[10] * mz + view[14];
    d3 t = d3make(vx, vy, vz);
    if (xclamp) t.x = (txtzf > limxf ? (double)limxf : -(double)limxf) * t.z;
    if (yclamp) t.y = (tytzf > limyf ? (double)limyf : -(double)limyf) * t.z;
    const double x_grad_mul = xclamp ? 0 : 1, y_grad_mul = yclamp ? 0 : 1;
    const double dfx = fx, dfy = fy;
    dm3 J = dm3cols(dfx / t.z, 0.0, -(dfx * t.x) / (t.z * t.z), 0.0, dfy / t.z, -(dfy * t.y) / (t.z * t.z), 0, 0, 0);
    dm3 Wm = dm3cols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    dm3 T = dm3mul(&Wm, &J);
    dm3 V = dm3cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
    dm3 Tt = dm3T(&T), Vt = dm3T(&V);
    dm3 TtV = dm3mul(&Tt, &Vt);
    dm3 cov2D = dm3mul(&TtV, &T);
    const double a = cov2D.c[0][0] + (double)0.3f, b = cov2D.c[0][1], c = cov2D.c[1][1] + (double)0.3f;
    const double denom = a * c - b * b;
    const double denom2inv = 1.0 / ((denom * denom) + (double)0.0000001f);
    double dL_da = 0, dL_db = 0, dL_dc = 0;
#define Tm(i, j) (T.c[i][j])
#define Vm(i, j) (V.c[i][j])
    if (denom2inv != 0) {
        dL_da = denom2inv * (-c * c * dL_dconic[0] + 2 * b * c * dL_dconic[1] + (denom - a * c) * dL_dconic[2]);
        dL_dc = denom2inv * (-a * a * dL_dconic[2] + 2 * a * b * dL_dconic[1] + (denom - a * c) * dL_dconic[0]);
        dL_db = denom2inv * 2 * (b * c * dL_dconic[0] - (denom + 2 * b * b) * dL_dconic[1] + a * b * dL_dconic[2]);
        dL_dcov[0] = Tm(0, 0) * Tm(0, 0) * dL_da + Tm(0, 0) * Tm(1, 0) * dL_db + Tm(1, 0) * Tm(1, 0) * dL_dc;
        dL_dcov[3] = Tm(0, 1) * Tm(0, 1) * dL_da + Tm(0, 1) * Tm(1, 1) * dL_db + Tm(1, 1) * Tm(1, 1) * dL_dc;
        dL_dcov[5] = Tm(0, 2) * Tm(0, 2) * dL_da + Tm(0, 2) * Tm(1, 2) * dL_db + Tm(1, 2) * Tm(1, 2) * dL_dc;
        dL_dcov[1] = 2 * Tm(0, 0) * Tm(0, 1) * dL_da + (Tm(0, 0) * Tm(1, 1) + Tm(0, 1) * Tm(1, 0)) * dL_db +
                     2 * Tm(1, 0) * Tm(1, 1) * dL_dc;
        dL_dcov[2] = 2 * Tm(0, 0) * Tm(0, 2) * dL_da + (Tm(0, 0) * Tm(1, 2) + Tm(0, 2) * Tm(1, 0)) * dL_db +
                     2 * Tm(1, 0) * Tm(1, 2) * dL_dc;
        dL_dcov[4] = 2 * Tm(0, 2) * Tm(0, 1) * dL_da + (Tm(0, 1) * Tm(1, 2) + Tm(0, 2) * Tm(1, 1)) * dL_db +
                     2 * Tm(1, 1) * Tm(1, 2) * dL_dc;
    } else {
        for (int i = 0; i < 6; ++i) dL_dcov[i] = 0;
    }
    double dL_dT[2][3];  /* backward.cu:230-241: dL_dT0k, dL_dT1k */
    for (int k = 0; k < 3; ++k) {
        const double tv0 = Tm(0, 0) * Vm(k, 0) + Tm(0, 1) * Vm(k, 1) + Tm(0, 2) * Vm(k, 2);
        const double tv1 = Tm(1, 0) * Vm(k, 0) + Tm(1, 1) * Vm(k, 1) + Tm(1, 2) * Vm(k, 2);
        dL_dT[0][k] = 2 * tv0 * dL_da + tv1 * dL_db;
        dL_dT[1][k] = 2 * tv1 * dL_dc + tv0 * dL_db;
    }
#undef Tm
#undef Vm
#define Wd(i, j) (Wm.c[i][j])
    const double dL_dJ00 = Wd(0, 0) * dL_dT[0][0] + Wd(0, 1) * dL_dT[0][1] + Wd(0, 2) * dL_dT[0][2];
    const double dL_dJ02 = Wd(2, 0) * dL_dT[0][0] + Wd(2, 1) * dL_dT[0][1] + Wd(2, 2) * dL_dT[0][2];
    const double dL_dJ11 = Wd(1, 0) * dL_dT[1][0] + Wd(1, 1) * dL_dT[1][1] + Wd(1, 2) * dL_dT[1][2];
    const double dL_dJ12 = Wd(2, 0) * dL_dT[1][0] + Wd(2, 1) * dL_dT[1][1] + Wd(2, 2) * dL_dT[1][2];
#undef Wd
    const double tz = 1.0 / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    const double dL_dtx = x_grad_mul * -dfx * tz2 * dL_dJ02;
    const double dL_dty = y_grad_mul * -dfy * tz2 * dL_dJ12;
    const double dL_dtz = -dfx * tz2 * dL_dJ00 - dfy * tz2 * dL_dJ11 + (2 * dfx * t.x) * tz3 * dL_dJ02 +
                          (2 * dfy * t.y) * tz3 * dL_dJ12;
    /* transformVec4x3Transpose (auxiliary.h:89-97) */
    return d3make((double)view[0] * dL_dtx + (double)view[1] * dL_dty + (double)view[2] * dL_dtz,
                  (double)view[4] * dL_dtx + (double)view[5] * dL_dty + (double)view[6] * dL_dtz,
                  (double)view[8] * dL_dtx + (double)view[9] * dL_dty + (double)view[10] * dL_dtz);
}

/* auxiliary.h:107-117 in double */
static d3 dnormvdv3_f64(d3 v, d3 dv) {
    const double sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    const double invsum32 = 1.0 / sqrt(sum2 * sum2 * sum2);
    return d3make(((sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32,
                  (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32,
                  (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32);
}

/* backward.cu:20-139 in double: writes dL_dsh ((deg+1)^2 rows), returns the view-direction mean gradient */
static d3 sh_bwd_f64(int deg, const float *posf, const float *camf, const float *sh_g, const unsigned char *clamped,
                     const double dL_dcolor[3], double *dL_dsh) {
    const d3 dir_orig = d3make((double)posf[0] - camf[0], (double)posf[1] - camf[1], (double)posf[2] - camf[2]);
    const double len = sqrt(d3dot(dir_orig, dir_orig));
    const double x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
#define SH(k) d3ld(sh_g + 3 * (k))
#define DSH(k, val) do { d3 _v = (val); dL_dsh[3 * (k)] = _v.x; dL_dsh[3 * (k) + 1] = _v.y; dL_dsh[3 * (k) + 2] = _v.z; } while (0)
    const d3 g = d3make(clamped[0] ? 0 : dL_dcolor[0], clamped[1] ? 0 : dL_dcolor[1], clamped[2] ? 0 : dL_dcolor[2]);
    d3 dx = d3make(0, 0, 0), dy = d3make(0, 0, 0), dz = d3make(0, 0, 0);
    DSH(0, d3scale(g, kD0));
    if (deg > 0) {
        DSH(1, d3scale(g, -kD1 * y));
        DSH(2, d3scale(g, kD1 * z));
        DSH(3, d3scale(g, -kD1 * x));
        dx = d3scale(SH(3), -kD1);
        dy = d3scale(SH(1), -kD1);
        dz = d3scale(SH(2), kD1);
        if (deg > 1) {
            const double xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            DSH(4, d3scale(g, kD2[0] * xy));
            DSH(5, d3scale(g, kD2[1] * yz));
            DSH(6, d3scale(g, kD2[2] * (2 * zz - xx - yy)));
            DSH(7, d3scale(g, kD2[3] * xz));
            DSH(8, d3scale(g, kD2[4] * (xx - yy)));
            dx = d3add(dx, d3add(d3add(d3add(d3scale(SH(4), kD2[0] * y), d3scale(SH(6), kD2[2] * 2 * -x)),
                                       d3scale(SH(7), kD2[3] * z)), d3scale(SH(8), kD2[4] * 2 * x)));
            dy = d3add(dy, d3add(d3add(d3add(d3scale(SH(4), kD2[0] * x), d3scale(SH(5), kD2[1] * z)),
                                       d3scale(SH(6), kD2[2] * 2 * -y)), d3scale(SH(8), kD2[4] * 2 * -y)));
            dz = d3add(dz, d3add(d3add(d3scale(SH(5), kD2[1] * y), d3scale(SH(6), kD2[2] * 2 * 2 * z)),
                                 d3scale(SH(7), kD2[3] * x)));
            if (deg > 2) {
                DSH(9, d3scale(g, kD3[0] * y * (3 * xx - yy)));
                DSH(10, d3scale(g, kD3[1] * xy * z));
                DSH(11, d3scale(g, kD3[2] * y * (4 * zz - xx - yy)));
                DSH(12, d3scale(g, kD3[3] * z * (2 * zz - 3 * xx - 3 * yy)));
                DSH(13, d3scale(g, kD3[4] * x * (4 * zz - xx - yy)));
                DSH(14, d3scale(g, kD3[5] * z * (xx - yy)));
                DSH(15, d3scale(g, kD3[6] * x * (xx - 3 * yy)));
                d3 tx = d3scale(SH(9), kD3[0] * 3 * 2 * xy);
                tx = d3add(tx, d3scale(SH(10), kD3[1] * yz));
                tx = d3add(tx, d3scale(SH(11), kD3[2] * -2 * xy));
                tx = d3add(tx, d3scale(SH(12), kD3[3] * -3 * 2 * xz));
                tx = d3add(tx, d3scale(SH(13), kD3[4] * (-3 * xx + 4 * zz - yy)));
                tx = d3add(tx, d3scale(SH(14), kD3[5] * 2 * xz));
                tx = d3add(tx, d3scale(SH(15), kD3[6] * 3 * (xx - yy)));
                d3 ty = d3scale(SH(9), kD3[0] * 3 * (xx - yy));
                ty = d3add(ty, d3scale(SH(10), kD3[1] * xz));
                ty = d3add(ty, d3scale(SH(11), kD3[2] * (-3 * yy + 4 * zz - xx)));
                ty = d3add(ty, d3scale(SH(12), kD3[3] * -3 * 2 * yz));
                ty = d3add(ty, d3scale(SH(13), kD3[4] * -2 * xy));
                ty = d3add(ty, d3scale(SH(14), kD3[5] * -2 * yz));
                ty = d3add(ty, d3scale(SH(15), kD3[6] * -3 * 2 * xy));
                d3 tzv = d3scale(SH(10), kD3[1] * xy);
                tzv = d3add(tzv, d3scale(SH(11), kD3[2] * 4 * 2 * yz));
                tzv = d3add(tzv, d3scale(SH(12), kD3[3] * 3 * (2 * zz - xx - yy)));
                tzv = d3add(tzv, d3scale(SH(13), kD3[4] * 4 * 2 * xz));
                tzv = d3add(tzv, d3scale(SH(14), kD3[5] * (xx - yy)));
                dx = d3add(dx, tx);
                dy = d3add(dy, ty);
                dz = d3add(dz, tzv);
            }
        }
    }
#undef SH
#undef DSH
    return dnormvdv3_f64(dir_orig, d3make(d3dot(dx, g), d3dot(dy, g), d3dot(dz, g)));
}

/* backward.cu:278-341 in double: gradients w.r.t. (mod * scale) and the unnormalised quaternion */
static void cov3d_bwd_f64(const float *scale, float mod, const float *rot, const double *dL_dcov3D, double *dL_dscale,
                          double *dL_drot) {
    const double r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    dm3 R = rot_matrix(r, x, y, z);
    const d3 s = d3make((double)mod * scale[0], (double)mod * scale[1], (double)mod * scale[2]);
    dm3 S = dm3cols(s.x, 0, 0, 0, s.y, 0, 0, 0, s.z);
    dm3 M = dm3mul(&S, &R);
    const double *g = dL_dcov3D;
    dm3 dSig = dm3cols(g[0], 0.5 * g[1], 0.5 * g[2], 0.5 * g[1], g[3], 0.5 * g[4], 0.5 * g[2], 0.5 * g[4], g[5]);
    dm3 M2;
    for (int c = 0; c < 3; ++c)
        for (int rr = 0; rr < 3; ++rr) M2.c[c][rr] = 2.0 * M.c[c][rr];
    dm3 dM = dm3mul(&M2, &dSig);
    dm3 Rt = dm3T(&R), dMt = dm3T(&dM);
    for (int i = 0; i < 3; ++i)
        dL_dscale[i] = Rt.c[i][0] * dMt.c[i][0] + Rt.c[i][1] * dMt.c[i][1] + Rt.c[i][2] * dMt.c[i][2];
    for (int k = 0; k < 3; ++k) { dMt.c[0][k] *= s.x; dMt.c[1][k] *= s.y; dMt.c[2][k] *= s.z; }
#define D(i, j) (dMt.c[i][j])
    dL_drot[0] = 2 * z * (D(0, 1) - D(1, 0)) + 2 * y * (D(2, 0) - D(0, 2)) + 2 * x * (D(1, 2) - D(2, 1));
    dL_drot[1] = 2 * y * (D(1, 0) + D(0, 1)) + 2 * z * (D(2, 0) + D(0, 2)) + 2 * r * (D(1, 2) - D(2, 1)) - 4 * x * (D(2, 2) + D(1, 1));
    dL_drot[2] = 2 * x * (D(1, 0) + D(0, 1)) + 2 * r * (D(2, 0) - D(0, 2)) + 2 * z * (D(1, 2) + D(2, 1)) - 4 * y * (D(2, 2) + D(0, 0));
    dL_drot[3] = 2 * r * (D(0, 1) - D(1, 0)) + 2 * x * (D(2, 0) + D(0, 2)) + 2 * y * (D(1, 2) + D(2, 1)) - 4 * z * (D(1, 1) + D(0, 0));
#undef D
}

int go_backward_chain_f64(go_state *st, const go_settings *s, const go_inputs *in, const double *g9,
                          double *dL_dmeans3D, double *dL_dcov3D, double *dL_dsh, double *dL_dscales,
                          double *dL_drotations) {
    const int P = in->P, M = in->M;
    if (P == 0) return GO_OK;
    memset(dL_dmeans3D, 0, 3 * (size_t)P * sizeof(double));
    memset(dL_dcov3D, 0, 6 * (size_t)P * sizeof(double));
    if (M > 0 && dL_dsh) memset(dL_dsh, 0, (size_t)P * M * 3 * sizeof(double));
    memset(dL_dscales, 0, 3 * (size_t)P * sizeof(double));
    memset(dL_drotations, 0, 4 * (size_t)P * sizeof(double));
    const float fy = s->image_height / (2.0f * s->tanfovy); /* rasterizer_impl.cu:190-191 (float constants) */
    const float fx = s->image_width / (2.0f * s->tanfovx);
    const float *proj = s->projmatrix;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; ++i) {
        if (!(st->radii[i] > 0)) continue;
        const double *g = g9 + 9 * (size_t)i;
        const float *mf = in->means3D + 3 * (size_t)i;
        double cov3[6];
        if (in->cov3D_precomp)
            for (int k = 0; k < 6; ++k) cov3[k] = in->cov3D_precomp[6 * (size_t)i + k];
        else
            cov3d_f64(in->scales + 3 * (size_t)i, s->scale_modifier, in->rotations + 4 * (size_t)i, cov3);
        const double gcon[3] = {g[2], g[3], g[4]};
        double *dcov = dL_dcov3D + 6 * (size_t)i;
        d3 gm = cov2d_bwd_f64(mf, fx, fy, s->tanfovx, s->tanfovy, cov3, s->viewmatrix, gcon, dcov);
        /* preprocessCUDA bwd (backward.cu:370-387) */
        const d3 m = d3ld(mf);
        const double mh3 = (double)proj[3] * m.x + (double)proj[7] * m.y + (double)proj[11] * m.z + proj[15];
        const double m_w = 1.0 / (mh3 + (double)0.0000001f);
        const double mul1 = ((double)proj[0] * m.x + (double)proj[4] * m.y + (double)proj[8] * m.z + proj[12]) * m_w * m_w;
        const double mul2 = ((double)proj[1] * m.x + (double)proj[5] * m.y + (double)proj[9] * m.z + proj[13]) * m_w * m_w;
        d3 dm;
        dm.x = (proj[0] * m_w - proj[3] * mul1) * g[0] + (proj[1] * m_w - proj[3] * mul2) * g[1];
        dm.y = (proj[4] * m_w - proj[7] * mul1) * g[0] + (proj[5] * m_w - proj[7] * mul2) * g[1];
        dm.z = (proj[8] * m_w - proj[11] * mul1) * g[0] + (proj[9] * m_w - proj[11] * mul2) * g[1];
        gm = d3add(gm, dm);
        if (in->shs)
            gm = d3add(gm, sh_bwd_f64(s->sh_degree, mf, s->campos, in->shs + (size_t)i * M * 3, st->clamped + 3 * (size_t)i,
                                      g + 6, dL_dsh + (size_t)i * M * 3));
        dL_dmeans3D[3 * (size_t)i] = gm.x;
        dL_dmeans3D[3 * (size_t)i + 1] = gm.y;
        dL_dmeans3D[3 * (size_t)i + 2] = gm.z;
        if (in->scales)
            cov3d_bwd_f64(in->scales + 3 * (size_t)i, s->scale_modifier, in->rotations + 4 * (size_t)i, dcov,
                          dL_dscales + 3 * (size_t)i, dL_drotations + 4 * (size_t)i);
    }
    return GO_OK;
}
