/*
 * gs_oracle.c — CPU restatement of the reference 3DGS rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY (see gs_oracle.h).  Every function cites the
 * reference file:line it restates; paths are relative to
 *   /root/reference/gaussiansplatting/submodules/diff-gaussian-rasterization/
 *
 * Conventions kept from the reference:
 *   - matrices are the reference's column-major float[16] (auxiliary.h:58-97);
 *   - 3x3 products follow glm's column-major semantics and evaluation order
 *     (glm mat3(a..i) takes column 0 first; operator* sums columns k=0,1,2);
 *   - ndc2Pix evaluates in double (its 1.0 literals, auxiliary.h:41-44);
 *   - stable (tile, depth) key sort: equal keys keep Gaussian-index order.
 */
#include "gs_oracle.h"
#include "gs_oracle_internal.h"

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif


/* auxiliary.h:22-39 */
static const float kC0 = 0.28209479177387814f;
static const float kC1 = 0.4886025119029199f;
static const float kC2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                             -1.0925484305920792f, 0.5462742152960396f};
static const float kC3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                             0.3731763325901154f,  -0.4570457994644658f, 1.445305721320277f,
                             -0.5900435899266435f};

static int g_threads = 1;

void go_set_threads(int n) {
    g_threads = n < 1 ? 1 : n;
#ifdef _OPENMP
    omp_set_num_threads(g_threads);
#endif
}
int go_get_threads(void) { return g_threads; }

/* ------------------------------------------------------------------ */
/* small vector / glm-style helpers                                    */
/* ------------------------------------------------------------------ */
typedef struct { float x, y, z; } v3;
typedef struct { float c[3][3]; } cm3; /* c[col][row], like glm::mat3 */

static v3 v3make(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static v3 v3add(v3 a, v3 b) { return v3make(a.x + b.x, a.y + b.y, a.z + b.z); }
static v3 v3sub(v3 a, v3 b) { return v3make(a.x - b.x, a.y - b.y, a.z - b.z); }
static v3 v3scale(v3 a, float s) { return v3make(a.x * s, a.y * s, a.z * s); }
static float v3dot(v3 a, v3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
static v3 v3ld(const float *p) { return v3make(p[0], p[1], p[2]); }

/* glm operator*(mat3, mat3): R[c] = A[0]*B[c][0] + A[1]*B[c][1] + A[2]*B[c][2] */
static cm3 cm3mul(const cm3 *A, const cm3 *B) {
    cm3 R;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r)
            R.c[c][r] = A->c[0][r] * B->c[c][0] + A->c[1][r] * B->c[c][1] + A->c[2][r] * B->c[c][2];
    return R;
}
static cm3 cm3T(const cm3 *A) {
    cm3 R;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) R.c[c][r] = A->c[r][c];
    return R;
}
/* glm mat3(a,b,c, d,e,f, g,h,i): column 0 = (a,b,c) */
static cm3 cm3cols(float a, float b, float c, float d, float e, float f, float g, float h, float i) {
    cm3 R;
    R.c[0][0] = a; R.c[0][1] = b; R.c[0][2] = c;
    R.c[1][0] = d; R.c[1][1] = e; R.c[1][2] = f;
    R.c[2][0] = g; R.c[2][1] = h; R.c[2][2] = i;
    return R;
}

/* auxiliary.h:58-77 */
static v3 xform_point43(v3 p, const float *m) {
    return v3make(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                  m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                  m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
static void xform_point44(v3 p, const float *m, float out[4]) {
    out[0] = m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12];
    out[1] = m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13];
    out[2] = m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14];
    out[3] = m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15];
}
/* auxiliary.h:89-97 */
static v3 xform_vec43_T(v3 p, const float *m) {
    return v3make(m[0] * p.x + m[1] * p.y + m[2] * p.z,
                  m[4] * p.x + m[5] * p.y + m[6] * p.z,
                  m[8] * p.x + m[9] * p.y + m[10] * p.z);
}

/* The blend's exp (forward.cu:345, backward.cu:495, apply_weights.cu): the
 * reference calls CUDA's expf (<= 2 ulp, unavailable here).  The oracle fixes
 * ONE exp as a sequence of IEEE single operations (<= 0.97 ulp vs exp over
 * [-10, 1], <= 0.86 ulp over every float of [-6, 0]; NaN -> NaN) that the HIP
 * path (dge_amd/csrc/gs_common.h gs_exp) evaluates identically, so every
 * alpha, every skip/stop decision, T and n_contrib can be compared bit for
 * bit.  fmaf is the correctly rounded fused multiply-add (built -mfma). */
GO_EXACT static float gs_expf(float x) {
    GO_EXACT_BODY
    float u = fmaf(x, 1.44269504f, 12582912.0f); /* 1.5 * 2^23 + rint(x log2e), the product unrounded */
    u = fminf(fmaxf(u, 12582912.0f - 120.0f), 12582912.0f + 120.0f);
    const float n = u - 12582912.0f;
    const float r = fmaf(n, -0.693147182f, x);
    float p = fmaf(1.98412698e-4f, r, 1.38888889e-3f);
    p = fmaf(p, r, 8.33333377e-3f);
    p = fmaf(p, r, 4.16666679e-2f);
    p = fmaf(p, r, 1.66666672e-1f);
    p = fmaf(p, r, 0.5f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    uint32_t ub, sb;
    memcpy(&ub, &u, 4);
    sb = (ub << 23) + 0x3F800000u; /* 2^n */
    float sc;
    memcpy(&sc, &sb, 4);
    return p * sc;
}

float go_expf1(float x) { return gs_expf(x); }

GO_EXACT int go_pixel_alpha(const float *co, float dx, float dy, float *G, float *alpha) {
    GO_EXACT_BODY
    const float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
    if (power > 0.0f) return 0;
    *G = gs_expf(power);
    *alpha = fminf(0.99f, co[3] * *G);
    return !(*alpha < 1.0f / 255.0f);
}

/* Test hook: gs_expf over an array (bit-compared with the GPU's gs_exp). */
void go_expf(int n, const float *x, float *y) {
    for (int i = 0; i < n; ++i) y[i] = gs_expf(x[i]);
}

/* auxiliary.h:41-44 — evaluated in double because of the 1.0 literals */
static float ndc_to_pixel(float v, int S) { return (float)((((double)v + 1.0) * S - 1.0) * 0.5); }

/* auxiliary.h:46-56 */
static void tile_rect(float px, float py, int r, int gx, int gy, int *x0, int *y0, int *x1, int *y1) {
    int a;
    a = (int)((px - (float)r) / (float)TILE_X); a = a < 0 ? 0 : a; *x0 = a > gx ? gx : a;
    a = (int)((py - (float)r) / (float)TILE_Y); a = a < 0 ? 0 : a; *y0 = a > gy ? gy : a;
    a = (int)((((px + (float)r) + (float)TILE_X) - 1.0f) / (float)TILE_X); a = a < 0 ? 0 : a; *x1 = a > gx ? gx : a;
    a = (int)((((py + (float)r) + (float)TILE_Y) - 1.0f) / (float)TILE_Y); a = a < 0 ? 0 : a; *y1 = a > gy ? gy : a;
}

/* ------------------------------------------------------------------ */
/* state                                                                */
/* ------------------------------------------------------------------ */
/* struct go_state: gs_oracle_internal.h */

void go_free(go_state *st) {
    if (!st) return;
    free(st->depths); free(st->clamped); free(st->radii); free(st->means2D); free(st->cov3D);
    free(st->conic_opacity); free(st->rgb); free(st->tiles_touched); free(st->point_offsets);
    free(st->point_keys); free(st->point_list); free(st->ranges); free(st->final_T);
    free(st->n_contrib);
    free(st->n_visited);
    free(st);
}

long go_state_get(go_state *st, const char *name, void **ptr) {
    struct { const char *n; void *p; long c; } t[] = {
        {"depths", st->depths, st->P},
        {"clamped", st->clamped, 3L * st->P},
        {"radii", st->radii, st->P},
        {"means2D", st->means2D, 2L * st->P},
        {"cov3D", st->cov3D, 6L * st->P},
        {"conic_opacity", st->conic_opacity, 4L * st->P},
        {"rgb", st->rgb, 3L * st->P},
        {"tiles_touched", st->tiles_touched, st->P},
        {"point_offsets", st->point_offsets, st->P},
        {"point_keys", st->point_keys, st->K},
        {"point_list", st->point_list, st->K},
        {"ranges", st->ranges, 2L * st->gx * st->gy},
        {"final_T", st->final_T, (long)st->W * st->H},
        {"n_contrib", st->n_contrib, (long)st->W * st->H},
        {"n_visited", st->n_visited, (long)st->W * st->H},
    };
    for (size_t i = 0; i < sizeof(t) / sizeof(t[0]); ++i)
        if (strcmp(t[i].n, name) == 0) { *ptr = t[i].p; return t[i].c; }
    *ptr = NULL;
    return -1;
}

/* ------------------------------------------------------------------ */
/* forward per-Gaussian math                                           */
/* ------------------------------------------------------------------ */

/* forward.cu:118-152 (quaternion deliberately NOT normalised, :127) */
static void cov3d_from_scale_rot(const float *scale, float mod, const float *rot, float out[6]) {
    cm3 S = cm3cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    S.c[0][0] = mod * scale[0];
    S.c[1][1] = mod * scale[1];
    S.c[2][2] = mod * scale[2];
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    cm3 R = cm3cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                    2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                    2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    cm3 M = cm3mul(&S, &R);
    cm3 Mt = cm3T(&M);
    cm3 Sig = cm3mul(&Mt, &M);
    out[0] = Sig.c[0][0]; out[1] = Sig.c[0][1]; out[2] = Sig.c[0][2];
    out[3] = Sig.c[1][1]; out[4] = Sig.c[1][2]; out[5] = Sig.c[2][2];
}

/* the shared camera-space Jacobian setup of forward.cu:80-104 and backward.cu:166-194 */
typedef struct {
    v3 t;            /* clamped camera-space mean */
    float txtz, tytz, limx, limy;
    cm3 J, W, T, V;
} ewa_ctx;

GO_EXACT static void ewa_setup(v3 mean, float fx, float fy, float tanfovx, float tanfovy, const float *cov3D,
                               const float *view, ewa_ctx *e) {
    GO_EXACT_BODY
    v3 t = xform_point43(mean, view);
    e->limx = 1.3f * tanfovx;
    e->limy = 1.3f * tanfovy;
    e->txtz = t.x / t.z;
    e->tytz = t.y / t.z;
    t.x = fminf(e->limx, fmaxf(-e->limx, e->txtz)) * t.z;
    t.y = fminf(e->limy, fmaxf(-e->limy, e->tytz)) * t.z;
    e->t = t;
    e->J = cm3cols(fx / t.z, 0.0f, -(fx * t.x) / (t.z * t.z), 0.0f, fy / t.z, -(fy * t.y) / (t.z * t.z), 0, 0, 0);
    e->W = cm3cols(view[0], view[4], view[8], view[1], view[5], view[9], view[2], view[6], view[10]);
    e->T = cm3mul(&e->W, &e->J);
    e->V = cm3cols(cov3D[0], cov3D[1], cov3D[2], cov3D[1], cov3D[3], cov3D[4], cov3D[2], cov3D[4], cov3D[5]);
}

/* forward.cu:74-113: returns (a, b, c) of the filtered 2D covariance */
static void ewa_cov2d(const ewa_ctx *e, float *a, float *b, float *c) {
    cm3 Tt = cm3T(&e->T), Vt = cm3T(&e->V);
    cm3 TtV = cm3mul(&Tt, &Vt);
    cm3 cov = cm3mul(&TtV, &e->T);
    *a = cov.c[0][0] + 0.3f;
    *b = cov.c[0][1];
    *c = cov.c[1][1] + 0.3f;
}

/* forward.cu:20-71 */
static void sh_to_rgb(int deg, int M, v3 pos, v3 campos, const float *shs_g, unsigned char clamped[3], float out[3]) {
    v3 dir = v3sub(pos, campos);
    float len = sqrtf(v3dot(dir, dir));
    dir = v3make(dir.x / len, dir.y / len, dir.z / len);
    const float *sh = shs_g;
    (void)M;
#define SH(k) v3ld(sh + 3 * (k))
    v3 res = v3scale(SH(0), kC0);
    if (deg > 0) {
        float x = dir.x, y = dir.y, z = dir.z;
        res = v3sub(v3add(v3sub(res, v3scale(SH(1), kC1 * y)), v3scale(SH(2), kC1 * z)), v3scale(SH(3), kC1 * x));
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            res = v3add(res, v3scale(SH(4), kC2[0] * xy));
            res = v3add(res, v3scale(SH(5), kC2[1] * yz));
            res = v3add(res, v3scale(SH(6), kC2[2] * (2.0f * zz - xx - yy)));
            res = v3add(res, v3scale(SH(7), kC2[3] * xz));
            res = v3add(res, v3scale(SH(8), kC2[4] * (xx - yy)));
            if (deg > 2) {
                res = v3add(res, v3scale(SH(9), kC3[0] * y * (3.0f * xx - yy)));
                res = v3add(res, v3scale(SH(10), kC3[1] * xy * z));
                res = v3add(res, v3scale(SH(11), kC3[2] * y * (4.0f * zz - xx - yy)));
                res = v3add(res, v3scale(SH(12), kC3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy)));
                res = v3add(res, v3scale(SH(13), kC3[4] * x * (4.0f * zz - xx - yy)));
                res = v3add(res, v3scale(SH(14), kC3[5] * z * (xx - yy)));
                res = v3add(res, v3scale(SH(15), kC3[6] * x * (xx - 3.0f * yy)));
            }
        }
    }
#undef SH
    res = v3make(res.x + 0.5f, res.y + 0.5f, res.z + 0.5f);
    clamped[0] = res.x < 0; clamped[1] = res.y < 0; clamped[2] = res.z < 0;
    out[0] = fmaxf(res.x, 0.0f); out[1] = fmaxf(res.y, 0.0f); out[2] = fmaxf(res.z, 0.0f);
}

/* forward.cu:155-256 (+ in_frustum, auxiliary.h:139-164); returns 0 or GO_ERR_PREFILTERED */
static int preprocess_one(int i, const go_settings *s, const go_inputs *in, float fx, float fy, go_state *st,
                          int want_rgb) {
    st->radii[i] = 0;
    st->tiles_touched[i] = 0;
    const float *view = s->viewmatrix, *proj = s->projmatrix;
    v3 p = v3ld(in->means3D + 3 * (size_t)i);
    float ph[4];
    xform_point44(p, proj, ph);
    float pw = 1.0f / (ph[3] + 0.0000001f);
    float pproj_x = ph[0] * pw, pproj_y = ph[1] * pw;
    v3 pv = xform_point43(p, view);
    if (pv.z <= 0.2f) return s->prefiltered ? GO_ERR_PREFILTERED : GO_OK;

    float *cov3 = st->cov3D + 6 * (size_t)i;
    if (in->cov3D_precomp) memcpy(cov3, in->cov3D_precomp + 6 * (size_t)i, 6 * sizeof(float));
    else cov3d_from_scale_rot(in->scales + 3 * (size_t)i, s->scale_modifier, in->rotations + 4 * (size_t)i, cov3);

    ewa_ctx e;
    ewa_setup(p, fx, fy, s->tanfovx, s->tanfovy, cov3, view, &e);
    float ca, cb, cc;
    ewa_cov2d(&e, &ca, &cb, &cc);
    float det = ca * cc - cb * cb;
    if (det == 0.0f) return GO_OK;
    float det_inv = 1.f / det;
    float con_x = cc * det_inv, con_y = -cb * det_inv, con_z = ca * det_inv;
    float mid = 0.5f * (ca + cc);
    float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    float rad = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
    float px = ndc_to_pixel(pproj_x, s->image_width), py = ndc_to_pixel(pproj_y, s->image_height);
    int x0, y0, x1, y1;
    tile_rect(px, py, (int)rad, st->gx, st->gy, &x0, &y0, &x1, &y1);
    if ((x1 - x0) * (y1 - y0) == 0) return GO_OK;

    if (want_rgb && !in->colors_precomp) {
        sh_to_rgb(s->sh_degree, in->M, p, v3ld(s->campos), in->shs + (size_t)i * in->M * 3, st->clamped + 3 * (size_t)i,
                  st->rgb + 3 * (size_t)i);
    }
    st->depths[i] = pv.z;
    st->radii[i] = (int)rad;
    st->means2D[2 * (size_t)i] = px;
    st->means2D[2 * (size_t)i + 1] = py;
    st->conic_opacity[4 * (size_t)i + 0] = con_x;
    st->conic_opacity[4 * (size_t)i + 1] = con_y;
    st->conic_opacity[4 * (size_t)i + 2] = con_z;
    st->conic_opacity[4 * (size_t)i + 3] = in->opacities[i];
    st->tiles_touched[i] = (uint32_t)((y1 - y0) * (x1 - x0));
    return GO_OK;
}

/* stable LSD radix sort of (u64 key, u32 value) — the semantics of cub::DeviceRadixSort::SortPairs */
static void sort_pairs_u64(uint64_t *keys, uint32_t *vals, size_t n) {
    if (n < 2) return;
    uint64_t *k2 = (uint64_t *)malloc(n * sizeof(uint64_t));
    uint32_t *v2 = (uint32_t *)malloc(n * sizeof(uint32_t));
    for (int shift = 0; shift < 64; shift += 8) {
        size_t cnt[257] = {0};
        for (size_t i = 0; i < n; ++i) cnt[((keys[i] >> shift) & 0xff) + 1]++;
        int trivial = 0;
        for (int d = 1; d <= 256; ++d) if (cnt[d] == n) trivial = 1;
        if (trivial) continue;
        for (int d = 1; d <= 256; ++d) cnt[d] += cnt[d - 1];
        for (size_t i = 0; i < n; ++i) {
            size_t o = cnt[(keys[i] >> shift) & 0xff]++;
            k2[o] = keys[i];
            v2[o] = vals[i];
        }
        memcpy(keys, k2, n * sizeof(uint64_t));
        memcpy(vals, v2, n * sizeof(uint32_t));
    }
    free(k2);
    free(v2);
}

static go_state *state_alloc(int P, int W, int H) {
    go_state *st = (go_state *)calloc(1, sizeof(go_state));
    st->P = P; st->W = W; st->H = H;
    st->gx = (W + TILE_X - 1) / TILE_X;
    st->gy = (H + TILE_Y - 1) / TILE_Y;
    size_t p = P > 0 ? (size_t)P : 1;
    st->depths = (float *)calloc(p, sizeof(float));
    st->clamped = (unsigned char *)calloc(3 * p, 1);
    st->radii = (int *)calloc(p, sizeof(int));
    st->means2D = (float *)calloc(2 * p, sizeof(float));
    st->cov3D = (float *)calloc(6 * p, sizeof(float));
    st->conic_opacity = (float *)calloc(4 * p, sizeof(float));
    st->rgb = (float *)calloc(3 * p, sizeof(float));
    st->tiles_touched = (uint32_t *)calloc(p, sizeof(uint32_t));
    st->point_offsets = (uint32_t *)calloc(p, sizeof(uint32_t));
    st->ranges = (uint32_t *)calloc(2 * (size_t)st->gx * st->gy, sizeof(uint32_t));
    st->final_T = (float *)calloc((size_t)W * H, sizeof(float));
    st->n_contrib = (uint32_t *)calloc((size_t)W * H, sizeof(uint32_t));
    st->n_visited = (uint32_t *)calloc((size_t)W * H, sizeof(uint32_t));
    return st;
}

/* rasterizer_impl.cu:179-285 minus render: preprocess, scan, duplicate, sort, ranges */
static int bin_gaussians(go_state *st, const go_settings *s, const go_inputs *in, int want_rgb) {
    const int P = in->P;
    const float fy = s->image_height / (2.0f * s->tanfovy); /* rasterizer_impl.cu:190-191 */
    const float fx = s->image_width / (2.0f * s->tanfovx);
    int err = GO_OK;
#pragma omp parallel for schedule(static) reduction(max : err)
    for (int i = 0; i < P; ++i) {
        int e = preprocess_one(i, s, in, fx, fy, st, want_rgb);
        if (e > err) err = e;
    }
    if (err) return err;
    /* inclusive scan (rasterizer_impl.cu:229-232) */
    uint32_t acc = 0;
    for (int i = 0; i < P; ++i) { acc += st->tiles_touched[i]; st->point_offsets[i] = acc; }
    st->K = (int)acc;
    size_t K = acc;
    st->point_keys = (uint64_t *)malloc((K ? K : 1) * sizeof(uint64_t));
    st->point_list = (uint32_t *)malloc((K ? K : 1) * sizeof(uint32_t));
    /* duplicateWithKeys (rasterizer_impl.cu:67-100) */
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; ++i) {
        if (st->radii[i] <= 0) continue;
        uint32_t off = i == 0 ? 0 : st->point_offsets[i - 1];
        int x0, y0, x1, y1;
        tile_rect(st->means2D[2 * (size_t)i], st->means2D[2 * (size_t)i + 1], st->radii[i], st->gx, st->gy, &x0, &y0, &x1, &y1);
        uint32_t dbits;
        memcpy(&dbits, &st->depths[i], 4);
        for (int y = y0; y < y1; ++y)
            for (int x = x0; x < x1; ++x) {
                st->point_keys[off] = ((uint64_t)(uint32_t)(y * st->gx + x) << 32) | dbits;
                st->point_list[off] = (uint32_t)i;
                off++;
            }
    }
    sort_pairs_u64(st->point_keys, st->point_list, K);
    /* identifyTileRanges (rasterizer_impl.cu:105-125) on zeroed ranges */
    for (size_t k = 0; k < K; ++k) {
        uint32_t tile = (uint32_t)(st->point_keys[k] >> 32);
        if (k == 0) st->ranges[2 * tile] = 0;
        else {
            uint32_t prev = (uint32_t)(st->point_keys[k - 1] >> 32);
            if (prev != tile) { st->ranges[2 * prev + 1] = (uint32_t)k; st->ranges[2 * tile] = (uint32_t)k; }
        }
        if (k == K - 1) st->ranges[2 * tile + 1] = (uint32_t)K;
    }
    return GO_OK;
}

/* forward.cu:261-379, one pixel */
static void render_pixel(const go_state *st, const float *features, const float *bg, int tile, int px, int py,
                         float *out_color, float *out_depth) {
    const uint32_t r0 = st->ranges[2 * tile], r1 = st->ranges[2 * tile + 1];
    const float pfx = (float)px, pfy = (float)py;
    float T = 1.0f, C[3] = {0, 0, 0}, D = 0;
    uint32_t contributor = 0, last = 0, visited_stop = 0;
    for (uint32_t k = r0; k < r1; ++k) {
        contributor++;
        visited_stop = contributor;
        uint32_t id = st->point_list[k];
        float dx = st->means2D[2 * (size_t)id] - pfx, dy = st->means2D[2 * (size_t)id + 1] - pfy;
        const float *co = st->conic_opacity + 4 * (size_t)id;
        float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
        if (power > 0.0f) continue;
        float alpha = fminf(0.99f, co[3] * gs_expf(power));
        if (alpha < 1.0f / 255.0f) continue;
        float test_T = T * (1 - alpha);
        if (test_T < 0.0001f) break;
        /* forward.cu:355-357 `C += f * alpha * T` as nvcc's default fmad contracts it:
         * fma(f * alpha, T, C) (the HIP blend evaluates the same operations) */
        for (int ch = 0; ch < 3; ++ch) C[ch] = fmaf(features[3 * (size_t)id + ch] * alpha, T, C[ch]);
        D = fmaf(st->depths[id] * alpha, T, D);
        T = test_T;
        last = contributor;
    }
    const size_t pix = (size_t)st->W * py + px;
    st->final_T[pix] = T;
    st->n_contrib[pix] = last;
    st->n_visited[pix] = visited_stop;
    const size_t HW = (size_t)st->W * st->H;
    /* forward.cu:376 `C + T * bg`, contracted: fma(T, bg, C) */
    for (int ch = 0; ch < 3; ++ch) out_color[ch * HW + pix] = fmaf(T, bg[ch], C[ch]);
    out_depth[pix] = D;
}

go_state *go_forward(const go_settings *s, const go_inputs *in, float *out_color, float *out_depth, int *radii,
                     int *num_rendered, int *err) {
    const int W = s->image_width, H = s->image_height, P = in->P;
    *err = GO_OK;
    *num_rendered = 0;
    go_state *st = state_alloc(P, W, H);
    if (P == 0) { /* rasterize_points.cu:57-72: outputs stay zero, no render */
        memset(out_color, 0, 3 * (size_t)W * H * sizeof(float));
        memset(out_depth, 0, (size_t)W * H * sizeof(float));
        st->point_keys = (uint64_t *)malloc(8);
        st->point_list = (uint32_t *)malloc(4);
        return st;
    }
    int e = bin_gaussians(st, s, in, 1);
    if (e) { *err = e; go_free(st); return NULL; }
    st->features = in->colors_precomp ? in->colors_precomp : st->rgb;
    const int ntiles = st->gx * st->gy;
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < ntiles; ++t) {
        const int tx = t % st->gx, ty = t / st->gx;
        for (int yy = 0; yy < TILE_Y; ++yy)
            for (int xx = 0; xx < TILE_X; ++xx) {
                int px = tx * TILE_X + xx, py = ty * TILE_Y + yy;
                if (px < W && py < H) render_pixel(st, st->features, s->bg, t, px, py, out_color, out_depth);
            }
    }
    memcpy(radii, st->radii, (size_t)P * sizeof(int));
    *num_rendered = st->K;
    return st;
}

/* ------------------------------------------------------------------ */
/* backward                                                            */
/* ------------------------------------------------------------------ */

/* backward.cu:399-557, one pixel.  Per-(instance) gradient records are kept
 * in double at the instance's sorted position: rec[9*k + {mx,my,cx,cy,cw,op,r,g,b}] */
/* mag (nullable): per instance, the same 9 fields of sum |sub-term|, the scale
 * against which a different summation order or factoring is judged (a
 * cancellation-aware tolerance: see tests/helpers.py raster_grads_close).  Each
 * gradient term is bounded by the absolute values of the products it adds:
 * dL_dalpha by sum_ch (|c| + |accum|) |dL_dch| T + |T_final/(1-alpha) bg.dL_dpix|,
 * dG/d(delx) by |G dx a| + |G dy b|, and so on. */
/* em (nullable): every (pixel, instance) term set appended as (Gaussian id, 9 float terms), in the order this
 * pixel computes them (go_backward_truth sums them in float in several admissible atomic arrival orders). */
static void emit_terms(go_emit *em, uint32_t id, const float t[9]) {
    if (em->n == em->cap) {
        em->cap = em->cap ? 2 * em->cap : 4096;
        em->ids = (uint32_t *)realloc(em->ids, em->cap * sizeof(uint32_t));
        em->terms = (float *)realloc(em->terms, em->cap * 9 * sizeof(float));
    }
    em->ids[em->n] = id;
    memcpy(em->terms + 9 * em->n, t, 9 * sizeof(float));
    em->n++;
}

static void render_pixel_bwd(const go_state *st, const float *colors, const float *bg, const float *dL_dpix, int tile,
                             int px, int py, double *rec, double *mag, go_emit *em) {
    const uint32_t r0 = st->ranges[2 * tile], r1 = st->ranges[2 * tile + 1];
    const float pfx = (float)px, pfy = (float)py;
    const size_t pix = (size_t)st->W * py + px, HW = (size_t)st->W * st->H;
    const float T_final = st->final_T[pix];
    float T = T_final;
    uint32_t contributor = r1 - r0;
    const uint32_t last_contributor = st->n_contrib[pix];
    float accum_rec[3] = {0, 0, 0}, dL_dpixel[3], last_color[3] = {0, 0, 0}, last_alpha = 0;
    for (int ch = 0; ch < 3; ++ch) dL_dpixel[ch] = dL_dpix[ch * HW + pix];
    const float ddelx_dx = (float)(0.5 * st->W), ddely_dy = (float)(0.5 * st->H);
    for (uint32_t k = r1; k-- > r0;) {
        contributor--;
        if (contributor >= last_contributor) continue;
        uint32_t id = st->point_list[k];
        float dx = st->means2D[2 * (size_t)id] - pfx, dy = st->means2D[2 * (size_t)id + 1] - pfy;
        const float *co = st->conic_opacity + 4 * (size_t)id;
        float G, alpha;
        if (!go_pixel_alpha(co, dx, dy, &G, &alpha)) continue;
        T = T / (1.f - alpha);
        float dchannel_dcolor = alpha * T;
        float dL_dalpha = 0.0f;
        float t9[9];
        for (int ch = 0; ch < 3; ++ch) {
            float c = colors[3 * (size_t)id + ch];
            accum_rec[ch] = last_alpha * last_color[ch] + (1.f - last_alpha) * accum_rec[ch];
            last_color[ch] = c;
            float dL_dch = dL_dpixel[ch];
            dL_dalpha += (c - accum_rec[ch]) * dL_dch;
            t9[6 + ch] = dchannel_dcolor * dL_dch;
        }
        dL_dalpha *= T;
        last_alpha = alpha;
        float bg_dot = 0;
        for (int ch = 0; ch < 3; ++ch) bg_dot += bg[ch] * dL_dpixel[ch];
        dL_dalpha += (-T_final / (1.f - alpha)) * bg_dot;
        float dL_dG = co[3] * dL_dalpha;
        float gdx = G * dx, gdy = G * dy;
        float dG_ddelx = -gdx * co[0] - gdy * co[1];
        float dG_ddely = -gdy * co[2] - gdx * co[1];
        t9[0] = dL_dG * dG_ddelx * ddelx_dx;
        t9[1] = dL_dG * dG_ddely * ddely_dy;
        t9[2] = -0.5f * gdx * dx * dL_dG;
        t9[3] = -0.5f * gdx * dy * dL_dG;
        t9[4] = -0.5f * gdy * dy * dL_dG;
        t9[5] = G * dL_dalpha;
        if (rec) {
            double *r = rec + 9 * (size_t)k;
            for (int j = 0; j < 9; ++j) r[j] += (double)t9[j];
        }
        if (em) emit_terms(em, id, t9);
        if (mag) {
            double ma = 0, bgm = 0;
            for (int ch = 0; ch < 3; ++ch) {
                double c = fabs((double)colors[3 * (size_t)id + ch]);
                ma += (c + fabs((double)accum_rec[ch])) * fabs((double)dL_dpixel[ch]);
                bgm += fabs((double)bg[ch] * dL_dpixel[ch]);
            }
            ma = ma * T + fabs((double)T_final / (1.0 - alpha)) * bgm; /* bounds |dL_dalpha| */
            const double mG = fabs((double)co[3]) * ma;                   /* bounds |dL_dG| */
            double *m = mag + 9 * (size_t)k;
            m[0] += mG * (fabs((double)gdx * co[0]) + fabs((double)gdy * co[1])) * ddelx_dx;
            m[1] += mG * (fabs((double)gdy * co[2]) + fabs((double)gdx * co[1])) * ddely_dy;
            m[2] += 0.5 * fabs((double)gdx * dx) * mG;
            m[3] += 0.5 * fabs((double)gdx * dy) * mG;
            m[4] += 0.5 * fabs((double)gdy * dy) * mG;
            m[5] += fabs((double)G) * ma;
            for (int ch = 0; ch < 3; ++ch) m[6 + ch] += fabs((double)dchannel_dcolor * dL_dpixel[ch]);
        }
    }
}

void go_render_pixel_terms(const go_state *st, const float *colors, const float *bg, const float *dL_dpix, int tile,
                           int px, int py, go_emit *em) {
    render_pixel_bwd(st, colors, bg, dL_dpix, tile, px, py, NULL, NULL, em);
}

/* backward.cu:144-274: writes dL_dcov (6) and returns the cov-path mean grad */
static v3 cov2d_bwd(v3 mean, float fx, float fy, float tanfovx, float tanfovy, const float *cov3D, const float *view,
                    const float dL_dconic[3], float dL_dcov[6]) {
    ewa_ctx e;
    ewa_setup(mean, fx, fy, tanfovx, tanfovy, cov3D, view, &e);
    const float x_grad_mul = e.txtz < -e.limx || e.txtz > e.limx ? 0 : 1;
    const float y_grad_mul = e.tytz < -e.limy || e.tytz > e.limy ? 0 : 1;
    const cm3 *T = &e.T, *W = &e.W, *V = &e.V;
    cm3 Tt = cm3T(T), Vt = cm3T(V);
    cm3 TtV = cm3mul(&Tt, &Vt);
    cm3 cov2D = cm3mul(&TtV, T);
    float a = cov2D.c[0][0] += 0.3f;
    float b = cov2D.c[0][1];
    float c = cov2D.c[1][1] += 0.3f;
    float denom = a * c - b * b;
    float dL_da = 0, dL_db = 0, dL_dc = 0;
    float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
#define Tm(i, j) (T->c[i][j])
#define Vm(i, j) (V->c[i][j])
    if (denom2inv != 0) {
        dL_da = denom2inv * (-c * c * dL_dconic[0] + 2 * b * c * dL_dconic[1] + (denom - a * c) * dL_dconic[2]);
        dL_dc = denom2inv * (-a * a * dL_dconic[2] + 2 * a * b * dL_dconic[1] + (denom - a * c) * dL_dconic[0]);
        dL_db = denom2inv * 2 * (b * c * dL_dconic[0] - (denom + 2 * b * b) * dL_dconic[1] + a * b * dL_dconic[2]);
        dL_dcov[0] = (Tm(0, 0) * Tm(0, 0) * dL_da + Tm(0, 0) * Tm(1, 0) * dL_db + Tm(1, 0) * Tm(1, 0) * dL_dc);
        dL_dcov[3] = (Tm(0, 1) * Tm(0, 1) * dL_da + Tm(0, 1) * Tm(1, 1) * dL_db + Tm(1, 1) * Tm(1, 1) * dL_dc);
        dL_dcov[5] = (Tm(0, 2) * Tm(0, 2) * dL_da + Tm(0, 2) * Tm(1, 2) * dL_db + Tm(1, 2) * Tm(1, 2) * dL_dc);
        dL_dcov[1] = 2 * Tm(0, 0) * Tm(0, 1) * dL_da + (Tm(0, 0) * Tm(1, 1) + Tm(0, 1) * Tm(1, 0)) * dL_db + 2 * Tm(1, 0) * Tm(1, 1) * dL_dc;
        dL_dcov[2] = 2 * Tm(0, 0) * Tm(0, 2) * dL_da + (Tm(0, 0) * Tm(1, 2) + Tm(0, 2) * Tm(1, 0)) * dL_db + 2 * Tm(1, 0) * Tm(1, 2) * dL_dc;
        dL_dcov[4] = 2 * Tm(0, 2) * Tm(0, 1) * dL_da + (Tm(0, 1) * Tm(1, 2) + Tm(0, 2) * Tm(1, 1)) * dL_db + 2 * Tm(1, 1) * Tm(1, 2) * dL_dc;
    } else {
        for (int i = 0; i < 6; ++i) dL_dcov[i] = 0;
    }
    float dL_dT00 = 2 * (Tm(0, 0) * Vm(0, 0) + Tm(0, 1) * Vm(0, 1) + Tm(0, 2) * Vm(0, 2)) * dL_da +
                    (Tm(1, 0) * Vm(0, 0) + Tm(1, 1) * Vm(0, 1) + Tm(1, 2) * Vm(0, 2)) * dL_db;
    float dL_dT01 = 2 * (Tm(0, 0) * Vm(1, 0) + Tm(0, 1) * Vm(1, 1) + Tm(0, 2) * Vm(1, 2)) * dL_da +
                    (Tm(1, 0) * Vm(1, 0) + Tm(1, 1) * Vm(1, 1) + Tm(1, 2) * Vm(1, 2)) * dL_db;
    float dL_dT02 = 2 * (Tm(0, 0) * Vm(2, 0) + Tm(0, 1) * Vm(2, 1) + Tm(0, 2) * Vm(2, 2)) * dL_da +
                    (Tm(1, 0) * Vm(2, 0) + Tm(1, 1) * Vm(2, 1) + Tm(1, 2) * Vm(2, 2)) * dL_db;
    float dL_dT10 = 2 * (Tm(1, 0) * Vm(0, 0) + Tm(1, 1) * Vm(0, 1) + Tm(1, 2) * Vm(0, 2)) * dL_dc +
                    (Tm(0, 0) * Vm(0, 0) + Tm(0, 1) * Vm(0, 1) + Tm(0, 2) * Vm(0, 2)) * dL_db;
    float dL_dT11 = 2 * (Tm(1, 0) * Vm(1, 0) + Tm(1, 1) * Vm(1, 1) + Tm(1, 2) * Vm(1, 2)) * dL_dc +
                    (Tm(0, 0) * Vm(1, 0) + Tm(0, 1) * Vm(1, 1) + Tm(0, 2) * Vm(1, 2)) * dL_db;
    float dL_dT12 = 2 * (Tm(1, 0) * Vm(2, 0) + Tm(1, 1) * Vm(2, 1) + Tm(1, 2) * Vm(2, 2)) * dL_dc +
                    (Tm(0, 0) * Vm(2, 0) + Tm(0, 1) * Vm(2, 1) + Tm(0, 2) * Vm(2, 2)) * dL_db;
#undef Tm
#undef Vm
#define Wm(i, j) (W->c[i][j])
    float dL_dJ00 = Wm(0, 0) * dL_dT00 + Wm(0, 1) * dL_dT01 + Wm(0, 2) * dL_dT02;
    float dL_dJ02 = Wm(2, 0) * dL_dT00 + Wm(2, 1) * dL_dT01 + Wm(2, 2) * dL_dT02;
    float dL_dJ11 = Wm(1, 0) * dL_dT10 + Wm(1, 1) * dL_dT11 + Wm(1, 2) * dL_dT12;
    float dL_dJ12 = Wm(2, 0) * dL_dT10 + Wm(2, 1) * dL_dT11 + Wm(2, 2) * dL_dT12;
#undef Wm
    const v3 t = e.t;
    float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    float dL_dtx = x_grad_mul * -fx * tz2 * dL_dJ02;
    float dL_dty = y_grad_mul * -fy * tz2 * dL_dJ12;
    float dL_dtz = -fx * tz2 * dL_dJ00 - fy * tz2 * dL_dJ11 + (2 * fx * t.x) * tz3 * dL_dJ02 + (2 * fy * t.y) * tz3 * dL_dJ12;
    return xform_vec43_T(v3make(dL_dtx, dL_dty, dL_dtz), view);
}

/* auxiliary.h:107-117 */
static v3 dnormvdv3(v3 v, v3 dv) {
    float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    return v3make(((+sum2 - v.x * v.x) * dv.x - v.y * v.x * dv.y - v.z * v.x * dv.z) * invsum32,
                  (-v.x * v.y * dv.x + (sum2 - v.y * v.y) * dv.y - v.z * v.y * dv.z) * invsum32,
                  (-v.x * v.z * dv.x - v.y * v.z * dv.y + (sum2 - v.z * v.z) * dv.z) * invsum32);
}

/* backward.cu:20-139: writes dL_dsh for (deg+1)^2 coefficients, returns the view-dir mean grad */
static v3 sh_bwd(int deg, v3 pos, v3 campos, const float *sh_g, const unsigned char *clamped, const float *dL_dcolor,
                 float *dL_dsh) {
    v3 dir_orig = v3sub(pos, campos);
    float len = sqrtf(v3dot(dir_orig, dir_orig));
    v3 dir = v3make(dir_orig.x / len, dir_orig.y / len, dir_orig.z / len);
#define SH(k) v3ld(sh_g + 3 * (k))
#define DSH(k, val) do { v3 _v = (val); dL_dsh[3 * (k)] = _v.x; dL_dsh[3 * (k) + 1] = _v.y; dL_dsh[3 * (k) + 2] = _v.z; } while (0)
    v3 g = v3make(dL_dcolor[0] * (clamped[0] ? 0 : 1), dL_dcolor[1] * (clamped[1] ? 0 : 1),
                  dL_dcolor[2] * (clamped[2] ? 0 : 1));
    v3 dx = v3make(0, 0, 0), dy = v3make(0, 0, 0), dz = v3make(0, 0, 0);
    float x = dir.x, y = dir.y, z = dir.z;
    DSH(0, v3scale(g, kC0));
    if (deg > 0) {
        DSH(1, v3scale(g, -kC1 * y));
        DSH(2, v3scale(g, kC1 * z));
        DSH(3, v3scale(g, -kC1 * x));
        dx = v3scale(SH(3), -kC1);
        dy = v3scale(SH(1), -kC1);
        dz = v3scale(SH(2), kC1);
        if (deg > 1) {
            float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            DSH(4, v3scale(g, kC2[0] * xy));
            DSH(5, v3scale(g, kC2[1] * yz));
            DSH(6, v3scale(g, kC2[2] * (2.f * zz - xx - yy)));
            DSH(7, v3scale(g, kC2[3] * xz));
            DSH(8, v3scale(g, kC2[4] * (xx - yy)));
            v3 sx = v3add(v3add(v3add(v3scale(SH(4), kC2[0] * y), v3scale(SH(6), kC2[2] * 2.f * -x)), v3scale(SH(7), kC2[3] * z)),
                          v3scale(SH(8), kC2[4] * 2.f * x));
            v3 sy = v3add(v3add(v3add(v3scale(SH(4), kC2[0] * x), v3scale(SH(5), kC2[1] * z)), v3scale(SH(6), kC2[2] * 2.f * -y)),
                          v3scale(SH(8), kC2[4] * 2.f * -y));
            v3 sz = v3add(v3add(v3scale(SH(5), kC2[1] * y), v3scale(SH(6), kC2[2] * 2.f * 2.f * z)), v3scale(SH(7), kC2[3] * x));
            dx = v3add(dx, sx);
            dy = v3add(dy, sy);
            dz = v3add(dz, sz);
            if (deg > 2) {
                DSH(9, v3scale(g, kC3[0] * y * (3.f * xx - yy)));
                DSH(10, v3scale(g, kC3[1] * xy * z));
                DSH(11, v3scale(g, kC3[2] * y * (4.f * zz - xx - yy)));
                DSH(12, v3scale(g, kC3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy)));
                DSH(13, v3scale(g, kC3[4] * x * (4.f * zz - xx - yy)));
                DSH(14, v3scale(g, kC3[5] * z * (xx - yy)));
                DSH(15, v3scale(g, kC3[6] * x * (xx - 3.f * yy)));
                v3 tx = v3scale(SH(9), kC3[0] * 3.f * 2.f * xy);
                tx = v3add(tx, v3scale(SH(10), kC3[1] * yz));
                tx = v3add(tx, v3scale(SH(11), kC3[2] * -2.f * xy));
                tx = v3add(tx, v3scale(SH(12), kC3[3] * -3.f * 2.f * xz));
                tx = v3add(tx, v3scale(SH(13), kC3[4] * (-3.f * xx + 4.f * zz - yy)));
                tx = v3add(tx, v3scale(SH(14), kC3[5] * 2.f * xz));
                tx = v3add(tx, v3scale(SH(15), kC3[6] * 3.f * (xx - yy)));
                v3 ty = v3scale(SH(9), kC3[0] * 3.f * (xx - yy));
                ty = v3add(ty, v3scale(SH(10), kC3[1] * xz));
                ty = v3add(ty, v3scale(SH(11), kC3[2] * (-3.f * yy + 4.f * zz - xx)));
                ty = v3add(ty, v3scale(SH(12), kC3[3] * -3.f * 2.f * yz));
                ty = v3add(ty, v3scale(SH(13), kC3[4] * -2.f * xy));
                ty = v3add(ty, v3scale(SH(14), kC3[5] * -2.f * yz));
                ty = v3add(ty, v3scale(SH(15), kC3[6] * -3.f * 2.f * xy));
                v3 tzv = v3scale(SH(10), kC3[1] * xy);
                tzv = v3add(tzv, v3scale(SH(11), kC3[2] * 4.f * 2.f * yz));
                tzv = v3add(tzv, v3scale(SH(12), kC3[3] * 3.f * (2.f * zz - xx - yy)));
                tzv = v3add(tzv, v3scale(SH(13), kC3[4] * 4.f * 2.f * xz));
                tzv = v3add(tzv, v3scale(SH(14), kC3[5] * (xx - yy)));
                dx = v3add(dx, tx);
                dy = v3add(dy, ty);
                dz = v3add(dz, tzv);
            }
        }
    }
#undef SH
#undef DSH
    v3 dL_ddir = v3make(v3dot(dx, g), v3dot(dy, g), v3dot(dz, g));
    return dnormvdv3(dir_orig, dL_ddir);
}

/* backward.cu:278-341: gradients w.r.t. (mod*scale) and the unnormalised quaternion */
static void cov3d_bwd(const float *scale, float mod, const float *rot, const float *dL_dcov3D, float *dL_dscale,
                      float *dL_drot) {
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    cm3 R = cm3cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                    2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                    2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    cm3 S = cm3cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    v3 s = v3make(mod * scale[0], mod * scale[1], mod * scale[2]);
    S.c[0][0] = s.x; S.c[1][1] = s.y; S.c[2][2] = s.z;
    cm3 M = cm3mul(&S, &R);
    const float *g = dL_dcov3D;
    cm3 dSig = cm3cols(g[0], 0.5f * g[1], 0.5f * g[2], 0.5f * g[1], g[3], 0.5f * g[4], 0.5f * g[2], 0.5f * g[4], g[5]);
    cm3 M2;
    for (int c = 0; c < 3; ++c) for (int rr = 0; rr < 3; ++rr) M2.c[c][rr] = 2.0f * M.c[c][rr];
    cm3 dM = cm3mul(&M2, &dSig);
    cm3 Rt = cm3T(&R), dMt = cm3T(&dM);
    dL_dscale[0] = Rt.c[0][0] * dMt.c[0][0] + Rt.c[0][1] * dMt.c[0][1] + Rt.c[0][2] * dMt.c[0][2];
    dL_dscale[1] = Rt.c[1][0] * dMt.c[1][0] + Rt.c[1][1] * dMt.c[1][1] + Rt.c[1][2] * dMt.c[1][2];
    dL_dscale[2] = Rt.c[2][0] * dMt.c[2][0] + Rt.c[2][1] * dMt.c[2][1] + Rt.c[2][2] * dMt.c[2][2];
    for (int k = 0; k < 3; ++k) { dMt.c[0][k] *= s.x; dMt.c[1][k] *= s.y; dMt.c[2][k] *= s.z; }
#define D(i, j) (dMt.c[i][j])
    dL_drot[0] = 2 * z * (D(0, 1) - D(1, 0)) + 2 * y * (D(2, 0) - D(0, 2)) + 2 * x * (D(1, 2) - D(2, 1));
    dL_drot[1] = 2 * y * (D(1, 0) + D(0, 1)) + 2 * z * (D(2, 0) + D(0, 2)) + 2 * r * (D(1, 2) - D(2, 1)) - 4 * x * (D(2, 2) + D(1, 1));
    dL_drot[2] = 2 * x * (D(1, 0) + D(0, 1)) + 2 * r * (D(2, 0) - D(0, 2)) + 2 * z * (D(1, 2) + D(2, 1)) - 4 * y * (D(2, 2) + D(0, 0));
    dL_drot[3] = 2 * r * (D(0, 1) - D(1, 0)) + 2 * x * (D(2, 0) + D(0, 2)) + 2 * y * (D(1, 2) + D(2, 1)) - 4 * z * (D(1, 1) + D(0, 0));
#undef D
}

/* computeCov2DCUDA + preprocessCUDA bwd (backward.cu:144-396) of Gaussian i from
 * its summed rasterizer gradients g9 = (dL_dmean2D x, y, dL_dconic x, y, w,
 * dL_dopacity, dL_dcolor r, g, b) in float. */
static void gauss_chain(const go_state *st, const go_settings *s, const go_inputs *in, int i, const float g9[9],
                        float *dL_dmeans3D, float *dL_dcov3D, float *dL_dsh, float *dL_dscales, float *dL_drotations) {
    const int M = in->M;
    if (!(st->radii[i] > 0)) return;
    const float fy = s->image_height / (2.0f * s->tanfovy);
    const float fx = s->image_width / (2.0f * s->tanfovx);
    const float *proj = s->projmatrix;
    const float g2x = g9[0], g2y = g9[1];
    const float gcon[3] = {g9[2], g9[3], g9[4]};
    v3 m = v3ld(in->means3D + 3 * (size_t)i);
    const float *cov3 = in->cov3D_precomp ? in->cov3D_precomp + 6 * (size_t)i : st->cov3D + 6 * (size_t)i;
    /* computeCov2DCUDA: assignment (backward.cu:273) */
    v3 gm = cov2d_bwd(m, fx, fy, s->tanfovx, s->tanfovy, cov3, s->viewmatrix, gcon, dL_dcov3D + 6 * (size_t)i);
    /* preprocessCUDA bwd (backward.cu:370-387) */
    float mh[4];
    xform_point44(m, proj, mh);
    float m_w = 1.0f / (mh[3] + 0.0000001f);
    float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
    float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
    v3 dm;
    dm.x = (proj[0] * m_w - proj[3] * mul1) * g2x + (proj[1] * m_w - proj[3] * mul2) * g2y;
    dm.y = (proj[4] * m_w - proj[7] * mul1) * g2x + (proj[5] * m_w - proj[7] * mul2) * g2y;
    dm.z = (proj[8] * m_w - proj[11] * mul1) * g2x + (proj[9] * m_w - proj[11] * mul2) * g2y;
    gm = v3add(gm, dm);
    if (in->shs) {
        v3 gdir = sh_bwd(s->sh_degree, m, v3ld(s->campos), in->shs + (size_t)i * M * 3, st->clamped + 3 * (size_t)i,
                         g9 + 6, dL_dsh + (size_t)i * M * 3);
        gm = v3add(gm, gdir);
    }
    dL_dmeans3D[3 * (size_t)i] = gm.x;
    dL_dmeans3D[3 * (size_t)i + 1] = gm.y;
    dL_dmeans3D[3 * (size_t)i + 2] = gm.z;
    if (in->scales)
        cov3d_bwd(in->scales + 3 * (size_t)i, s->scale_modifier, in->rotations + 4 * (size_t)i,
                  dL_dcov3D + 6 * (size_t)i, dL_dscales + 3 * (size_t)i, dL_drotations + 4 * (size_t)i);
}

static void zero_param_grads(const go_inputs *in, float *dL_dmeans3D, float *dL_dcov3D, float *dL_dsh,
                             float *dL_dscales, float *dL_drotations) {
    const int P = in->P, M = in->M;
    memset(dL_dmeans3D, 0, 3 * (size_t)P * sizeof(float));
    memset(dL_dcov3D, 0, 6 * (size_t)P * sizeof(float));
    if (M > 0 && dL_dsh) memset(dL_dsh, 0, (size_t)P * M * 3 * sizeof(float));
    memset(dL_dscales, 0, 3 * (size_t)P * sizeof(float));
    memset(dL_drotations, 0, 4 * (size_t)P * sizeof(float));
}

int go_backward(go_state *st, const go_settings *s, const go_inputs *in, const float *dL_dpix, float *dL_dmeans2D,
                float *dL_dcolors, float *dL_dopacity, float *dL_dmeans3D, float *dL_dcov3D, float *dL_dsh,
                float *dL_dscales, float *dL_drotations, float *dL_dconic, float *mag9) {
    const int P = in->P;
    if (P == 0) return GO_OK;
    memset(dL_dmeans2D, 0, 3 * (size_t)P * sizeof(float));
    memset(dL_dcolors, 0, 3 * (size_t)P * sizeof(float));
    memset(dL_dopacity, 0, (size_t)P * sizeof(float));
    zero_param_grads(in, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations);
    if (dL_dconic) memset(dL_dconic, 0, 4 * (size_t)P * sizeof(float));

    const size_t K = (size_t)st->K;
    double *rec = (double *)calloc((K ? K : 1) * 9, sizeof(double));
    double *mrec = mag9 ? (double *)calloc((K ? K : 1) * 9, sizeof(double)) : NULL;
    const float *colors = in->colors_precomp ? in->colors_precomp : st->rgb;
    const int ntiles = st->gx * st->gy, W = st->W, H = st->H;
#pragma omp parallel for schedule(dynamic, 4)
    for (int t = 0; t < ntiles; ++t) {
        const int tx = t % st->gx, ty = t / st->gx;
        for (int yy = 0; yy < TILE_Y; ++yy)
            for (int xx = 0; xx < TILE_X; ++xx) {
                int px = tx * TILE_X + xx, py = ty * TILE_Y + yy;
                if (px < W && py < H) render_pixel_bwd(st, colors, s->bg, dL_dpix, t, px, py, rec, mrec, NULL);
            }
    }
    /* per-Gaussian sums over its instances, in sorted order (deterministic) */
    double *acc = (double *)calloc((size_t)P * 9, sizeof(double));
    double *macc = mag9 ? (double *)calloc((size_t)P * 9, sizeof(double)) : NULL;
    for (size_t k = 0; k < K; ++k) {
        double *a = acc + 9 * (size_t)st->point_list[k];
        const double *r = rec + 9 * k;
        for (int j = 0; j < 9; ++j) a[j] += r[j];
        if (macc) {
            double *ma = macc + 9 * (size_t)st->point_list[k];
            for (int j = 0; j < 9; ++j) ma[j] += mrec[9 * k + j];
        }
    }
    free(rec);
    free(mrec);
    if (macc) {
        for (size_t j = 0; j < (size_t)P * 9; ++j) mag9[j] = (float)macc[j];
        free(macc);
    }

#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; ++i) {
        const double *a = acc + 9 * (size_t)i;
        float g9[9];
        for (int j = 0; j < 9; ++j) g9[j] = (float)a[j];
        dL_dmeans2D[3 * (size_t)i] = g9[0];
        dL_dmeans2D[3 * (size_t)i + 1] = g9[1];
        dL_dopacity[i] = g9[5];
        for (int ch = 0; ch < 3; ++ch) dL_dcolors[3 * (size_t)i + ch] = g9[6 + ch];
        if (dL_dconic) {
            dL_dconic[4 * (size_t)i] = g9[2];
            dL_dconic[4 * (size_t)i + 1] = g9[3];
            dL_dconic[4 * (size_t)i + 3] = g9[4];
        }
        gauss_chain(st, s, in, i, g9, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations);
    }
    free(acc);
    return GO_OK;
}

/* The per-Gaussian chain alone, from given float sums g9 [P,9] (the layout of
 * gauss_chain): isolates the rasterizer's summation (order-dependent) from the
 * chain rule after it (fixed IEEE operations, comparable bit for bit). */
int go_backward_chain(go_state *st, const go_settings *s, const go_inputs *in, const float *g9, float *dL_dmeans3D,
                      float *dL_dcov3D, float *dL_dsh, float *dL_dscales, float *dL_drotations) {
    const int P = in->P;
    if (P == 0) return GO_OK;
    zero_param_grads(in, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; ++i)
        gauss_chain(st, s, in, i, g9 + 9 * (size_t)i, dL_dmeans3D, dL_dcov3D, dL_dsh, dL_dscales, dL_drotations);
    return GO_OK;
}

/* ------------------------------------------------------------------ */
/* Magnitude of the chain's terms (test infrastructure for the per-    */
/* element gradient bar): gauss_chain evaluated in absolute arithmetic */
/* ------------------------------------------------------------------ */
/* Every output of the chain is a sum of products (forward-state coefficient) x (a rasterizer sum).
 * go_backward_chain_mag evaluates the same chain with each coefficient's absolute value, each
 * subtraction as an addition and the inputs replaced by per-sum magnitudes m9 (the oracle's mag9:
 * sums of |sub-term| over the contributing pixels), in double: the result bounds |chain(g)| for any
 * |g| <= m9, so it is the scale against which both a reordered rasterizer sum and the chain's own
 * float rounding (whose error is u x the terms it adds, cancelled or not) are measured.  Coefficients
 * (T, V, W, the SH direction terms, R, S, ...) are computed exactly as the float chain computes them:
 * they are forward state, identical wherever the forward is. */
#define FA(x) fabs((double)(x))
static void cov2d_bwd_mag(v3 mean, float fx, float fy, float tanfovx, float tanfovy, const float *cov3D,
                          const float *view, const double mcon[3], double mcov[6], double mgm[3]) {
    ewa_ctx e;
    ewa_setup(mean, fx, fy, tanfovx, tanfovy, cov3D, view, &e);
    const double xm = e.txtz < -e.limx || e.txtz > e.limx ? 0 : 1;
    const double ym = e.tytz < -e.limy || e.tytz > e.limy ? 0 : 1;
    const cm3 *T = &e.T, *W = &e.W, *V = &e.V;
    cm3 Tt = cm3T(T), Vt = cm3T(V);
    cm3 TtV = cm3mul(&Tt, &Vt);
    cm3 cov2D = cm3mul(&TtV, T);
    float a = cov2D.c[0][0] += 0.3f;
    float b = cov2D.c[0][1];
    float c = cov2D.c[1][1] += 0.3f;
    float denom = a * c - b * b;
    float denom2inv = 1.0f / ((denom * denom) + 0.0000001f);
    double ma = 0, mb = 0, mc = 0;
#define Tm(i, j) (T->c[i][j])
#define Vm(i, j) (V->c[i][j])
    for (int i = 0; i < 6; ++i) mcov[i] = 0;
    if (denom2inv != 0) {
        ma = FA(denom2inv) * (FA(c * c) * mcon[0] + FA(2 * b * c) * mcon[1] + FA(denom - a * c) * mcon[2]);
        mc = FA(denom2inv) * (FA(a * a) * mcon[2] + FA(2 * a * b) * mcon[1] + FA(denom - a * c) * mcon[0]);
        mb = FA(denom2inv) * 2 * (FA(b * c) * mcon[0] + FA(denom + 2 * b * b) * mcon[1] + FA(a * b) * mcon[2]);
        mcov[0] = FA(Tm(0, 0) * Tm(0, 0)) * ma + FA(Tm(0, 0) * Tm(1, 0)) * mb + FA(Tm(1, 0) * Tm(1, 0)) * mc;
        mcov[3] = FA(Tm(0, 1) * Tm(0, 1)) * ma + FA(Tm(0, 1) * Tm(1, 1)) * mb + FA(Tm(1, 1) * Tm(1, 1)) * mc;
        mcov[5] = FA(Tm(0, 2) * Tm(0, 2)) * ma + FA(Tm(0, 2) * Tm(1, 2)) * mb + FA(Tm(1, 2) * Tm(1, 2)) * mc;
        mcov[1] = FA(2 * Tm(0, 0) * Tm(0, 1)) * ma + (FA(Tm(0, 0) * Tm(1, 1)) + FA(Tm(0, 1) * Tm(1, 0))) * mb +
                  FA(2 * Tm(1, 0) * Tm(1, 1)) * mc;
        mcov[2] = FA(2 * Tm(0, 0) * Tm(0, 2)) * ma + (FA(Tm(0, 0) * Tm(1, 2)) + FA(Tm(0, 2) * Tm(1, 0))) * mb +
                  FA(2 * Tm(1, 0) * Tm(1, 2)) * mc;
        mcov[4] = FA(2 * Tm(0, 2) * Tm(0, 1)) * ma + (FA(Tm(0, 1) * Tm(1, 2)) + FA(Tm(0, 2) * Tm(1, 1))) * mb +
                  FA(2 * Tm(1, 1) * Tm(1, 2)) * mc;
    }
    double mT[2][3];
    for (int k = 0; k < 3; ++k) {  /* dL_dT0k, dL_dT1k (backward.cu:230-241), terms kept separate */
        double tv0 = 0, tv1 = 0;
        for (int j = 0; j < 3; ++j) { tv0 += FA(Tm(0, j) * Vm(k, j)); tv1 += FA(Tm(1, j) * Vm(k, j)); }
        mT[0][k] = 2 * tv0 * ma + tv1 * mb;
        mT[1][k] = 2 * tv1 * mc + tv0 * mb;
    }
#undef Tm
#undef Vm
#define Wm(i, j) FA(W->c[i][j])
    double mJ00 = Wm(0, 0) * mT[0][0] + Wm(0, 1) * mT[0][1] + Wm(0, 2) * mT[0][2];
    double mJ02 = Wm(2, 0) * mT[0][0] + Wm(2, 1) * mT[0][1] + Wm(2, 2) * mT[0][2];
    double mJ11 = Wm(1, 0) * mT[1][0] + Wm(1, 1) * mT[1][1] + Wm(1, 2) * mT[1][2];
    double mJ12 = Wm(2, 0) * mT[1][0] + Wm(2, 1) * mT[1][1] + Wm(2, 2) * mT[1][2];
#undef Wm
    const v3 t = e.t;
    float tz = 1.f / t.z, tz2 = tz * tz, tz3 = tz2 * tz;
    double mtx = xm * FA(fx * tz2) * mJ02;
    double mty = ym * FA(fy * tz2) * mJ12;
    double mtz = FA(fx * tz2) * mJ00 + FA(fy * tz2) * mJ11 + FA((2 * fx * t.x) * tz3) * mJ02 + FA((2 * fy * t.y) * tz3) * mJ12;
    /* xform_vec43_T with |view| */
    mgm[0] = FA(view[0]) * mtx + FA(view[1]) * mty + FA(view[2]) * mtz;
    mgm[1] = FA(view[4]) * mtx + FA(view[5]) * mty + FA(view[6]) * mtz;
    mgm[2] = FA(view[8]) * mtx + FA(view[9]) * mty + FA(view[10]) * mtz;
}

/* sh_bwd in absolute arithmetic: |dL_dsh| bounds and the view-direction mean-gradient magnitude */
static void sh_bwd_mag(int deg, v3 pos, v3 campos, const float *sh_g, const unsigned char *clamped,
                       const double mcol[3], double *msh, double mdir[3]) {
    v3 dir_orig = v3sub(pos, campos);
    float len = sqrtf(v3dot(dir_orig, dir_orig));
    float x = dir_orig.x / len, y = dir_orig.y / len, z = dir_orig.z / len;
    const double mg[3] = {clamped[0] ? 0 : mcol[0], clamped[1] ? 0 : mcol[1], clamped[2] ? 0 : mcol[2]};
    /* basis coefficient of each SH row (the DSH scalars of sh_bwd) */
    float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
    float basis[16] = {kC0, -kC1 * y, kC1 * z, -kC1 * x, kC2[0] * xy, kC2[1] * yz, kC2[2] * (2.f * zz - xx - yy),
                       kC2[3] * xz, kC2[4] * (xx - yy), kC3[0] * y * (3.f * xx - yy), kC3[1] * xy * z,
                       kC3[2] * y * (4.f * zz - xx - yy), kC3[3] * z * (2.f * zz - 3.f * xx - 3.f * yy),
                       kC3[4] * x * (4.f * zz - xx - yy), kC3[5] * z * (xx - yy), kC3[6] * x * (xx - 3.f * yy)};
    const int n = deg == 0 ? 1 : deg == 1 ? 4 : deg == 2 ? 9 : 16;
    for (int k = 0; k < n; ++k)
        for (int ch = 0; ch < 3; ++ch) msh[3 * k + ch] = FA(basis[k]) * mg[ch];
    /* dL_ddir = (dx.g, dy.g, dz.g): dx, dy, dz do not depend on g (forward state), recomputed here with
     * sh_bwd's sums */
    double mdd[3] = {0, 0, 0};
    if (deg > 0) {
#define SH(k) v3ld(sh_g + 3 * (k))
        v3 dx = v3scale(SH(3), -kC1), dy = v3scale(SH(1), -kC1), dz = v3scale(SH(2), kC1);
        if (deg > 1) {
            v3 sx = v3add(v3add(v3add(v3scale(SH(4), kC2[0] * y), v3scale(SH(6), kC2[2] * 2.f * -x)), v3scale(SH(7), kC2[3] * z)),
                          v3scale(SH(8), kC2[4] * 2.f * x));
            v3 sy = v3add(v3add(v3add(v3scale(SH(4), kC2[0] * x), v3scale(SH(5), kC2[1] * z)), v3scale(SH(6), kC2[2] * 2.f * -y)),
                          v3scale(SH(8), kC2[4] * 2.f * -y));
            v3 sz = v3add(v3add(v3scale(SH(5), kC2[1] * y), v3scale(SH(6), kC2[2] * 2.f * 2.f * z)), v3scale(SH(7), kC2[3] * x));
            dx = v3add(dx, sx); dy = v3add(dy, sy); dz = v3add(dz, sz);
            if (deg > 2) {
                v3 tx = v3scale(SH(9), kC3[0] * 3.f * 2.f * xy);
                tx = v3add(tx, v3scale(SH(10), kC3[1] * yz));
                tx = v3add(tx, v3scale(SH(11), kC3[2] * -2.f * xy));
                tx = v3add(tx, v3scale(SH(12), kC3[3] * -3.f * 2.f * xz));
                tx = v3add(tx, v3scale(SH(13), kC3[4] * (-3.f * xx + 4.f * zz - yy)));
                tx = v3add(tx, v3scale(SH(14), kC3[5] * 2.f * xz));
                tx = v3add(tx, v3scale(SH(15), kC3[6] * 3.f * (xx - yy)));
                v3 ty = v3scale(SH(9), kC3[0] * 3.f * (xx - yy));
                ty = v3add(ty, v3scale(SH(10), kC3[1] * xz));
                ty = v3add(ty, v3scale(SH(11), kC3[2] * (-3.f * yy + 4.f * zz - xx)));
                ty = v3add(ty, v3scale(SH(12), kC3[3] * -3.f * 2.f * yz));
                ty = v3add(ty, v3scale(SH(13), kC3[4] * -2.f * xy));
                ty = v3add(ty, v3scale(SH(14), kC3[5] * -2.f * yz));
                ty = v3add(ty, v3scale(SH(15), kC3[6] * -3.f * 2.f * xy));
                v3 tzv = v3scale(SH(10), kC3[1] * xy);
                tzv = v3add(tzv, v3scale(SH(11), kC3[2] * 4.f * 2.f * yz));
                tzv = v3add(tzv, v3scale(SH(12), kC3[3] * 3.f * (2.f * zz - xx - yy)));
                tzv = v3add(tzv, v3scale(SH(13), kC3[4] * 4.f * 2.f * xz));
                tzv = v3add(tzv, v3scale(SH(14), kC3[5] * (xx - yy)));
                dx = v3add(dx, tx); dy = v3add(dy, ty); dz = v3add(dz, tzv);
            }
        }
#undef SH
        mdd[0] = FA(dx.x) * mg[0] + FA(dx.y) * mg[1] + FA(dx.z) * mg[2];
        mdd[1] = FA(dy.x) * mg[0] + FA(dy.y) * mg[1] + FA(dy.z) * mg[2];
        mdd[2] = FA(dz.x) * mg[0] + FA(dz.y) * mg[1] + FA(dz.z) * mg[2];
    }
    /* dnormvdv3 with absolute coefficients */
    v3 v = dir_orig;
    float sum2 = v.x * v.x + v.y * v.y + v.z * v.z;
    float invsum32 = 1.0f / sqrtf(sum2 * sum2 * sum2);
    mdir[0] = (FA(sum2 - v.x * v.x) * mdd[0] + FA(v.y * v.x) * mdd[1] + FA(v.z * v.x) * mdd[2]) * FA(invsum32);
    mdir[1] = (FA(v.x * v.y) * mdd[0] + FA(sum2 - v.y * v.y) * mdd[1] + FA(v.z * v.y) * mdd[2]) * FA(invsum32);
    mdir[2] = (FA(v.x * v.z) * mdd[0] + FA(v.y * v.z) * mdd[1] + FA(sum2 - v.z * v.z) * mdd[2]) * FA(invsum32);
}

/* cov3d_bwd in absolute arithmetic */
static void cov3d_bwd_mag(const float *scale, float mod, const float *rot, const double mcov[6], double mscale[3],
                          double mrot[4]) {
    float r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    cm3 R = cm3cols(1.f - 2.f * (y * y + z * z), 2.f * (x * y - r * z), 2.f * (x * z + r * y),
                    2.f * (x * y + r * z), 1.f - 2.f * (x * x + z * z), 2.f * (y * z - r * x),
                    2.f * (x * z - r * y), 2.f * (y * z + r * x), 1.f - 2.f * (x * x + y * y));
    cm3 S = cm3cols(1, 0, 0, 0, 1, 0, 0, 0, 1);
    v3 s = v3make(mod * scale[0], mod * scale[1], mod * scale[2]);
    S.c[0][0] = s.x; S.c[1][1] = s.y; S.c[2][2] = s.z;
    cm3 M = cm3mul(&S, &R);
    /* dSig (col-major, symmetric) magnitudes */
    double dS[3][3] = {{mcov[0], 0.5 * mcov[1], 0.5 * mcov[2]}, {0.5 * mcov[1], mcov[3], 0.5 * mcov[4]},
                       {0.5 * mcov[2], 0.5 * mcov[4], mcov[5]}};
    double dM[3][3];  /* dM = (2M) * dSig, glm order: dM[c][r] = sum_k 2M[k][r] dSig[c][k] */
    for (int c = 0; c < 3; ++c)
        for (int rr = 0; rr < 3; ++rr)
            dM[c][rr] = FA(2.0f * M.c[0][rr]) * dS[c][0] + FA(2.0f * M.c[1][rr]) * dS[c][1] + FA(2.0f * M.c[2][rr]) * dS[c][2];
    /* Rt.c[i][k] = R.c[k][i]; dMt.c[i][k] = dM[k][i] */
    for (int i = 0; i < 3; ++i) mscale[i] = FA(R.c[0][i]) * dM[0][i] + FA(R.c[1][i]) * dM[1][i] + FA(R.c[2][i]) * dM[2][i];
    double D[3][3];
    const double sv[3] = {FA(s.x), FA(s.y), FA(s.z)};
    for (int i = 0; i < 3; ++i)
        for (int k = 0; k < 3; ++k) D[i][k] = dM[k][i] * sv[i];
    mrot[0] = FA(2 * z) * (D[0][1] + D[1][0]) + FA(2 * y) * (D[2][0] + D[0][2]) + FA(2 * x) * (D[1][2] + D[2][1]);
    mrot[1] = FA(2 * y) * (D[1][0] + D[0][1]) + FA(2 * z) * (D[2][0] + D[0][2]) + FA(2 * r) * (D[1][2] + D[2][1]) +
              FA(4 * x) * (D[2][2] + D[1][1]);
    mrot[2] = FA(2 * x) * (D[1][0] + D[0][1]) + FA(2 * r) * (D[2][0] + D[0][2]) + FA(2 * z) * (D[1][2] + D[2][1]) +
              FA(4 * y) * (D[2][2] + D[0][0]);
    mrot[3] = FA(2 * r) * (D[0][1] + D[1][0]) + FA(2 * x) * (D[2][0] + D[0][2]) + FA(2 * y) * (D[1][2] + D[2][1]) +
              FA(4 * z) * (D[1][1] + D[0][0]);
}

/* gauss_chain in absolute arithmetic from magnitudes m9 [P,9] (same layout as g9); outputs as gauss_chain's
 * (dL_dmeans3D [P,3], dL_dcov3D [P,6], dL_dsh [P,M,3], dL_dscales [P,3], dL_drotations [P,4]) in double. */
int go_backward_chain_mag(go_state *st, const go_settings *s, const go_inputs *in, const float *m9, double *m_means3D,
                          double *m_cov3D, double *m_sh, double *m_scales, double *m_rotations) {
    const int P = in->P, M = in->M;
    if (P == 0) return GO_OK;
    memset(m_means3D, 0, 3 * (size_t)P * sizeof(double));
    memset(m_cov3D, 0, 6 * (size_t)P * sizeof(double));
    if (M > 0 && m_sh) memset(m_sh, 0, (size_t)P * M * 3 * sizeof(double));
    memset(m_scales, 0, 3 * (size_t)P * sizeof(double));
    memset(m_rotations, 0, 4 * (size_t)P * sizeof(double));
    const float fy = s->image_height / (2.0f * s->tanfovy);
    const float fx = s->image_width / (2.0f * s->tanfovx);
    const float *proj = s->projmatrix;
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; ++i) {
        if (!(st->radii[i] > 0)) continue;
        const float *g = m9 + 9 * (size_t)i;
        const double mcon[3] = {FA(g[2]), FA(g[3]), FA(g[4])};
        v3 m = v3ld(in->means3D + 3 * (size_t)i);
        const float *cov3 = in->cov3D_precomp ? in->cov3D_precomp + 6 * (size_t)i : st->cov3D + 6 * (size_t)i;
        double mgm[3];
        cov2d_bwd_mag(m, fx, fy, s->tanfovx, s->tanfovy, cov3, s->viewmatrix, mcon, m_cov3D + 6 * (size_t)i, mgm);
        float mh[4];
        xform_point44(m, proj, mh);
        float m_w = 1.0f / (mh[3] + 0.0000001f);
        float mul1 = (proj[0] * m.x + proj[4] * m.y + proj[8] * m.z + proj[12]) * m_w * m_w;
        float mul2 = (proj[1] * m.x + proj[5] * m.y + proj[9] * m.z + proj[13]) * m_w * m_w;
        const double g2x = FA(g[0]), g2y = FA(g[1]);
        mgm[0] += FA(proj[0] * m_w - proj[3] * mul1) * g2x + FA(proj[1] * m_w - proj[3] * mul2) * g2y;
        mgm[1] += FA(proj[4] * m_w - proj[7] * mul1) * g2x + FA(proj[5] * m_w - proj[7] * mul2) * g2y;
        mgm[2] += FA(proj[8] * m_w - proj[11] * mul1) * g2x + FA(proj[9] * m_w - proj[11] * mul2) * g2y;
        if (in->shs && m_sh) {
            const double mcol[3] = {FA(g[6]), FA(g[7]), FA(g[8])};
            double mdir[3];
            sh_bwd_mag(s->sh_degree, m, v3ld(s->campos), in->shs + (size_t)i * M * 3, st->clamped + 3 * (size_t)i,
                       mcol, m_sh + (size_t)i * M * 3, mdir);
            for (int k = 0; k < 3; ++k) mgm[k] += mdir[k];
        }
        for (int k = 0; k < 3; ++k) m_means3D[3 * (size_t)i + k] = mgm[k];
        if (in->scales)
            cov3d_bwd_mag(in->scales + 3 * (size_t)i, s->scale_modifier, in->rotations + 4 * (size_t)i,
                          m_cov3D + 6 * (size_t)i, m_scales + 3 * (size_t)i, m_rotations + 4 * (size_t)i);
    }
    return GO_OK;
}
#undef FA

/* rasterizer_impl.cu:53-63 */
void go_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                     unsigned char *present) {
    (void)projmatrix;
    for (int i = 0; i < P; ++i) {
        v3 pv = xform_point43(v3ld(means3D + 3 * (size_t)i), viewmatrix);
        present[i] = pv.z > 0.2f;
    }
}

/* rasterizer_impl.cu:343-447 + apply_weights.cu:239-356 */
int go_apply_weights(const go_settings *s, const go_inputs *in, int C, const float *image_weights, float *weights,
                     int *cnt) {
    if (C < 1 || C > 3) return GO_ERR_INVALID;
    const int P = in->P, W = s->image_width, H = s->image_height;
    if (P == 0) return GO_OK;
    go_state *st = state_alloc(P, W, H);
    go_inputs in2 = *in;
    in2.colors_precomp = weights; /* the reference passes weights in the colors slot */
    int e = bin_gaussians(st, s, &in2, 0);
    if (e) { go_free(st); return e; }
    double *wacc = (double *)calloc((size_t)P * C, sizeof(double));
    long *cacc = (long *)calloc((size_t)P, sizeof(long));
    const size_t HW = (size_t)W * H;
    const int ntiles = st->gx * st->gy;
    /* sequential over tiles: the accumulation targets are shared */
    for (int t = 0; t < ntiles; ++t) {
        const int tx = t % st->gx, ty = t / st->gx;
        const uint32_t r0 = st->ranges[2 * t], r1 = st->ranges[2 * t + 1];
        for (int yy = 0; yy < TILE_Y; ++yy)
            for (int xx = 0; xx < TILE_X; ++xx) {
                int px = tx * TILE_X + xx, py = ty * TILE_Y + yy;
                if (px >= W || py >= H) continue;
                const size_t pix = (size_t)W * py + px;
                float Cw[3] = {0, 0, 0};
                for (int ch = 0; ch < C; ++ch) Cw[ch] = image_weights[ch * HW + pix];
                float T = 1.0f;
                for (uint32_t k = r0; k < r1; ++k) {
                    uint32_t id = st->point_list[k];
                    float dx = st->means2D[2 * (size_t)id] - (float)px, dy = st->means2D[2 * (size_t)id + 1] - (float)py;
                    const float *co = st->conic_opacity + 4 * (size_t)id;
                    float power = -0.5f * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;
                    if (power > 0.0f) continue;
                    float alpha = fminf(0.99f, co[3] * gs_expf(power));
                    if (alpha < 1.0f / 255.0f) continue;
                    float test_T = T * (1 - alpha);
                    if (test_T < 0.0001f) break;
                    for (int ch = 0; ch < C; ++ch) {
                        wacc[(size_t)id * C + ch] += Cw[ch];
                        cacc[id] += 1;
                    }
                    T = test_T;
                }
            }
    }
    for (size_t j = 0; j < (size_t)P * C; ++j) weights[j] = (float)((double)weights[j] + wacc[j]);
    for (int i = 0; i < P; ++i) cnt[i] += (int)cacc[i];
    free(wacc);
    free(cacc);
    go_free(st);
    return GO_OK;
}

/* Test hook: forward.cu:20-71 for N points (pins the SH path against the
 * reference's own eval_sh). pos/campos -> rgb [N,3] and clamped [N,3]. */
void go_sh_to_rgb(int N, int deg, int M, const float *pos, const float *campos, const float *shs, float *rgb,
                  unsigned char *clamped) {
    for (int i = 0; i < N; ++i)
        sh_to_rgb(deg, M, v3ld(pos + 3 * (size_t)i), v3ld(campos), shs + (size_t)i * M * 3, clamped + 3 * (size_t)i,
                  rgb + 3 * (size_t)i);
}
