/*
 * gs_oracle.h — CPU restatement of the reference 3DGS rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in dge_amd/ links, loads or calls this
 * library: only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg use it, and only as the checker / CPU baseline.
 *
 * It restates, formula by formula, the algorithm of
 *   gaussiansplatting/submodules/diff-gaussian-rasterization/cuda_rasterizer/
 *     forward.cu:20-379, backward.cu:20-557, rasterizer_impl.cu:36-341,
 *     auxiliary.h:18-164, apply_weights.cu:148-356
 * in plain single-precision C (sums over pixels kept in double, which is one
 * admissible order of the reference's float atomics).
 *
 * Parity pinning: see oracle/README.md and DESIGN.md §Oracle (SH evaluation
 * and camera matrices pinned against the reference's own Python functions;
 * image and gradients pinned against an independent PyTorch autograd
 * formulation and known-answer scenes in tests/).
 */
#ifndef GS_ORACLE_H
#define GS_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct go_settings {
    int image_width;
    int image_height;
    float tanfovx;
    float tanfovy;
    float bg[3];
    float scale_modifier;
    float viewmatrix[16]; /* reference layout: column-major view transform */
    float projmatrix[16];
    int sh_degree;
    float campos[3];
    int prefiltered;
} go_settings;

typedef struct go_inputs {
    int P;
    int M;                       /* SH coefficients per channel, 0 when no SH */
    const float *means3D;        /* [P,3] */
    const float *shs;            /* [P,M,3] or NULL */
    const float *colors_precomp; /* [P,3] or NULL */
    const float *opacities;      /* [P] */
    const float *scales;         /* [P,3] or NULL */
    const float *rotations;      /* [P,4] (w,x,y,z) or NULL */
    const float *cov3D_precomp;  /* [P,6] or NULL */
} go_inputs;

typedef struct go_state go_state;

/* Error codes mirror include/gs_raster.h. */
#define GO_OK 0
#define GO_ERR_INVALID 1
#define GO_ERR_PREFILTERED 4

void go_set_threads(int n);
int go_get_threads(void);

/* Forward render.  Outputs: out_color [3,H,W], out_depth [H,W], radii [P].
 * Returns a state (intermediates) that go_backward consumes. */
go_state *go_forward(const go_settings *s, const go_inputs *in, float *out_color, float *out_depth,
                     int *radii, int *num_rendered, int *err);

/* Backward.  All outputs are fully written (no pre-zeroing needed).
 * dL_dconic (optional, [P,4] x,y,_,w as the reference's [P,2,2]).
 * mag9 (optional, [P,9]): per Gaussian, sum over its (pixel, instance) terms of
 * the absolute sub-products of (dL_dmean2D x, y, dL_dconic x, y, w, dL_dopacity,
 * dL_dcolor r, g, b) — the scale a summation-order difference is judged by. */
int go_backward(go_state *st, const go_settings *s, const go_inputs *in, const float *dL_dpix,
                float *dL_dmeans2D, float *dL_dcolors, float *dL_dopacity, float *dL_dmeans3D,
                float *dL_dcov3D, float *dL_dsh, float *dL_dscales, float *dL_drotations,
                float *dL_dconic, float *mag9);

/* The per-Gaussian chain (computeCov2DCUDA + preprocessCUDA bwd) alone, from
 * float rasterizer sums g9 [P,9] = (dL_dmean2D x, y, dL_dconic x, y, w,
 * dL_dopacity, dL_dcolor r, g, b); st from go_forward. */
int go_backward_chain(go_state *st, const go_settings *s, const go_inputs *in, const float *g9,
                      float *dL_dmeans3D, float *dL_dcov3D, float *dL_dsh, float *dL_dscales,
                      float *dL_drotations);

/* The chain in absolute arithmetic (test infrastructure): from per-sum magnitudes m9 [P,9] (the
 * layout of g9, e.g. go_backward's mag9), the magnitude of the terms every chain output is made of,
 * in double (|chain(g)| <= chain_mag(m9) whenever |g| <= m9 elementwise). */
int go_backward_chain_mag(go_state *st, const go_settings *s, const go_inputs *in, const float *m9,
                          double *m_means3D, double *m_cov3D, double *m_sh, double *m_scales, double *m_rotations);

/* The fp64 truth for the per-element gradient bar (gs_truth.c; test infrastructure):
 * go_backward_truth: sums_d [P,9] (layout of g9; NULL: not computed) — backward.cu's per-pixel formulas in double at the float
 * forward's state, summed in double; sums_f [n_orders,P,9] (n_orders <= 4) — the oracle's float per-pixel
 * terms summed in float one by one, as the reference's float atomics add them, in n_orders admissible
 * arrival orders (0: tiles ascending / pixels row-major / entries back to front, 1: its reverse, 2: the
 * even-numbered terms then the odd ones, 3: a seeded pseudo-random permutation).
 * go_backward_chain_f64: the per-Gaussian chain (backward.cu:20-396) in double from double sums, the
 * forward quantities recomputed in double from the float inputs, the decisions the float forward's. */
int go_backward_truth(go_state *st, const go_settings *s, const go_inputs *in, const float *dL_dpix, int n_orders,
                      float *sums_f, double *sums_d);
int go_backward_chain_f64(go_state *st, const go_settings *s, const go_inputs *in, const double *g9,
                          double *dL_dmeans3D, double *dL_dcov3D, double *dL_dsh, double *dL_dscales,
                          double *dL_drotations);

/* Access an intermediate array by name; returns element count or -1. */
long go_state_get(go_state *st, const char *name, void **ptr);
void go_free(go_state *st);

/* rasterizer_impl.cu:53-63 (checkFrustum) */
void go_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                     unsigned char *present);

/* rasterizer_impl.cu:343-447 + apply_weights.cu:148-356.  weights [P,C] is
 * also the colors_precomp input; cnt [P]. C in {1,2,3}. */
int go_apply_weights(const go_settings *s, const go_inputs *in, int C, const float *image_weights,
                     float *weights, int *cnt);

/* forward.cu:20-71 for N points (test hook). */
/* the blend exp (bit-identical to the HIP gs_exp), elementwise */
void go_expf(int n, const float *x, float *y);
void go_sh_to_rgb(int N, int deg, int M, const float *pos, const float *campos, const float *shs, float *rgb,
                  unsigned char *clamped);

#ifdef __cplusplus
}
#endif
#endif
