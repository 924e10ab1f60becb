/*
 * gs_oracle_internal.h — the oracle's state, shared by its translation units (gs_oracle.c, gs_truth.c).
 * TEST INFRASTRUCTURE ONLY (see gs_oracle.h).
 */
#ifndef GS_ORACLE_INTERNAL_H
#define GS_ORACLE_INTERNAL_H

#include <stddef.h>
#include <stdint.h>

#include "gs_oracle.h"

/* The oracle is built three times (oracle/Makefile): without contraction (liboracle.so, the model every
 * bit-exact comparison uses) and with a*b+c contracted to fma by gcc and by clang (liboracle_fma_gcc.so,
 * liboracle_fma_clang.so: two admissible models of nvcc's default -fmad=true, used only as further fp32
 * evaluations of the backward for the fp64-truth bar).  GO_EXACT marks the code whose results must not depend
 * on the build — the blend exp, the alpha test and the EWA setup, i.e. every decision the backward takes
 * from the forward — so a contracted build's backward takes the forward's decisions on its state. */
#if defined(__clang__)
#define GO_EXACT
#define GO_EXACT_BODY _Pragma("clang fp contract(off)")
#else
#define GO_EXACT __attribute__((optimize("fp-contract=off")))
#define GO_EXACT_BODY
#endif

#define TILE_X 16
#define TILE_Y 16

struct go_state {
    int P, W, H, gx, gy, K;
    float *depths;         /* P */
    unsigned char *clamped; /* 3P */
    int *radii;            /* P */
    float *means2D;        /* 2P */
    float *cov3D;          /* 6P */
    float *conic_opacity;  /* 4P */
    float *rgb;            /* 3P */
    uint32_t *tiles_touched; /* P */
    uint32_t *point_offsets; /* P, inclusive scan */
    uint64_t *point_keys;    /* K sorted */
    uint32_t *point_list;    /* K sorted */
    uint32_t *ranges;        /* 2 * tiles */
    float *final_T;          /* HW */
    uint32_t *n_contrib;     /* HW */
    uint32_t *n_visited;     /* HW: list entries visited before stopping (diagnostic) */
    const float *features;   /* rgb or colors_precomp (borrowed) */
};

/* (pixel, instance) gradient terms of the backward as the oracle's float arithmetic computes them */
typedef struct go_emit {
    uint32_t *ids;  /* Gaussian of each term set */
    float *terms;   /* 9 floats per set: (dL_dmean2D x, y, dL_dconic x, y, w, dL_dopacity, dL_dcolor r, g, b) */
    size_t n, cap;
} go_emit;

/* the alpha test of forward.cu:336-348 / backward.cu:491-501 on the float state: 1 when the entry is blended
 * at a pixel the forward reached (power <= 0, alpha >= 1/255), with G and alpha */
int go_pixel_alpha(const float *conic_opacity, float dx, float dy, float *G, float *alpha);
/* the blend exp (gs_oracle.c gs_expf), one value */
float go_expf1(float x);
/* render_pixel_bwd of gs_oracle.c for one pixel, appending its float terms to em (no sums) */
void go_render_pixel_terms(const go_state *st, const float *colors, const float *bg, const float *dL_dpix, int tile,
                           int px, int py, go_emit *em);

#endif
