/*
 * gs_raster.h — C ABI of the MI355X-native differentiable 3D Gaussian
 * Splatting rasterizer (libgs_raster.so, HIP kernels for gfx950).
 *
 * This is the drop-in boundary that replaces the reference's native surface
 * (paths relative to gaussiansplatting/submodules/diff-gaussian-rasterization/):
 *
 *   gs_rasterize_forward   <- _C.rasterize_gaussians            ext.cpp:16
 *                             RasterizeGaussiansCUDA             rasterize_points.cu:35-95
 *                             CudaRasterizer::Rasterizer::forward rasterizer.h:30-57,
 *                                                                rasterizer_impl.cu:179-285
 *   gs_rasterize_backward  <- _C.rasterize_gaussians_backward   ext.cpp:17
 *                             RasterizeGaussiansBackwardCUDA     rasterize_points.cu:97-157
 *                             Rasterizer::backward               rasterizer_impl.cu:289-341
 *   gs_mark_visible        <- _C.mark_visible                   ext.cpp:18
 *                             markVisible / checkFrustum         rasterize_points.cu:159-175,
 *                                                                rasterizer_impl.cu:53-63,128-133
 *   gs_apply_weights       <- _C.apply_weights                  ext.cpp:19
 *                             applyWeightsGaussiansCUDA          rasterize_points.cu:177-234
 *                             Rasterizer::apply_weights          rasterizer_impl.cu:343-447
 *
 * Conventions (identical to the reference's tensors, so a binding passes
 * data_ptr()s straight through):
 *   - every pointer is DEVICE memory unless noted; float32, contiguous;
 *   - means3D [P,3]; shs [P,M,3]; colors_precomp [P,3]; opacities [P];
 *     scales [P,3]; rotations [P,4] as (w,x,y,z); cov3D_precomp [P,6];
 *   - viewmatrix/projmatrix: the reference's 4x4 tensors (row-major memory
 *     holding the column-major transform, auxiliary.h:58-97);
 *   - "absent" inputs are NULL (the reference's empty tensors);
 *   - out_color [3,H,W]; out_depth [1,H,W]; radii [P] int32;
 *   - geometry/binning/image buffers are opaque bytes owned by the caller,
 *     obtained through the gs_alloc_fn callback exactly like the reference's
 *     std::function<char*(size_t)> resize functors (rasterize_points.cu:27-33);
 *     only their round trip from forward to backward is contractual;
 *   - all work is enqueued on `stream` (a hipStream_t); the only host
 *     synchronisation is the read-back of num_rendered, as in the reference
 *     (rasterizer_impl.cu:236-239), whose value the API returns;
 *   - return 0 on success, a GS_ERR_* code otherwise; gs_last_error() holds
 *     the message.  No C++ exception crosses this boundary.
 */
#ifndef GS_RASTER_H
#define GS_RASTER_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GS_RASTER_ABI_VERSION 21

#define GS_OK 0
#define GS_ERR_INVALID_ARG 1   /* AT_ERROR / std::runtime_error in the reference */
#define GS_ERR_HIP 2           /* HIP runtime error (CHECK_CUDA, auxiliary.h:166-173) */
#define GS_ERR_ALLOC 3         /* allocator callback returned NULL */
#define GS_ERR_PREFILTERED 4   /* prefiltered set but a point was culled (auxiliary.h:156-160) */
#define GS_ERR_UNSUPPORTED 5   /* e.g. apply_weights channel count (apply_weights.cu:377-380) */
#define GS_ERR_RETRY 6         /* gs_views_check: a speculative binning capacity was exceeded */

typedef void *gs_stream_t; /* hipStream_t */

/* Allocation callback: returns a device pointer to at least nbytes (16-byte
 * aligned), or NULL.  `which` is 0 = geometry, 1 = binning, 2 = image. */
typedef void *(*gs_alloc_fn)(void *ctx, int which, size_t nbytes);

/* GaussianRasterizationSettings (diff_gaussian_rasterization/__init__.py:228-240). */
typedef struct gs_settings {
    int image_height;
    int image_width;
    float tanfovx;
    float tanfovy;
    const float *bg;         /* device [3] */
    float scale_modifier;
    const float *viewmatrix; /* device [16] */
    const float *projmatrix; /* device [16] */
    int sh_degree;
    const float *campos;     /* device [3] */
    int prefiltered;
    int debug;               /* synchronise + check after every launch */
} gs_settings;

/* Forward render.  Replaces Rasterizer::forward (rasterizer_impl.cu:179-285).
 * M = SH coefficients per channel (shs.size(1)), 0 when shs is NULL. */
int gs_rasterize_forward(const gs_settings *s, int P, int M, const float *means3D, const float *shs,
                         const float *colors_precomp, const float *opacities, const float *scales,
                         const float *rotations, const float *cov3D_precomp, float *out_color,
                         float *out_depth, int *radii, gs_alloc_fn alloc, void *alloc_ctx,
                         gs_stream_t stream, int *num_rendered);

/* Backward.  Replaces Rasterizer::backward (rasterizer_impl.cu:289-341).
 * R = num_rendered from the forward.  Every output is fully written (the
 * caller need not zero it): dL_dmeans2D [P,3] (z = 0), dL_dcolors [P,3],
 * dL_dopacity [P], dL_dmeans3D [P,3], dL_dcov3D [P,6], dL_dsh [P,M,3]
 * (may be NULL when M == 0), dL_dscales [P,3], dL_drotations [P,4].
 * The backward writes scratch inside the forward's geometry/binning/image
 * buffers (gradient records and flags, the live list, counters): calls for ONE
 * forward must be ordered (same stream, or the later one waits for the earlier
 * one); calls for different forwards may run concurrently. */
int gs_rasterize_backward(const gs_settings *s, int P, int M, int R, const float *means3D,
                          const float *shs, const float *colors_precomp, const float *scales,
                          const float *rotations, const float *cov3D_precomp, const int *radii,
                          const void *geom_buffer, const void *binning_buffer, const void *img_buffer,
                          const float *dL_dpix, float *dL_dmeans2D, float *dL_dcolors,
                          float *dL_dopacity, float *dL_dmeans3D, float *dL_dcov3D, float *dL_dsh,
                          float *dL_dscales, float *dL_drotations, gs_stream_t stream);

/* Extended entry points.  gs_params describes the Gaussians with split SH
 * storage and optional in-kernel activations, so a GaussianModel's raw
 * parameters (gaussian_model.py:42-57, 221-258: _xyz, _features_dc,
 * _features_rest, _opacity, _scaling, _rotation) are consumed in place: no
 * torch.cat of the SH, no separate sigmoid/exp/normalize kernels, and the
 * backward returns gradients w.r.t. those raw tensors.  The reference-shaped
 * gs_rasterize_forward/backward above are thin wrappers over these. */
typedef struct gs_params {
    int P;
    int M;                        /* SH coefficients per channel, 0 when no SH */
    const float *means3D;         /* [P,3] */
    const float *sh_dc;           /* coefficient 0 of Gaussian i at sh_dc + i*sh_dc_stride (x3 floats) */
    const float *sh_rest;         /* coefficient k>=1 at sh_rest + i*sh_rest_stride + 3*(k-1) */
    int sh_dc_stride;             /* in floats; [P,M,3] SH: dc = shs, rest = shs + 3, both strides 3*M */
    int sh_rest_stride;
    const float *colors_precomp;  /* [P,3] or NULL */
    const float *opacities;       /* [P] */
    const float *scales;          /* [P,3] or NULL */
    const float *rotations;       /* [P,4] or NULL */
    const float *cov3D_precomp;   /* [P,6] or NULL */
    int activation;               /* 0: values used as given (the reference's contract);
                                     1: raw parameters: opacity = sigmoid(x), scale = exp(x),
                                        rotation = x / max(|x|, 1e-12) (F.normalize) */
    int sh_half;                  /* 1: sh_dc / sh_rest hold IEEE fp16 values (strides in elements),
                                     upcast in-kernel (the local-edit path's fp16 SH storage);
                                     the SH gradients stay fp32 */
    const int *index;             /* NULL, or [P] ascending rows: Gaussian i of the render is row
                                     index[i] of means3D/sh/opacities/scales/rotations/cov3D_precomp
                                     (the GaussianModel's `localize` subset pc[mask], gathered
                                     in-kernel).  The backward then writes the parameter-shaped
                                     gradients (means3D, sh, opacity, scales, rotations, cov3D) at
                                     those rows only; means2D / colors / radii stay [P]. */
    uint8_t *visible_out;         /* forward only: NULL, or [P] bytes set to (radii > 0) — render()'s
                                     visibility_filter as a bool tensor, without a separate pass */
    int forward_only;             /* forward only: 1 = no backward will follow (a render without autograd,
                                     e.g. torch.no_grad): the binning and blend skip the backward's
                                     scratch (gradient-record flags, checkpoints, blended bits, the
                                     replay's work list, the touched bytes) and the binning buffer
                                     leaves it out; a backward of such a forward is an error */
    const uint8_t *aux_mask;      /* NULL, or [P] bytes 0/1 (a bool tensor; row index[i] with `index`): a
                                     forward with backward bookkeeping also composites these values as a
                                     grey colour along the same alpha / transmittance chain and keeps the
                                     result in its image buffer — the image a recolor render with
                                     colors[i] = (m_i, m_i, m_i) gives, which gs_render_recolor then serves
                                     without a second blend (DGE renders the edit mask of each view right
                                     after its training render, threestudio/systems/DGE.py:198-204) (ABI 18) */
} gs_params;

/* gs_grads.accumulate bits: output i is ADDED to (out += grad) instead of
 * overwritten — fused gradient accumulation into existing .grad buffers. */
#define GS_ACC_MEANS2D   (1u << 0)
#define GS_ACC_COLORS    (1u << 1)
#define GS_ACC_OPACITY   (1u << 2)
#define GS_ACC_MEANS3D   (1u << 3)
#define GS_ACC_COV3D     (1u << 4)
#define GS_ACC_SH        (1u << 5)   /* dL_dsh_dc and dL_dsh_rest */
#define GS_ACC_SCALES    (1u << 7)
#define GS_ACC_ROTATIONS (1u << 8)

typedef struct gs_grads {         /* backward outputs, every element written */
    float *dL_dmeans2D;           /* [P,3], z = 0 */
    float *dL_dcolors;            /* [P,3]; may be NULL in the _ex entry point (not written) */
    float *dL_dopacity;           /* [P] (w.r.t. the raw opacity when activation = 1) */
    float *dL_dmeans3D;           /* [P,3] */
    float *dL_dcov3D;             /* [P,6] or NULL */
    float *dL_dsh_dc;             /* same addressing as gs_params.sh_dc, or NULL */
    float *dL_dsh_rest;
    int dsh_dc_stride;
    int dsh_rest_stride;
    float *dL_dscales;            /* [P,3] (raw when activation = 1) */
    float *dL_drotations;         /* [P,4] (raw when activation = 1) */
    unsigned int accumulate;      /* GS_ACC_* bits; 0: overwrite every output (reference behaviour) */
    /* Optional per-Gaussian gradient mask (the GaussianModel's grad-mask hooks,
     * gaussian_model.py:837-856: grad * mask[:, None]): outputs whose GS_ACC_*
     * bit is set in mask_bits are multiplied by grad_mask[i] (0/1; grad_mask[index[i]] with
     * gs_params.index); NULL: none. */
    const uint8_t *grad_mask;     /* [P] */
    unsigned int mask_bits;
    /* Optional [P,3] output (not in the reference's API; parity tests): each
     * Gaussian's summed conic gradient (x, y, w of backward.cu's dL_dconic2D),
     * the input of the per-Gaussian chain; NULL: not written. */
    float *dL_dconic;
    /* Optional hipEvent_t (NULL: none): the stream waits for it right before
     * the first write of an ACCUMULATED output (the per-Gaussian pass), not
     * before the gradient replay.  Backward calls of different views that add
     * into the same .grad buffers from different streams are ordered by it
     * while the replay of one overlaps the per-Gaussian pass of the other. */
    void *writes_after;
    /* GS_ACC_* bits of accumulated outputs that hold exactly zero for every
     * Gaussian before this call (the caller cleared them this step, e.g. a
     * gradient bucket filled with zeros): the first write this call makes for
     * a Gaussian stores its gradient instead of adding it, so the zeros are
     * never read.  gs_views_backward honours view 0's bits for the batch: the
     * first view that has a Gaussian live stores, later views add.  0: plain
     * accumulation (ABI 12). */
    unsigned int zeroed;
    /* Row pitches (in floats) of the parameter-shaped outputs: element (i, c) of dL_dmeans3D at
     * dL_dmeans3D[i * pitch_means3D + c], likewise dL_dopacity, dL_dscales, dL_drotations; 0 = the
     * reference's packed [P,3] / [P] / [P,3] / [P,4].  With dsh_dc_stride / dsh_rest_stride they let every
     * parameter gradient of a Gaussian live in ONE row of a row-major gradient bucket (the .grad tensors
     * then strided views of it: dge_amd.multiview.GradBucket), so the per-Gaussian pass reads and writes
     * two cache lines per live Gaussian instead of one or two in each of six arrays.  dL_drotations rows
     * must stay 16-byte aligned (pitch a multiple of 4).  (ABI 17) */
    int pitch_means3D, pitch_opacity, pitch_scales, pitch_rotations;
    /* Optional [rows] bytes (NULL: none): set to 1 at the parameter row of every Gaussian whose
     * accumulated gradients this call may write — a row-major gradient bucket's record of its nonzero rows,
     * so its next clear zeroes only those (gs_rows_zero_dirty).  gs_views_backward / _passes take view 0's.
     * (ABI 19) */
    uint8_t *dirty_rows;
} gs_grads;

int gs_rasterize_forward_ex(const gs_settings *s, const gs_params *g, float *out_color, float *out_depth,
                            int *radii, gs_alloc_fn alloc, void *alloc_ctx, gs_stream_t stream,
                            int *num_rendered);
/* gs_rasterize_forward_ex in two halves, so a caller rendering several views
 * can enqueue every view's first half before it waits for any instance count
 * (the reference's one host sync per forward, rasterizer_impl.cu:236-239:
 * num_rendered sizes the binning buffer).
 *   _begin: allocates the geometry/image buffers (alloc which = 0, 2) and
 *           enqueues the preprocess, the counter read-back, the depth sort and
 *           the instance scan; *state receives an opaque handle.  Does not wait.
 *   _end:   waits for that view's instance count, allocates the binning buffer
 *           (which = 1), enqueues the rest and writes out_color/out_depth;
 *           always consumes the handle (also on error).  `stream` must be the
 *           begin stream or one ordered after it.
 *   _release: drops a handle that will not be ended.
 * The inputs named by s and g must stay valid and unmodified until _end. */
typedef struct gs_forward_state gs_forward_state;
int gs_rasterize_forward_begin(const gs_settings *s, const gs_params *g, int *radii, gs_alloc_fn alloc,
                               void *alloc_ctx, gs_stream_t stream, gs_forward_state **state);
int gs_rasterize_forward_end(gs_forward_state *state, float *out_color, float *out_depth, gs_alloc_fn alloc,
                             void *alloc_ctx, gs_stream_t stream, int *num_rendered);
void gs_rasterize_forward_release(gs_forward_state *state);

/* The same render with other colours: the forward-only blend over a finished
 * raw-parameter or precomputed-colour forward's buffers (geom/binning/img of
 * num_rendered instances, a forward WITH backward bookkeeping — not
 * forward_only), the Gaussians' colours replaced by colors [P,3] (the
 * colors_precomp of rasterize_points.cu:45 — DGE's semantic render,
 * threestudio/systems/DGE.py:198-204, uses the same camera and Gaussians as
 * the training render just before it, so their preprocess, depth order and
 * tile lists are identical and only the blend differs).  out_color/out_depth
 * are bit-identical to a full forward with colors_precomp = colors; img_out
 * (gs_image_buffer_size) receives that blend's per-pixel state (final T,
 * n_contrib, the tile / quadrant windows) when the blend runs, and is scratch
 * whose per-pixel state is UNDEFINED when the aux match below serves the image
 * (only out_color / out_depth are written then); the source buffers are only
 * read.  s must describe the source forward (image size, grid); its bg is the
 * one blended.  Enqueued on `stream`, which must be ordered after the source
 * forward.  src_aux_mask: NULL, or the gs_params.aux_mask the source forward
 * composited (the same bytes, unchanged since), addressed like colors: byte i
 * belongs to colors[i].  It is unsupported with a source forward that used
 * gs_params.index (that forward read aux_mask[index[i]]); pass NULL there, or
 * the mask gathered by the index.  Where colors holds exactly (m_i, m_i, m_i)
 * for every Gaussian (checked on the device, bit for bit) the image is composed
 * from that forward's grey sum and transmittance instead of blended again — the
 * same bits; otherwise the blend runs (ABI 18). */
int gs_render_recolor(const gs_settings *s, int P, int num_rendered, const void *geom_buffer,
                      const void *binning_buffer, const void *img_buffer, const float *colors, void *img_out,
                      float *out_color, float *out_depth, const uint8_t *src_aux_mask, gs_stream_t stream);
int gs_rasterize_backward_ex(const gs_settings *s, const gs_params *g, int R, const int *radii,
                             const void *geom_buffer, const void *binning_buffer, const void *img_buffer,
                             const float *dL_dpix, const gs_grads *out, gs_stream_t stream);
/* gs_rasterize_backward_ex in its two halves, for a caller that defers the per-Gaussian passes of several
 * views' backwards to the end of one autograd backward (DGE's loop renders its views one by one and
 * backpropagates their stacked loss once, threestudio/systems/DGE.py:179-222, 672):
 *   _replay: the gradient replay of one view (its per-(slot, quadrant) records, kept in that view's
 *            binning buffer); the arguments are the ones gs_rasterize_backward_ex would get;
 *   _passes: the per-Gaussian passes of n replayed views, in view order — ONE merged pass (the one
 *            gs_views_backward runs) when the views render one scene into the same gradient outputs and
 *            every view after the first accumulates (GS_ACC_*) into all of them, else one pass per view.
 *            out[0]->writes_after orders the first accumulated write.  `stream` must be ordered after
 *            every view's replay.  Bitwise the per-view gs_rasterize_backward_ex calls in that order.
 * (ABI 18) */
int gs_rasterize_backward_replay(const gs_settings *s, const gs_params *g, int R, const int *radii,
                                 const void *geom_buffer, const void *binning_buffer, const void *img_buffer,
                                 const float *dL_dpix, const gs_grads *out, gs_stream_t stream);
int gs_rasterize_backward_passes(int n, const gs_settings *const *s, const gs_params *const *g, const int *R,
                                 const int *const *radii, const void *const *geom_buffer,
                                 const void *const *binning_buffer, const gs_grads *const *out, gs_stream_t stream);

/* A batch of views of ONE scene (DGE renders a batch of edited views per step,
 * threestudio/systems/DGE.py:170-239): view v on streams[v], its outputs
 * out_color[v] [3,H,W], out_depth[v] [1,H,W], radii[v] [P] (and
 * g[v]->visible_out).  Every view's first half (preprocess, depth sort,
 * instance scan) is enqueued before any view's second half.
 *   mode GS_VIEWS_EXACT: each view's second half waits for its instance count
 *     (the reference's host sync, rasterizer_impl.cu:236-239) and sizes its
 *     binning buffer exactly (alloc which = 16 + v);
 *   mode GS_VIEWS_SPECULATE: a view whose (P, W, H) this library has rendered
 *     before gets a binning buffer of 1.25 x the largest count seen + 64k
 *     instances; its emission, tile sort and blend read the count on the
 *     device and no host wait happens.  gs_views_check then reads the counts:
 *     GS_ERR_RETRY means some view exceeded its capacity (its outputs and any
 *     backward of it are invalid; a second forward of the batch fits, the
 *     capacity having grown).  Views without history are rendered exactly.
 * All buffers but the exact binning ones come from ONE alloc(alloc_ctx, 0, bytes).
 * join: the caller's stream (a null handle is the legacy default stream) — the
 * views' streams start after its work so far, and it waits for all of the
 * views' work before the call returns. 
 * The outputs of a speculated batch are bit-identical to the exact ones when
 * gs_views_check returns GS_OK. */
#define GS_MAX_VIEWS 8
#define GS_VIEWS_EXACT 0
#define GS_VIEWS_SPECULATE 1
typedef struct gs_views gs_views;
int gs_views_forward(int n, const gs_settings *const *s, const gs_params *const *g, float *const *out_color,
                     float *const *out_depth, int *const *radii, int mode, gs_alloc_fn alloc, void *alloc_ctx,
                     const gs_stream_t *streams, gs_stream_t join, gs_views **out);
/* Waits for the speculated views' counts (already on the host for exact ones);
 * num_rendered [n] (optional) receives them.  GS_OK, GS_ERR_RETRY, GS_ERR_PREFILTERED. */
int gs_views_check(gs_views *h, int *num_rendered);
/* The backward of every view, view v on streams[v] with grads[v] (dL_dmeans2D
 * per view; the parameter gradients usually shared, GS_ACC_* set from the
 * second view on).  Each view's gradient replay runs on its stream; when the
 * views share their parameter-gradient outputs, ONE per-Gaussian pass on
 * streams[0] then adds every view's gradients in view order (else the views'
 * passes are chained in view order) — the first write after `writes_after`,
 * an optional hipEvent_t — so accumulated gradients add up in a fixed order,
 * bitwise those of per-view calls; `join` (the caller's stream, null = the
 * legacy default stream): the views start after its work so far (the image
 * gradients) and it waits for all of them. */
int gs_views_backward(gs_views *h, const float *const *dL_dpix, const gs_grads *const *grads,
                      const gs_stream_t *streams, void *writes_after, gs_stream_t join);
/* View v's buffers (which: 0 geometry, 1 binning, 2 image; gs_buffer_offset
 * addresses their fields with num_rendered = gs_views_layout(h, v)). */
/* flag[0] (one device byte) = 1 when some speculated view of the batch overflowed its capacity (or
 * needs the 32-bit depth sort) — gs_views_check's GS_ERR_RETRY decision, computed on the device on
 * `stream` (which must be ordered after the views' forwards) without a host wait, so a collective can
 * carry it: every rank of a view-sharded step then agrees on the recovery (ABI 14). */
int gs_views_overflow(const gs_views *h, uint8_t *flag, gs_stream_t stream);
void *gs_views_buffer(const gs_views *h, int v, int which);
long long gs_views_layout(const gs_views *h, int v);
void gs_views_release(gs_views *h);

/* present[i] = (view * means3D[i]).z > 0.2 (rasterizer_impl.cu:53-63). */
int gs_mark_visible(int P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                    uint8_t *present, gs_stream_t stream);

/* Back-projection of image weights onto Gaussians (apply_weights.cu:148-356).
 * weights [P,C] (also the colors_precomp input, as in the reference) and
 * cnt [P] int32 are accumulated in place; C = num_channels in {1,2,3}. */
int gs_apply_weights(const gs_settings *s, int P, int M, const float *means3D, float *weights,
                     int num_channels, const float *opacities, const float *scales,
                     const float *rotations, const float *cov3D_precomp, const float *shs,
                     const float *image_weights, int *cnt, gs_alloc_fn alloc, void *alloc_ctx,
                     gs_stream_t stream);

/* Fused Adam step over several parameter tensors in ONE launch — the
 * optimizer of the training loop (gaussian_model.py:336-380:
 * torch.optim.Adam(groups, lr=0.0, eps=1e-15), one group per parameter;
 * the float32 operation order of torch's foreach Adam on the GPU).  Per
 * segment the caller passes the group's step scalars (its own step count):
 * step_size = lr / (1 - beta1^t), bias_correction2_sqrt = sqrt(1 - beta2^t).
 * beta1/beta2 are doubles, as torch's Python floats: 1 - beta is formed in
 * double before the one rounding to float (ABI 7; a float beta rounds twice).
 * param, exp_avg, exp_avg_sq are updated in place; grad is read. */
#define GS_ADAM_MAX_SEGMENTS 8    /* per launch; longer lists take several */
typedef struct gs_adam_segment {
    float *param;
    const float *grad;
    float *exp_avg;
    float *exp_avg_sq;
    long long n;                  /* elements */
    float step_size;
    float bias_correction2_sqrt;
    /* grad's rows (ABI 17): element e at grad[(e / grad_width) * grad_pitch + e % grad_width] — a .grad
     * that is a column block of a row-major gradient bucket; grad_pitch 0: packed like param */
    int grad_width;
    int grad_pitch;
} gs_adam_segment;
int gs_adam_step(const gs_adam_segment *segs, int nseg, double beta1, double beta2, float eps,
                 gs_stream_t stream);

/* Sparse-row gradient exchange of the multi-view step (not in the reference,
 * whose loop is single-GPU: threestudio/systems/DGE.py:170-296 sums the views'
 * gradients in one process).  dge_amd/multiview.py GradBucket all-reduces only
 * the rows that are nonzero on some rank.  A bucket is up to
 * GS_ROWS_MAX_REGIONS row-major fp32 matrices sharing the row count (a
 * GaussianModel's six .grad tensors: 3 + 3 + 45 + 1 + 3 + 4 floats per row). */
#define GS_ROWS_MAX_REGIONS 8
typedef struct gs_rows_region {
    float *base;                  /* [n, width] row-major, rows `pitch` floats apart */
    int width;
    int pitch;                    /* 0: width (dense rows); else >= width (a column block of a wider row,
                                   * e.g. the 59 used columns of a 64-float bucket row: ABI 21) */
} gs_rows_region;
/* live[r] = 1 if row r of some region holds an element != 0 (NaN included) in its first `width`
 * columns, else 0. */
int gs_rows_live(const gs_rows_region *regions, int nreg, long long n, uint8_t *live, gs_stream_t stream);
/* packed[i, :] = row rows[i] of region 0, then of region 1, ... (m x sum(width)). */
int gs_rows_gather(const gs_rows_region *regions, int nreg, const long long *rows, long long m, float *packed,
                   gs_stream_t stream);
/* the inverse: row rows[i] of every region = its columns of packed[i, :]. */
int gs_rows_scatter(const gs_rows_region *regions, int nreg, const long long *rows, long long m,
                    const float *packed, gs_stream_t stream);
/* rows[0..count) = the ascending indices r < n with live[r] != 0, count_scratch[0] = count (int64),
 * with no host round trip (the sparse all-reduce's union of live rows, agreed on before the backward
 * runs: dge_amd/multiview.py GradBucket.allreduce_begin).  count_scratch holds 1 + ceil(n / 1024)
 * int64 (the rest is scratch); rows holds up to n. */
int gs_rows_compact(const uint8_t *live, long long n, long long *rows, long long *count_scratch, gs_stream_t stream);
/* gs_rows_gather / _scatter over a packed buffer of `cap` rows whose row list holds *count rows, the
 * count read on the device (gs_rows_compact's count_scratch[0]): the gather zero-fills the packed rows
 * past min(cap, *count), the scatter moves only the first min(cap, *count) — a collective shaped by a
 * capacity instead of a host read of the count (ABI 13); rows past the capacity are the caller's. */
int gs_rows_gather_dev(const gs_rows_region *regions, int nreg, const long long *rows, long long cap,
                       const long long *count, float *packed, gs_stream_t stream);
int gs_rows_scatter_dev(const gs_rows_region *regions, int nreg, const long long *rows, long long cap,
                        const long long *count, const float *packed, gs_stream_t stream);

/* rows[r * pitch + c] = 0 for c < width and every r < n with dirty[r] != 0, then dirty[r] = 0: the clear of a
 * row-major gradient bucket whose written rows the backward recorded (gs_grads.dirty_rows) — at c2 ~7% of
 * the rows instead of a 256 MB fill.  rows 16-B aligned, pitch and width multiples of 4 (ABI 19). */
int gs_rows_zero_dirty(float *rows, long long pitch, int width, uint8_t *dirty, long long n, gs_stream_t stream);
/* dirty[rows[i]] = 1 for i < m (count: NULL, or m read on the device as min(m, *count)): the rows a sparse
 * all-reduce's scatter wrote (ABI 19). */
int gs_rows_mark_dirty(uint8_t *dirty, const long long *rows, long long m, const long long *count, gs_stream_t stream);

/* Byte sizes of the opaque buffers (host arithmetic, no device work). */
size_t gs_geometry_buffer_size(int P);
size_t gs_image_buffer_size(int width, int height);
size_t gs_binning_buffer_size(int num_rendered, int num_tiles);

/* Offsets (bytes) of the per-Gaussian arrays inside the geometry buffer, for
 * field-by-field parity tests.  Names: "splat" (64-B records: "means2D" float2
 * at +0, "conic_opacity" float4 at +16, "rgbd" float4 = r,g,b,depth at +32 — the depth negated for
 * the Gaussians a forward's gs_params.aux_mask marks: the blend's aux bit, |depth| is the depth),
 * "tiles_touched" (u32), "clamped" (u8, bit c = channel c clamped), "radii"
 * (int32; a copy of the caller's radii, kept only when the caller passes none
 * or the tile grid exceeds 255 x 255).
 * Image buffer: "final_T" (float), "n_contrib" (u32), "ranges" (uint2 per tile).
 * Binning buffer: "point_list" (u32 per instance).  Returns -1 if unknown. */
long long gs_buffer_offset(const char *buffer, const char *field, int P, int width, int height,
                           int num_rendered);

/* Stage profiler (bench / diagnostics): when enabled, every stage of the
 * calls made on this host thread is bracketed by HIP events on its stream.
 * gs_profile_collect synchronises on the recorded events, writes the summed
 * milliseconds and launch counts per stage (n entries) and resets. */
int gs_profile_enable(int on);
/* Restrict the profiler to the stages whose bit (1 << stage index) is set
 * (default: all): every bracketed stage costs two events on the stream. */
int gs_profile_set_stages(unsigned int mask);
int gs_profile_num_stages(void);
const char *gs_profile_stage_name(int i);
int gs_profile_collect(double *total_ms, int *counts, int n);
/* Host time (ns, process total since load) the forward's second half spent
 * blocked on its instance-count read-back (the reference's one host sync,
 * rasterizer_impl.cu:236-239): the bench reports it per step. */
long long gs_host_wait_ns(void);

/* Blend-kernel diagnostics: when enabled, the forward blend and the backward
 * replay record per wave (8 u64) {start, end (s_memrealtime, 100 MHz), kept
 * entries, rounds, cycles inside the blend/replay loops, total cycles
 * (s_memtime), 0, 0}; gs_profile_diag_read copies the last launch's records
 * (which: 0 forward, 1 backward, 2 the per-Gaussian backward's phase stamps) to host memory and
 * returns the u64 count. */
int gs_profile_diag_enable(int on);
long long gs_profile_diag_read(int which, uint64_t *host, long long max_u64);

/* Step timer (bench.py's per-step GPU times): timing events without the system-scope fence — a record is a
 * marker in the stream's queue that writes back nothing for the host (a fenced one flushes the L2 the step's
 * gradient writes just dirtied).  gs_timer_elapsed_ms waits for `end`.  (Not in the reference's API; ABI 20.) */
int gs_timer_create(void **event);
int gs_timer_record(void *event, gs_stream_t stream);
int gs_timer_elapsed_ms(void *start, void *end, float *ms);
int gs_timer_destroy(void *event);

/* Test hook: the blend's exp (forward.cu:345 `exp(power)`) over n floats on the
 * device, evaluated exactly as the blend kernels do (packed pairs); bit-identical
 * to the oracle's gs_expf.  Returns GS_OK or an error code. */
int gs_blend_exp(long long n, const float *x, float *y, gs_stream_t stream);

/* Test hook: the raw-parameter activations the fused path applies in-kernel
 * (gs_params.activation; gaussian_model.py:42-57 get_opacity / get_scaling /
 * get_rotation: sigmoid, exp, F.normalize), over P rows on the device with the
 * preprocess's own device functions — what the oracle must be given to see the
 * values the kernels used.  Any output may be NULL (its input is then not read). */
int gs_activate_params(int P, const float *raw_opacity, const float *raw_scaling, const float *raw_rotation,
                       float *opacity, float *scaling, float *rotation, gs_stream_t stream);

const char *gs_last_error(void);
int gs_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* GS_RASTER_H */
