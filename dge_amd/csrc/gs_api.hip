// gs_api.hip — the C ABI (include/gs_raster.h): host orchestration of the
// gfx950 kernels.  Replaces CudaRasterizer::Rasterizer::{forward, backward,
// markVisible, apply_weights} (rasterizer_impl.cu:128-447) and the tensor glue
// of rasterize_points.cu:35-234.
//
// Forward stream order (one stream, no device-wide sync):
//   memset(counters, ranges, tile_last)
//   k_preprocess                      -> geometry + depth keys + instance total
//   D2H copy of {total, error} into pinned memory, event
//   depth radix sort (4 x 8-bit passes over P keys)
//   instance scan in depth order (reduce + top)
//   --- host waits on the event only (the sort keeps the GPU busy) ---
//   binning buffer allocation (caller's allocator, e.g. the torch caching allocator)
//   k_scan_emit                       -> (tile, slot) instances, depth-ordered
//   tile radix sort (1 pass up to 2048 tiles)
//   k_ranges                          -> ranges (the per-tile lists come out of the tile sort)
//   k_render_fwd                      -> color, depth, final_T, n_contrib, tile_last
#include <stdarg.h>
#include <stdlib.h>
#include <stdio.h>
#include <string.h>

#include <limits>
#include <memory>
#include <atomic>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "gs_common.h"
#include "gs_internal.h"
#include "gs_raster.h"

using namespace gs;

namespace {

thread_local std::string g_last_error;

int set_error(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define GS_HIP(call)                                                                                  \
    do {                                                                                              \
        hipError_t e_ = (call);                                                                       \
        if (e_ != hipSuccess) return set_error(GS_ERR_HIP, "%s failed: %s", #call, hipGetErrorString(e_)); \
    } while (0)

// after a launch: surface launch errors; in debug mode also synchronise
// (the reference's CHECK_CUDA, auxiliary.h:166-173)
#define GS_LAUNCHED(what)                                                                                     \
    do {                                                                                                      \
        hipError_t e_ = hipGetLastError();                                                                    \
        if (e_ != hipSuccess) return set_error(GS_ERR_HIP, "%s launch failed: %s", what, hipGetErrorString(e_)); \
        if (debug) {                                                                                          \
            e_ = hipStreamSynchronize(stream);                                                                \
            if (e_ != hipSuccess) return set_error(GS_ERR_HIP, "%s failed: %s", what, hipGetErrorString(e_)); \
        }                                                                                                     \
    } while (0)

// Per-(thread, device) pinned staging word + event for the num_rendered read-back.
// DGE_AMD_DEPTH_KEYS32=1 forces the 32-bit depth-key fallback (tests compare both orders)
bool force_depth_keys32() {
    const char* e = getenv("DGE_AMD_DEPTH_KEYS32");
    return e && e[0] == '1';
}

// DGE_AMD_TILE_SORT=2pass: the emission + two full tile-sort passes + k_ranges even where the
// two-level binning applies (tests compare both; read per forward)
bool tile_sort_unfused() {
    const char* e = getenv("DGE_AMD_TILE_SORT");
    return e && !strcmp(e, "2pass");
}

// depth-sort bits (three passes of kDepthPassBits; DGE_AMD_DEPTH_SORT_BITS overrides, for probes)
int depth_sort_bits() {
    static const int bits = [] {
        const char* e = getenv("DGE_AMD_DEPTH_SORT_BITS");
        const int b = e ? atoi(e) : 0;
        return (b >= 3 && b <= 30) ? b : kDepthSortBits;
    }();
    return bits;
}

// per-pass digit bits of the depth sort (DGE_AMD_DEPTH_PASS_BITS overrides; negative: low passes of
// that width, the remainder in the last)
int depth_pass_bits() {
    static const int bits = [] {
        const char* e = getenv("DGE_AMD_DEPTH_PASS_BITS");
        const int b = e ? atoi(e) : 0;
        return (b != 0 && b >= -10 && b <= 11) ? b : kDepthPassBits;
    }();
    return bits;
}

// Pinned read-back slot of one forward's preprocess counters + its event.  A
// pool per device: several forwards may be between begin and end at once
// (gs_rasterize_forward_begin / _end), each holding its own slot.
struct Staging {
    uint32_t* host = nullptr;
    hipEvent_t ev = nullptr;
    int dev = 0;
};
struct StagingPool {
    std::mutex mu;
    std::unordered_map<int, std::vector<Staging*>> free;
};
StagingPool& staging_pool() {
    static StagingPool p;
    return p;
}

int staging_acquire(Staging** out) {
    int dev = 0;
    GS_HIP(hipGetDevice(&dev));
    StagingPool& p = staging_pool();
    {
        std::lock_guard<std::mutex> g(p.mu);
        std::vector<Staging*>& v = p.free[dev];
        if (!v.empty()) {
            *out = v.back();
            v.pop_back();
            return GS_OK;
        }
    }
    Staging* s = new Staging();
    s->dev = dev;
    if (hipHostMalloc((void**)&s->host, 4 * kCounterSlots * kCounterStride, hipHostMallocDefault) != hipSuccess ||
        hipEventCreateWithFlags(&s->ev, hipEventDisableTiming) != hipSuccess) {
        delete s;
        return set_error(GS_ERR_HIP, "could not create the counter read-back slot");
    }
    *out = s;
    return GS_OK;
}

void staging_release(Staging* s) {
    if (!s) return;
    StagingPool& p = staging_pool();
    std::lock_guard<std::mutex> g(p.mu);
    p.free[s->dev].push_back(s);
}

// ---------------------------------------------------------------------
// stage profiler: HIP events recorded on the launch stream around each stage
// (gs_profile_enable / gs_profile_collect); off by default.
// ---------------------------------------------------------------------
enum Stage {
    ST_PREPROCESS = 0, ST_DEPTH_SORT, ST_SCAN, ST_EMIT, ST_TILE_SORT, ST_RANGES, ST_RENDER_FWD,
    ST_RENDER_BWD, ST_GAUSS_BWD, ST_APPLY_WEIGHTS, ST_COUNT
};
const char* kStageNames[ST_COUNT] = {"preprocess", "depth_sort", "scan", "emit", "tile_sort", "ranges",
                                     "render_fwd", "render_bwd", "gauss_bwd", "apply_weights"};
struct ProfRecord {
    int stage;
    hipEvent_t a, b;
};
// Process-wide: torch's autograd runs the backward on its own device thread.
struct Profiler {
    std::atomic<bool> on{false};
    std::atomic<uint32_t> mask{0xFFFFFFFFu};  // stages bracketed while on (gs_profile_set_stages)
    std::mutex mu;
    std::vector<ProfRecord> recs;
    std::vector<hipEvent_t> pool;
    hipEvent_t get() {
        {
            std::lock_guard<std::mutex> g(mu);
            if (!pool.empty()) {
                hipEvent_t e = pool.back();
                pool.pop_back();
                return e;
            }
        }
        // timing events without the system-scope release fence a plain event adds to the
        // stream (the fence alone stalls the queue ~10 us per event between two kernels)
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return nullptr;
        return e;
    }
    void add(int stage, hipEvent_t a, hipEvent_t b) {
        std::lock_guard<std::mutex> g(mu);
        recs.push_back({stage, a, b});
    }
};
Profiler& profiler() {
    static Profiler p;
    return p;
}
struct StageScope {
    Profiler& p;
    int stage;
    hipStream_t s;
    hipEvent_t a = nullptr;
    StageScope(int st, hipStream_t stream) : p(profiler()), stage(st), s(stream) {
        if (p.on.load(std::memory_order_relaxed) && ((p.mask.load(std::memory_order_relaxed) >> st) & 1u) &&
            (a = p.get()))
            (void)hipEventRecord(a, s);
    }
    ~StageScope() {
        if (!a) return;
        hipEvent_t b = p.get();
        if (!b) return;
        (void)hipEventRecord(b, s);
        p.add(stage, a, b);
    }
};

// ---------------------------------------------------------------------
// blend-kernel diagnostics (off by default): device buffers with per-wave
// timestamps, read back by gs_profile_diag_read.
// ---------------------------------------------------------------------
struct Diag {
    std::atomic<bool> on{false};
    std::mutex mu;
    uint64_t* buf[3] = {nullptr, nullptr, nullptr};
    size_t cap[3] = {0, 0, 0};
    size_t used[3] = {0, 0, 0};
};
Diag& diag() {
    static Diag d;
    return d;
}

template <typename T>
T* at(void* base, size_t off) {
    return reinterpret_cast<T*>(static_cast<char*>(base) + off);
}
template <typename T>
const T* at(const void* base, size_t off) {
    return reinterpret_cast<const T*>(static_cast<const char*>(base) + off);
}

struct Grid {
    int W, H, gx, gy, tiles;
    float fx, fy;
};

Grid make_grid(const gs_settings* s) {
    Grid g;
    g.W = s->image_width;
    g.H = s->image_height;
    g.gx = (g.W + kTile - 1) / kTile;
    g.gy = (g.H + kTile - 1) / kTile;
    g.tiles = g.gx * g.gy;
    // rasterizer_impl.cu:190-191
    g.fy = g.H / (2.0f * s->tanfovy);
    g.fx = g.W / (2.0f * s->tanfovx);
    return g;
}

int sh_coeffs_needed(int D) { return D >= 3 ? 16 : (D + 1) * (D + 1); }

gs_params make_params(int P, int M, const float* means3D, const float* shs, const float* colors_precomp,
                      const float* opacities, const float* scales, const float* rotations,
                      const float* cov3D_precomp) {
    gs_params g;
    g.P = P;
    g.M = shs ? M : 0;
    g.means3D = means3D;
    g.sh_dc = shs;
    g.sh_rest = shs ? shs + 3 : nullptr;
    g.sh_dc_stride = g.sh_rest_stride = 3 * M;
    g.colors_precomp = colors_precomp;
    g.opacities = opacities;
    g.scales = scales;
    g.rotations = rotations;
    g.cov3D_precomp = cov3D_precomp;
    g.activation = 0;
    g.sh_half = 0;
    g.index = nullptr;
    g.visible_out = nullptr;
    return g;
}

int validate_params(const gs_settings* s, const gs_params* g, bool need_opacity = true) {
    if (!s) return set_error(GS_ERR_INVALID_ARG, "settings is NULL");
    if (!g) return set_error(GS_ERR_INVALID_ARG, "params is NULL");
    if (s->image_width <= 0 || s->image_height <= 0)
        return set_error(GS_ERR_INVALID_ARG, "image size must be positive (got %dx%d)", s->image_width, s->image_height);
    if (g->P < 0) return set_error(GS_ERR_INVALID_ARG, "P must be >= 0");
    if (g->P == 0) return GS_OK;
    if (!g->means3D) return set_error(GS_ERR_INVALID_ARG, "means3D must have dimensions (num_points, 3)");
    if (need_opacity && !g->opacities) return set_error(GS_ERR_INVALID_ARG, "opacities are required");
    if (!s->viewmatrix || !s->projmatrix || !s->bg || !s->campos)
        return set_error(GS_ERR_INVALID_ARG, "viewmatrix, projmatrix, bg and campos are required");
    if (!g->sh_dc && !g->colors_precomp)
        return set_error(GS_ERR_INVALID_ARG, "Please provide excatly one of either SHs or precomputed colors!");
    if (g->sh_dc && g->M < sh_coeffs_needed(s->sh_degree))
        return set_error(GS_ERR_INVALID_ARG, "sh has %d coefficients per channel, degree %d needs %d", g->M,
                         s->sh_degree, sh_coeffs_needed(s->sh_degree));
    if (g->sh_dc && g->M > 1 && !g->sh_rest) return set_error(GS_ERR_INVALID_ARG, "sh_rest is required when M > 1");
    if (!g->cov3D_precomp && (!g->scales || !g->rotations))
        return set_error(GS_ERR_INVALID_ARG,
                         "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    if (g->activation && g->cov3D_precomp)
        return set_error(GS_ERR_INVALID_ARG, "activation = 1 needs scales/rotations, not cov3D_precomp");
    return GS_OK;
}

ShView sh_view(const gs_params& g) {
    ShView v;
    v.dc = g.sh_dc;
    v.rest = g.sh_rest ? g.sh_rest : g.sh_dc;
    v.dc_stride = g.sh_dc_stride;
    v.rest_stride = g.sh_rest_stride;
    v.half = g.sh_half;
    return v;
}

// A forward between its two halves: everything enqueued up to the instance
// count's read-back (bin_begin), the rest once the count is on the host (bin_end).
struct FwdState {
    gs_settings s;
    gs_params gp;
    Grid g;
    int* radii = nullptr;
    void* geom = nullptr;
    void* img = nullptr;
    Staging* st = nullptr;
    PreprocessArgs pa;
    EmitArgs ea;
    ~FwdState() { staging_release(st); }
};

// First half of the forward: buffers, preprocess, counter read-back, depth
// sort, instance scan (rasterizer_impl.cu:179-239 up to the num_rendered copy),
// in three steps so several views can share one preprocess launch
// (gs_rasterize_forward_begin_multi): bin_prepare (buffers, counter memset,
// the preprocess arguments), the preprocess, bin_after_preprocess.
int bin_prepare(FwdState& f, int copy_colors, gs_alloc_fn alloc, void* ctx, hipStream_t stream) {
    const gs_settings* s = &f.s;
    const Grid& g = f.g;
    const gs_params& gp = f.gp;
    const int P = gp.P;
    const GeomLayout gl = geom_layout(P);
    const ImgLayout il = img_layout(g.W, g.H);
    void* geom = alloc(ctx, 0, gl.total);
    void* img = alloc(ctx, 2, il.total);
    if (!geom || !img) return set_error(GS_ERR_ALLOC, "allocator returned NULL for the geometry/image buffer");
    f.geom = geom;
    f.img = img;

    uint32_t* counters = at<uint32_t>(img, il.counters);
    GS_HIP(hipMemsetAsync(counters, 0, il.total - il.counters, stream));  // counters, ranges, tile_last, ...

    PreprocessArgs& pa = f.pa;
    pa.P = P; pa.D = s->sh_degree; pa.M = gp.M; pa.W = g.W; pa.H = g.H; pa.gx = g.gx; pa.gy = g.gy;
    pa.means3D = gp.means3D; pa.sh = sh_view(gp); pa.colors_precomp = gp.colors_precomp;
    pa.opacities = gp.opacities; pa.scales = gp.scales; pa.rotations = gp.rotations;
    pa.index = gp.index;
    pa.cov3D_precomp = gp.cov3D_precomp; pa.activation = gp.activation;
    pa.view = s->viewmatrix; pa.proj = s->projmatrix; pa.campos = s->campos;
    pa.tanfovx = s->tanfovx; pa.tanfovy = s->tanfovy; pa.fx = g.fx; pa.fy = g.fy;
    pa.scale_modifier = s->scale_modifier;
    pa.prefiltered = s->prefiltered; pa.copy_colors = copy_colors;
    pa.radii_out = f.radii;
    pa.visible_out = gp.visible_out;
    pa.radii = at<int>(geom, gl.radii);
    pa.splat = at<Splat>(geom, gl.splat);
    pa.tiles_touched = at<uint32_t>(geom, gl.tiles_touched);
    pa.clamped = at<uint8_t>(geom, gl.clamped);
    pa.depth_key = at<uint32_t>(geom, gl.key0);
    pa.rect = at<uint32_t>(geom, gl.rect);
    pa.rect_packed = rect_packable(g.gx, g.gy) ? 1 : 0;
    pa.counters = counters;
    pa.touched = at<uint8_t>(geom, gl.touched);
    return GS_OK;
}

int bin_after_preprocess(FwdState& f, hipStream_t stream) {
    const gs_settings* s = &f.s;
    const Grid& g = f.g;
    const int P = f.gp.P;
    const bool debug = s->debug != 0;
    const GeomLayout gl = geom_layout(P);
    const ImgLayout il = img_layout(g.W, g.H);
    void* geom = f.geom;
    uint32_t* counters = at<uint32_t>(f.img, il.counters);
    PreprocessArgs& pa = f.pa;
    int rc = staging_acquire(&f.st);
    if (rc) return rc;
    GS_HIP(hipMemcpyAsync(f.st->host, counters, 4 * kCounterSlots * kCounterStride, hipMemcpyDeviceToHost, stream));
    GS_HIP(hipEventRecord(f.st->ev, stream));

    // depth order of the Gaussians (stable: ties keep index order)
    int cur;
    { StageScope sc(ST_DEPTH_SORT, stream);
    cur = radix_sort_aux(at<uint32_t>(geom, gl.key0), at<uint32_t>(geom, gl.key1), at<uint2>(geom, gl.val0),
                         at<uint2>(geom, gl.val1), pa.rect, (uint32_t)P, depth_sort_bits(), depth_pass_bits(),
                         kDepthSortIPT, at<uint32_t>(geom, gl.sort_hist), at<uint32_t>(geom, gl.sort_totals),
                         gl.sort_blocks, stream, nullptr, counters + 2); }
    if (cur < 0) return set_error(GS_ERR_INVALID_ARG, "depth sort: bad digit layout");
    GS_LAUNCHED("depth sort");

    EmitArgs& ea = f.ea;
    ea.P = P; ea.gx = g.gx; ea.gy = g.gy;
    ea.order = at<uint2>(geom, cur ? gl.val1 : gl.val0);
    ea.rect_packed = pa.rect_packed;
    ea.tiles_touched = pa.tiles_touched;
    ea.splat = pa.splat;
    ea.radii = pa.radii;
    ea.scan_sums = at<uint32_t>(geom, gl.scan_sums);
    ea.first_slot = at<uint32_t>(geom, gl.first_slot);
    ea.scan_blocks = gl.scan_blocks;
    ea.xhist = tile_sort_fused(g.gx, g.gy) && pa.rect_packed && !tile_sort_unfused() ? at<uint32_t>(geom, gl.emit_hist)
                                                                                    : nullptr;
    { StageScope sc(ST_SCAN, stream); launch_scan_reduce(ea, stream); }
    GS_LAUNCHED("instance scan");
    return GS_OK;
}

int bin_begin(FwdState& f, int copy_colors, gs_alloc_fn alloc, void* ctx, hipStream_t stream) {
    const bool debug = f.s.debug != 0;
    int rc = bin_prepare(f, copy_colors, alloc, ctx, stream);
    if (rc) return rc;
    { StageScope sc(ST_PREPROCESS, stream); launch_preprocess(f.pa, stream); }
    GS_LAUNCHED("preprocess");
    return bin_after_preprocess(f, stream);
}

// Second half: wait for the instance count (the reference's one host sync,
// rasterizer_impl.cu:236-239), then emission, tile sort and tile ranges.  On
// success *bin_out holds the binning buffer and *K_out the instance count.
int bin_end(FwdState& f, gs_alloc_fn alloc, void* ctx, hipStream_t stream, void** bin_out, int* K_out) {
    const gs_settings* s = &f.s;
    const Grid& g = f.g;
    const int P = f.gp.P;
    const bool debug = s->debug != 0;
    const GeomLayout gl = geom_layout(P);
    const ImgLayout il = img_layout(g.W, g.H);
    void* geom = f.geom;
    void* img = f.img;
    Staging* st = f.st;
    PreprocessArgs& pa = f.pa;
    EmitArgs& ea = f.ea;

    GS_HIP(hipEventSynchronize(st->ev));
    uint64_t K64 = 0;
    uint32_t kmax = 0, kmin_not = 0;
    for (int i = 0; i < kCounterSlots; ++i) {
        const uint32_t* c = st->host + kCounterStride * i;
        K64 += c[0];
        kmax = c[1] > kmax ? c[1] : kmax;
        kmin_not = c[2] > kmin_not ? c[2] : kmin_not;
    }
    const bool prefilter_fail = st->host[3] != 0;
    staging_release(st);
    f.st = nullptr;
    if (prefilter_fail) return set_error(GS_ERR_PREFILTERED, "Point is filtered although prefiltered is set. This shouldn't happen!");
    if (K64 > (uint64_t)std::numeric_limits<int>::max()) return set_error(GS_ERR_INVALID_ARG, "too many tile instances (%llu)", (unsigned long long)K64);
    const uint32_t K = (uint32_t)K64;
    if ((K && kmax - ~kmin_not >= (1u << depth_sort_bits())) || force_depth_keys32()) {
        // the visible depth keys span more bits than the short sort covered: redo the depth order
        // on the full 32-bit keys
        int cur;
        { StageScope sc(ST_DEPTH_SORT, stream);
        launch_depth_keys32(P, pa.rect, pa.splat, at<uint32_t>(geom, gl.key0), stream);
        cur = radix_sort_aux(at<uint32_t>(geom, gl.key0), at<uint32_t>(geom, gl.key1), at<uint2>(geom, gl.val0),
                             at<uint2>(geom, gl.val1), pa.rect, (uint32_t)P, 32, 8, kDepthSortIPT,
                             at<uint32_t>(geom, gl.sort_hist), at<uint32_t>(geom, gl.sort_totals), gl.sort_blocks,
                             stream); }
        ea.order = at<uint2>(geom, cur ? gl.val1 : gl.val0);
        { StageScope sc(ST_SCAN, stream); launch_scan_reduce(ea, stream); }
        GS_LAUNCHED("depth sort (32-bit keys)");
    }
    *K_out = (int)K;

    const BinLayout bl = bin_layout((int)K, g.tiles);
    void* bin = alloc(ctx, 1, bl.total);
    if (!bin) return set_error(GS_ERR_ALLOC, "allocator returned NULL for the binning buffer");
    *bin_out = bin;
    if (K == 0) return GS_OK;

    const TileSortPlan plan = tile_sort_plan(g.tiles);
    if (ea.xhist) {  // two-level binning (tile_sort_fused): column-ordered emission, row pass, ranges
        ea.tile_key = at<uint32_t>(bin, bl.key1);
        ea.pairs_out = at<uint2>(bin, bl.pair1);
        ea.xtotals = at<uint32_t>(bin, bl.sort_totals);
        ea.tile_count = at<uint32_t>(bin, bl.tile_count);
        ea.ntiles = g.tiles;
        ea.rec_flags32 = at<uint32_t>(bin, bl.rec_flags);
        { StageScope sc(ST_EMIT, stream); launch_emit_fused(ea, stream); }
        { StageScope sc(ST_TILE_SORT, stream);
        launch_row_pass(ea, K, at<uint2>(bin, bl.point_pairs), at<uint32_t>(bin, bl.sort_hist), bl.sort_blocks,
                        at<uint2>(img, il.ranges), stream); }
        GS_LAUNCHED("two-level binning");
        return GS_OK;
    }
    ea.tile_key = at<uint32_t>(bin, bl.key0);
    ea.slot_gauss = at<uint32_t>(bin, bl.slot_gauss);
    ea.rec_flags32 = at<uint32_t>(bin, bl.rec_flags);
    { StageScope sc(ST_EMIT, stream); launch_scan_emit(ea, stream); }
    GS_LAUNCHED("emit");

    int tc;
    { StageScope sc(ST_TILE_SORT, stream);
    tc = tile_sort(at<uint32_t>(bin, bl.key0), at<uint32_t>(bin, bl.key1), at<uint2>(bin, bl.pair0),
                   at<uint2>(bin, bl.pair1), at<uint32_t>(bin, bl.slot_gauss), K, plan.bits,
                   at<uint32_t>(bin, bl.sort_hist), at<uint32_t>(bin, bl.sort_totals), bl.sort_blocks, stream,
                   at<uint2>(img, il.ranges), at<uint32_t>(img, il.tile_order), g.tiles); }
    GS_LAUNCHED("tile sort");
    if (!tile_sort_writes_ranges(g.tiles)) {
        StageScope sc(ST_RANGES, stream);
        launch_ranges(at<uint32_t>(bin, tc ? bl.key1 : bl.key0), (int)K, at<uint2>(img, il.ranges), nullptr, stream);
        GS_LAUNCHED("ranges");
    }
    return GS_OK;
}

// Everything of the forward up to (and including) tile ranges, in one call.
int bin_forward(const gs_settings* s, const Grid& g, const gs_params& gp, int* radii_out, int copy_colors,
                gs_alloc_fn alloc, void* ctx, hipStream_t stream, void** geom_out, void** img_out, void** bin_out,
                int* K_out) {
    FwdState f;
    f.s = *s;
    f.gp = gp;
    f.g = g;
    f.radii = radii_out;
    int rc = bin_begin(f, copy_colors, alloc, ctx, stream);
    *geom_out = f.geom;
    *img_out = f.img;
    if (rc) return rc;
    return bin_end(f, alloc, ctx, stream, bin_out, K_out);
}

}  // namespace

struct gs_forward_state {
    FwdState f;
};

namespace gs {
int report_error(int code, const char* msg) { return set_error(code, "%s", msg); }

uint64_t* diag_buffer(int which, size_t n_u64) {
    Diag& d = diag();
    if (!d.on.load()) return nullptr;
    std::lock_guard<std::mutex> g(d.mu);
    if (d.cap[which] < n_u64) {
        if (d.buf[which]) (void)hipFree(d.buf[which]);
        d.buf[which] = nullptr;
        if (hipMalloc((void**)&d.buf[which], n_u64 * 8) != hipSuccess) return nullptr;
        d.cap[which] = n_u64;
    }
    d.used[which] = n_u64;
    return d.buf[which];
}
}  // namespace gs

extern "C" {

const char* gs_last_error(void) { return g_last_error.c_str(); }

int gs_profile_diag_enable(int on) {
    diag().on.store(on != 0);
    return GS_OK;
}

long long gs_profile_diag_read(int which, uint64_t* host, long long max_u64) {
    Diag& d = diag();
    std::lock_guard<std::mutex> g(d.mu);
    if (which < 0 || which > 2 || !d.buf[which]) return 0;
    const size_t n = d.used[which] < (size_t)max_u64 ? d.used[which] : (size_t)max_u64;
    GS_HIP(hipDeviceSynchronize());
    GS_HIP(hipMemcpy(host, d.buf[which], n * 8, hipMemcpyDeviceToHost));
    return (long long)n;
}

int gs_profile_enable(int on) {
    profiler().on.store(on != 0);
    return GS_OK;
}

int gs_profile_set_stages(unsigned int mask) {
    profiler().mask.store(mask);
    return GS_OK;
}

int gs_profile_num_stages(void) { return ST_COUNT; }
const char* gs_profile_stage_name(int i) { return (i >= 0 && i < ST_COUNT) ? kStageNames[i] : ""; }

int gs_profile_collect(double* total_ms, int* counts, int n) {
    Profiler& p = profiler();
    for (int i = 0; i < n; ++i) { total_ms[i] = 0.0; counts[i] = 0; }
    std::vector<ProfRecord> recs;
    {
        std::lock_guard<std::mutex> g(p.mu);
        recs.swap(p.recs);
    }
    for (const ProfRecord& r : recs) {
        GS_HIP(hipEventSynchronize(r.b));
        float ms = 0.f;
        GS_HIP(hipEventElapsedTime(&ms, r.a, r.b));
        if (r.stage < n) { total_ms[r.stage] += ms; counts[r.stage] += 1; }
    }
    std::lock_guard<std::mutex> g(p.mu);
    for (const ProfRecord& r : recs) { p.pool.push_back(r.a); p.pool.push_back(r.b); }
    return GS_OK;
}

int gs_abi_version(void) { return GS_RASTER_ABI_VERSION; }

int gs_blend_exp(long long n, const float* x, float* y, gs_stream_t stream) {
    if (n < 0 || (n > 0 && (!x || !y))) return set_error(GS_ERR_INVALID_ARG, "gs_blend_exp: bad arguments");
    if (n == 0) return GS_OK;
    if ((n + 3) / 4 > 255ll * 0x7FFFFFFF) return set_error(GS_ERR_INVALID_ARG, "gs_blend_exp: n too large");
    gs::launch_blend_exp(n, x, y, (hipStream_t)stream);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GS_OK : set_error(GS_ERR_HIP, "gs_blend_exp launch failed: %s", hipGetErrorString(e));
}

size_t gs_geometry_buffer_size(int P) { return geom_layout(P).total; }
size_t gs_image_buffer_size(int width, int height) { return img_layout(width, height).total; }
size_t gs_binning_buffer_size(int num_rendered, int num_tiles) { return bin_layout(num_rendered, num_tiles).total; }

long long gs_buffer_offset(const char* buffer, const char* field, int P, int width, int height, int num_rendered) {
    if (!buffer || !field) return -1;
    if (!strcmp(buffer, "geometry")) {
        const GeomLayout L = geom_layout(P);
        // the per-Gaussian render record (64 B stride: means2D at +0, conic_opacity at +16, rgbd at +32)
        if (!strcmp(field, "splat") || !strcmp(field, "means2D")) return (long long)L.splat;
        if (!strcmp(field, "conic_opacity")) return (long long)(L.splat + offsetof(Splat, co));
        if (!strcmp(field, "rgbd")) return (long long)(L.splat + offsetof(Splat, rgbd));
        if (!strcmp(field, "tiles_touched")) return (long long)L.tiles_touched;
        if (!strcmp(field, "clamped")) return (long long)L.clamped;
        if (!strcmp(field, "touched")) return (long long)L.touched;
        if (!strcmp(field, "radii")) return (long long)L.radii;
        if (!strcmp(field, "first_slot")) return (long long)L.first_slot;
    } else if (!strcmp(buffer, "image")) {
        const ImgLayout L = img_layout(width, height);
        if (!strcmp(field, "final_T")) return (long long)L.final_T;
        if (!strcmp(field, "n_contrib")) return (long long)L.n_contrib;
        if (!strcmp(field, "ranges")) return (long long)L.ranges;
        if (!strcmp(field, "tile_last")) return (long long)L.tile_last;
        if (!strcmp(field, "quad_last")) return (long long)L.quad_last;
    } else if (!strcmp(buffer, "binning")) {
        const int tiles = ((width + 15) / 16) * ((height + 15) / 16);
        const BinLayout L = bin_layout(num_rendered, tiles);
        if (!strcmp(field, "point_pairs")) return (long long)L.point_pairs;
        if (!strcmp(field, "slot_gauss")) return (long long)L.slot_gauss;
        if (!strcmp(field, "records")) return (long long)L.records;
        if (!strcmp(field, "rec_flags")) return (long long)L.rec_flags;
    }
    return -1;
}

int gs_rasterize_forward(const gs_settings* s, int P, int M, const float* means3D, const float* shs,
                         const float* colors_precomp, const float* opacities, const float* scales,
                         const float* rotations, const float* cov3D_precomp, float* out_color, float* out_depth,
                         int* radii, gs_alloc_fn alloc, void* alloc_ctx, gs_stream_t stream, int* num_rendered) {
    const gs_params g = make_params(P, M, means3D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp);
    return gs_rasterize_forward_ex(s, &g, out_color, out_depth, radii, alloc, alloc_ctx, stream, num_rendered);
}

int gs_rasterize_forward_begin(const gs_settings* s, const gs_params* gp, int* radii, gs_alloc_fn alloc,
                               void* alloc_ctx, gs_stream_t stream_, gs_forward_state** state) {
    try {
        hipStream_t stream = (hipStream_t)stream_;
        if (!state || !alloc) return set_error(GS_ERR_INVALID_ARG, "state and alloc are required");
        *state = nullptr;
        int rc = validate_params(s, gp);
        if (rc) return rc;
        std::unique_ptr<gs_forward_state> st(new gs_forward_state());
        FwdState& f = st->f;
        f.s = *s;
        f.gp = *gp;
        f.g = make_grid(s);
        f.radii = radii;
        if (gp->P == 0) {  // rasterize_points.cu:57-72: empty buffers (the outputs are zeroed by _end)
            alloc(alloc_ctx, 0, 0);
            alloc(alloc_ctx, 2, 0);
        } else {
            rc = bin_begin(f, 1, alloc, alloc_ctx, stream);
            if (rc) return rc;
        }
        *state = st.release();
        return GS_OK;
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

// Per-call events ordering the shared preprocess between the views' streams (a small pool per thread).
hipEvent_t multi_event(int i) {
    thread_local hipEvent_t ev[2 * kMaxViews] = {};
    if (!ev[i] && hipEventCreateWithFlags(&ev[i], hipEventDisableTiming) != hipSuccess) return nullptr;
    return ev[i];
}

bool same_scene(const gs_params& a, const gs_params& b) {
    return a.P == b.P && a.M == b.M && a.means3D == b.means3D && a.sh_dc == b.sh_dc && a.sh_rest == b.sh_rest &&
           a.sh_dc_stride == b.sh_dc_stride && a.sh_rest_stride == b.sh_rest_stride && a.sh_half == b.sh_half &&
           a.colors_precomp == b.colors_precomp && a.opacities == b.opacities && a.scales == b.scales &&
           a.rotations == b.rotations && a.cov3D_precomp == b.cov3D_precomp && a.index == b.index &&
           a.activation == b.activation;
}

int gs_rasterize_forward_begin_multi(int n, const gs_settings* const* s, const gs_params* const* gp, int* const* radii,
                                     gs_alloc_fn alloc, void* const* alloc_ctx, const gs_stream_t* streams,
                                     gs_forward_state** states) {
    if (n < 1 || n > kMaxViews || !s || !gp || !radii || !alloc || !alloc_ctx || !streams || !states)
        return set_error(GS_ERR_INVALID_ARG, "begin_multi: 1 <= n <= %d views and every array are required", kMaxViews);
    for (int v = 0; v < n; ++v) states[v] = nullptr;
    bool shared = gp[0]->P > 0 && !gp[0]->sh_half && !gp[0]->index;
    for (int v = 0; v < n && shared; ++v) {
        shared = same_scene(*gp[0], *gp[v]) && !s[v]->debug;
        if (v && (s[v]->image_width != s[0]->image_width || s[v]->image_height != s[0]->image_height)) shared = false;
    }
    if (!shared) {  // the per-view calls (identical outputs)
        for (int v = 0; v < n; ++v) {
            const int rc = gs_rasterize_forward_begin(s[v], gp[v], radii[v], alloc, alloc_ctx[v], streams[v], &states[v]);
            if (rc) {
                for (int u = 0; u < v; ++u) gs_rasterize_forward_release(states[u]);
                for (int u = 0; u < n; ++u) states[u] = nullptr;
                return rc;
            }
        }
        return GS_OK;
    }
    try {
        std::unique_ptr<gs_forward_state> st[kMaxViews];
        PreprocessMulti m;
        m.nv = n;
        hipStream_t s0 = (hipStream_t)streams[0];
        const bool debug = false;
        hipStream_t stream = s0;  // (GS_LAUNCHED)
        for (int v = 0; v < n; ++v) {
            int rc = validate_params(s[v], gp[v]);
            if (rc) return rc;
            st[v].reset(new gs_forward_state());
            FwdState& f = st[v]->f;
            f.s = *s[v];
            f.gp = *gp[v];
            f.g = make_grid(s[v]);
            f.radii = radii[v];
            rc = bin_prepare(f, 1, alloc, alloc_ctx[v], (hipStream_t)streams[v]);
            if (rc) return rc;
            m.a[v] = f.pa;
            if (v && streams[v] != streams[0]) {  // the shared pass writes view v's buffers after their zeroing
                hipEvent_t e = multi_event(v);
                if (!e) return set_error(GS_ERR_HIP, "begin_multi: event");
                GS_HIP(hipEventRecord(e, (hipStream_t)streams[v]));
                GS_HIP(hipStreamWaitEvent(s0, e, 0));
            }
        }
        { StageScope sc(ST_PREPROCESS, s0); launch_preprocess_multi(m, s0); }
        GS_LAUNCHED("preprocess (views)");
        hipEvent_t done = multi_event(kMaxViews);
        if (!done) return set_error(GS_ERR_HIP, "begin_multi: event");
        GS_HIP(hipEventRecord(done, s0));
        for (int v = 0; v < n; ++v) {
            hipStream_t sv = (hipStream_t)streams[v];
            if (sv != s0) GS_HIP(hipStreamWaitEvent(sv, done, 0));
            const int rc = bin_after_preprocess(st[v]->f, sv);
            if (rc) return rc;
        }
        for (int v = 0; v < n; ++v) states[v] = st[v].release();
        return GS_OK;
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

int gs_rasterize_forward_end(gs_forward_state* state, float* out_color, float* out_depth, gs_alloc_fn alloc,
                             void* alloc_ctx, gs_stream_t stream_, int* num_rendered) {
    std::unique_ptr<gs_forward_state> own(state);
    try {
        hipStream_t stream = (hipStream_t)stream_;
        if (!state) return set_error(GS_ERR_INVALID_ARG, "state is NULL");
        if (!num_rendered || !alloc || !out_color || !out_depth)
            return set_error(GS_ERR_INVALID_ARG, "num_rendered, alloc, out_color and out_depth are required");
        *num_rendered = 0;
        FwdState& f = state->f;
        const gs_settings* s = &f.s;
        const int P = f.gp.P;
        const bool debug = s->debug != 0;
        const Grid g = f.g;
        if (P == 0) {  // rasterize_points.cu:57-72: zero outputs, empty buffers, no render
            alloc(alloc_ctx, 1, 0);
            GS_HIP(hipMemsetAsync(out_color, 0, sizeof(float) * 3 * (size_t)g.W * g.H, stream));
            GS_HIP(hipMemsetAsync(out_depth, 0, sizeof(float) * (size_t)g.W * g.H, stream));
            return GS_OK;
        }
        void* geom = f.geom;
        void* img = f.img;
        void* bin = nullptr;
        int K = 0;
        int rc = bin_end(f, alloc, alloc_ctx, stream, &bin, &K);
        if (rc) return rc;
        const GeomLayout gl = geom_layout(P);
        const ImgLayout il = img_layout(g.W, g.H);
        const BinLayout bl = bin_layout(K, g.tiles);
        RenderArgs ra;
        ra.W = g.W; ra.H = g.H; ra.gx = g.gx; ra.gy = g.gy;
        ra.ranges = at<uint2>(img, il.ranges);
        ra.tile_order = at<uint32_t>(img, il.tile_order);
        ra.order_ready = K > 0 && tile_sort_writes_ranges(g.tiles) ? 1 : 0;
        ra.point_pairs = at<uint2>(bin, bl.point_pairs);
        ra.bwd_items = at<uint2>(bin, bl.bwd_items);
        ra.bwd_count = at<uint32_t>(img, il.bwd_count);
        ra.item_cap = (uint32_t)(4 * bl.nslots);
        ra.splat = at<Splat>(geom, gl.splat);
        ra.bg = s->bg;
        ra.final_T = at<float>(img, il.final_T);
        ra.n_contrib = at<uint32_t>(img, il.n_contrib);
        ra.tile_last = at<uint32_t>(img, il.tile_last);
        ra.quad_last = at<uint32_t>(img, il.quad_last);
        ra.ckpt = at<float4>(bin, bl.ckpt);
        ra.used = at<uint64_t>(bin, bl.used);
        ra.out_color = out_color;
        ra.out_depth = out_depth;
        ra.touched = at<uint8_t>(geom, gl.touched);
        ra.diag = diag_buffer(0, kDiagWords * (size_t)g.tiles * 4);
        { StageScope sc(ST_RENDER_FWD, stream); launch_render_forward(ra, stream); }
        GS_LAUNCHED("render");
        *num_rendered = K;
        return GS_OK;
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

void gs_rasterize_forward_release(gs_forward_state* state) { delete state; }

int gs_rasterize_forward_ex(const gs_settings* s, const gs_params* gp, float* out_color, float* out_depth, int* radii,
                            gs_alloc_fn alloc, void* alloc_ctx, gs_stream_t stream, int* num_rendered) {
    if (num_rendered) *num_rendered = 0;
    if (!num_rendered || !alloc || !out_color || !out_depth)
        return set_error(GS_ERR_INVALID_ARG, "num_rendered, alloc, out_color and out_depth are required");
    gs_forward_state* st = nullptr;
    const int rc = gs_rasterize_forward_begin(s, gp, radii, alloc, alloc_ctx, stream, &st);
    if (rc) return rc;
    return gs_rasterize_forward_end(st, out_color, out_depth, alloc, alloc_ctx, stream, num_rendered);
}

int gs_rasterize_backward(const gs_settings* s, int P, int M, int R, const float* means3D, const float* shs,
                          const float* colors_precomp, const float* scales, const float* rotations,
                          const float* cov3D_precomp, const int* radii, const void* geom, const void* binning,
                          const void* img, const float* dL_dpix, float* dL_dmeans2D, float* dL_dcolors,
                          float* dL_dopacity, float* dL_dmeans3D, float* dL_dcov3D, float* dL_dsh, float* dL_dscales,
                          float* dL_drotations, gs_stream_t stream) {
    const gs_params g = make_params(P, M, means3D, shs, colors_precomp, nullptr, scales, rotations, cov3D_precomp);
    gs_grads o;
    o.dL_dmeans2D = dL_dmeans2D; o.dL_dcolors = dL_dcolors; o.dL_dopacity = dL_dopacity;
    o.dL_dmeans3D = dL_dmeans3D; o.dL_dcov3D = dL_dcov3D;
    o.dL_dsh_dc = (shs || M > 0) ? dL_dsh : nullptr;
    o.dL_dsh_rest = o.dL_dsh_dc ? dL_dsh + 3 : nullptr;
    o.dsh_dc_stride = o.dsh_rest_stride = 3 * M;
    o.dL_dscales = dL_dscales; o.dL_drotations = dL_drotations;
    o.accumulate = 0;
    o.grad_mask = nullptr;
    o.mask_bits = 0;
    o.dL_dconic = nullptr;
    o.writes_after = nullptr;
    gs_params g2 = g;
    g2.M = M;  // dL_dsh is [P,M,3] even when shs is absent (then all zero)
    return gs_rasterize_backward_ex(s, &g2, R, radii, geom, binning, img, dL_dpix, &o, stream);
}

int gs_rasterize_backward_ex(const gs_settings* s, const gs_params* gp, int R, const int* radii, const void* geom,
                             const void* binning, const void* img, const float* dL_dpix, const gs_grads* o,
                             gs_stream_t stream_) {
    try {
        hipStream_t stream = (hipStream_t)stream_;
        if (!s || !gp || !o) return set_error(GS_ERR_INVALID_ARG, "settings, params and grads are required");
        const int P = gp->P;
        if (P < 0) return set_error(GS_ERR_INVALID_ARG, "P must be >= 0");
        if (P == 0) return GS_OK;
        if (s->image_width <= 0 || s->image_height <= 0) return set_error(GS_ERR_INVALID_ARG, "image size must be positive");
        if (!gp->means3D || !s->viewmatrix || !s->projmatrix || !s->bg || !s->campos)
            return set_error(GS_ERR_INVALID_ARG, "means3D, viewmatrix, projmatrix, bg and campos are required");
        if (gp->sh_dc && gp->M < sh_coeffs_needed(s->sh_degree))
            return set_error(GS_ERR_INVALID_ARG, "sh has %d coefficients per channel, degree %d needs %d", gp->M,
                             s->sh_degree, sh_coeffs_needed(s->sh_degree));
        if (!gp->cov3D_precomp && (!gp->scales || !gp->rotations))
            return set_error(GS_ERR_INVALID_ARG, "scales/rotations or cov3D_precomp are required");
        if (gp->activation && !gp->opacities)
            return set_error(GS_ERR_INVALID_ARG, "activation = 1 needs the raw opacities in the backward");
        if (!geom || !img || !radii || !dL_dpix)
            return set_error(GS_ERR_INVALID_ARG, "geometry/image buffers, radii and dL_dpix are required");
        if (!o->dL_dmeans2D || !o->dL_dopacity || !o->dL_dmeans3D || !o->dL_dscales ||
            !o->dL_drotations || (gp->M > 1 && o->dL_dsh_dc && !o->dL_dsh_rest))
            return set_error(GS_ERR_INVALID_ARG, "gradient outputs are required");
        if (R > 0 && !binning) return set_error(GS_ERR_INVALID_ARG, "binning buffer is required when num_rendered > 0");
        const bool debug = s->debug != 0;
        const Grid g = make_grid(s);
        const GeomLayout gl = geom_layout(P);
        const ImgLayout il = img_layout(g.W, g.H);
        const BinLayout bl = bin_layout(R, g.tiles);
        float4* records = R > 0 ? at<float4>(const_cast<void*>(binning), bl.records) : nullptr;
        uint8_t* rec_flags = R > 0 ? at<uint8_t>(const_cast<void*>(binning), bl.rec_flags) : nullptr;
        // per-Gaussian "has a record" bytes: k_gauss_bwd skips every Gaussian without one (all of
        // its gradients are zero), which is most of them (occluded behind saturated pixels)
        // (both zeroed by the forward: `touched` in preprocess, the flags with the tile ranges.  A
        // second backward of the same forward finds the bytes of the first, which it sets again: the
        // entries that get records depend on the forward alone)
        uint8_t* touched = at<uint8_t>(const_cast<void*>(geom), gl.touched);
        if (R > 0) {
            uint32_t* bwd_count = at<uint32_t>(const_cast<void*>(img), il.bwd_count);
            RenderBwdArgs rb;
            rb.W = g.W; rb.H = g.H; rb.gx = g.gx; rb.gy = g.gy;
            rb.ranges = at<uint2>(img, il.ranges);
            rb.point_pairs = at<uint2>(binning, bl.point_pairs);
            rb.bwd_items = at<uint2>(binning, bl.bwd_items);
            rb.bwd_count = bwd_count;
            rb.tile_last = at<uint32_t>(img, il.tile_last);
            rb.item_cap = (uint32_t)(4 * bl.nslots);
            rb.quad_last = at<uint32_t>(img, il.quad_last);
            rb.ckpt = at<float4>(binning, bl.ckpt);
            rb.used = at<uint64_t>(binning, bl.used);
            rb.splat = at<Splat>(geom, gl.splat);
            rb.bg = s->bg;
            rb.final_T = at<float>(img, il.final_T);
            rb.n_contrib = at<uint32_t>(img, il.n_contrib);
            rb.dL_dpix = dL_dpix;
            rb.records = records;
            rb.rec_flags = rec_flags;
            rb.touched = touched;
            rb.diag = diag_buffer(1, kDiagWords * 4 * bl.nslots);
            { StageScope sc(ST_RENDER_BWD, stream); launch_render_backward(rb, stream); }
            GS_LAUNCHED("render backward");
        }
        GaussBwdArgs ga;
        ga.P = P; ga.D = s->sh_degree; ga.M = gp->M; ga.W = g.W; ga.H = g.H; ga.gx = g.gx; ga.gy = g.gy;
        ga.means3D = gp->means3D; ga.scales = gp->scales; ga.rotations = gp->rotations;
        ga.cov3D_precomp = gp->cov3D_precomp; ga.opacities = gp->opacities;
        ga.index = gp->index;
        ga.sh = sh_view(*gp);
        ga.dsh.dc = o->dL_dsh_dc;
        ga.dsh.rest = o->dL_dsh_rest ? o->dL_dsh_rest : o->dL_dsh_dc;
        ga.dsh.dc_stride = o->dsh_dc_stride;
        ga.dsh.rest_stride = o->dsh_rest_stride;
        ga.activation = gp->activation;
        ga.view = s->viewmatrix; ga.proj = s->projmatrix; ga.campos = s->campos;
        ga.tanfovx = s->tanfovx; ga.tanfovy = s->tanfovy; ga.fx = g.fx; ga.fy = g.fy;
        ga.scale_modifier = s->scale_modifier;
        ga.radii = radii;
        ga.tiles_touched = at<uint32_t>(geom, gl.tiles_touched);
        ga.first_slot = at<uint32_t>(geom, gl.first_slot);
        ga.clamped = at<uint8_t>(geom, gl.clamped);
        ga.rec_flags = rec_flags;
        ga.touched = touched;
        ga.live_count = at<uint32_t>(const_cast<void*>(geom), gl.live_count);
        ga.live_list = at<uint32_t>(const_cast<void*>(geom), gl.live_list);
        ga.records = records;
        ga.merged = render_backward_merged();
        ga.dL_dmeans2D = o->dL_dmeans2D; ga.dL_dcolors = o->dL_dcolors; ga.dL_dopacity = o->dL_dopacity;
        ga.dL_dmeans3D = o->dL_dmeans3D; ga.dL_dcov3D = o->dL_dcov3D;
        ga.dL_dscales = o->dL_dscales; ga.dL_drot = o->dL_drotations;
        ga.acc = o->accumulate;
        ga.grad_mask = o->grad_mask;
        ga.mask_bits = o->grad_mask ? o->mask_bits : 0u;
        ga.dL_dconic = o->dL_dconic;
        ga.diag = diag_buffer(2, kDiagWords * 4 * (size_t)(P / 256 + 1));
        { StageScope sc(ST_GAUSS_BWD, stream);
        launch_gauss_backward(ga, stream, (hipEvent_t)o->writes_after); }
        GS_LAUNCHED("gaussian backward");
        return GS_OK;
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

int gs_mark_visible(int P, const float* means3D, const float* viewmatrix, const float* projmatrix, uint8_t* present,
                    gs_stream_t stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    (void)projmatrix;
    if (P < 0) return set_error(GS_ERR_INVALID_ARG, "P must be >= 0");
    if (P == 0) return GS_OK;
    if (!means3D || !viewmatrix || !present) return set_error(GS_ERR_INVALID_ARG, "means3D, viewmatrix, present required");
    launch_mark_visible(P, means3D, viewmatrix, present, stream);
    const bool debug = false;
    GS_LAUNCHED("mark_visible");
    return GS_OK;
}

int gs_apply_weights(const gs_settings* s, int P, int M, const float* means3D, float* weights, int num_channels,
                     const float* opacities, const float* scales, const float* rotations, const float* cov3D_precomp,
                     const float* shs, const float* image_weights, int* cnt, gs_alloc_fn alloc, void* alloc_ctx,
                     gs_stream_t stream_) {
    try {
        hipStream_t stream = (hipStream_t)stream_;
        if (num_channels < 1 || num_channels > 3)
            return set_error(GS_ERR_UNSUPPORTED, "Unsupported number of channels: %d", num_channels);
        if (!alloc || !weights || !image_weights || !cnt)
            return set_error(GS_ERR_INVALID_ARG, "alloc, weights, image_weights and cnt are required");
        const gs_params gp = make_params(P, M, means3D, shs, weights, opacities, scales, rotations, cov3D_precomp);
        int rc = validate_params(s, &gp);
        if (rc) return rc;
        if (P == 0) return GS_OK;
        const bool debug = s->debug != 0;
        const Grid g = make_grid(s);
        void *geom = nullptr, *img = nullptr, *bin = nullptr;
        int K = 0;
        rc = bin_forward(s, g, gp, nullptr, 0, alloc, alloc_ctx, stream, &geom, &img, &bin, &K);
        if (rc) return rc;
        if (K == 0) return GS_OK;
        const GeomLayout gl = geom_layout(P);
        const ImgLayout il = img_layout(g.W, g.H);
        const BinLayout bl = bin_layout(K, g.tiles);
        ApplyWeightsArgs aw;
        aw.W = g.W; aw.H = g.H; aw.gx = g.gx; aw.gy = g.gy; aw.C = num_channels;
        aw.ranges = at<uint2>(img, il.ranges);
        aw.point_pairs = at<uint2>(bin, bl.point_pairs);
        aw.splat = at<Splat>(geom, gl.splat);
        aw.image_weights = image_weights;
        aw.weights = weights;
        aw.cnt = cnt;
        { StageScope sc(ST_APPLY_WEIGHTS, stream); launch_render_apply_weights(aw, stream); }
        GS_LAUNCHED("apply_weights render");
        return GS_OK;
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

}  // extern "C"
