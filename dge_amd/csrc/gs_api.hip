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

#include <chrono>
#include <limits>
#include <memory>
#include <atomic>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "gs_common.h"
#include "gs_internal.h"
#include "gs_raster.h"

using namespace gs;

namespace {

thread_local std::string g_last_error;
std::atomic<long long> g_host_wait_ns{0};  // gs_host_wait_ns

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
// DGE_AMD_TILE_SORT=2pass (a test switch): the emission + radix tile sort (+ k_ranges) on every grid, in place
// of the direct emission (<= 2048 tiles) and the two-level binning (larger grids)
bool tile_sort_unfused() {
    const char* e = getenv("DGE_AMD_TILE_SORT");
    return e && !strcmp(e, "2pass");
}
// the two-level binning (column-ordered emission, row pass) for a gx x gy grid (grids over 2048 tiles:
// at c2's 1024 it measured slower than the single-pass tile sort, emit 32 -> 52 us)
bool two_level(int gx, int gy) {
    return tile_sort_fused(gx, gy) && rect_packable(gx, gy) && !tile_sort_unfused();
}
// the region emission (launch_region_emit) for a gx x gy grid, opt-in: DGE_AMD_BINNING=region (an A/B and test
// switch).  It measured slower than the two-level binning at c4 (emit 574 vs 423 us), which stays
// the default there
bool region_emission(int gx, int gy) {
    const char* e = getenv("DGE_AMD_BINNING");
    return region_emission_grid(gx, gy) && !tile_sort_unfused() && e && !strcmp(e, "region");
}

// Pinned (coherent) read-back slot of one forward's preprocess counters, written by the depth sort's first
// kernel (CountPublish) and followed by its sequence word, which the host polls.  A pool per device: several
// forwards may be between begin and end at once (gs_rasterize_forward_begin / _end), each holding its own slot.
constexpr int kStagingWords = kCounterSlots * kCounterStride + 16;  // counters, the sequence word, padding
struct Staging {
    uint32_t* host = nullptr;
    uint32_t* dev_view = nullptr;  // the device's address of `host`
    uint32_t seq = 0;              // the value this slot's publication ends with
    bool armed = false;            // the kernel that publishes it was launched (else nothing will land)
    int dev = 0;
};
std::atomic<uint32_t> g_staging_seq{0};

// Wait (host) until the slot's publication has landed: its sequence word equals s->seq.  A forward's
// publication always comes (the depth sort runs for every P > 0); the bound only turns a lost device into an
// error instead of a hang.
bool staging_wait(const Staging* s) {
    const volatile uint32_t* w = s->host + kCounterSlots * kCounterStride;
    if (*w == s->seq) return true;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned spin = 0;; ++spin) {
        if (*w == s->seq) return true;
        if ((spin & 1023u) == 1023u) {
            if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(60)) return false;
            std::this_thread::yield();
        }
    }
}
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
    if (hipHostMalloc((void**)&s->host, 4 * kStagingWords, hipHostMallocCoherent) != hipSuccess) {
        delete s;
        return set_error(GS_ERR_HIP, "could not create the counter read-back slot");
    }
    memset(s->host, 0, 4 * kStagingWords);
    if (hipHostGetDevicePointer((void**)&s->dev_view, s->host, 0) != hipSuccess) {
        (void)hipHostFree(s->host);
        delete s;
        return set_error(GS_ERR_HIP, "could not map the counter read-back slot");
    }
    *out = s;
    return GS_OK;
}

// the slot's next publication: a sequence value no earlier use of the slot wrote (0 is never used)
CountPublish staging_publish(Staging* s, const uint32_t* counters) {
    uint32_t q = ++g_staging_seq;
    if (q == 0) q = ++g_staging_seq;
    s->seq = q;
    CountPublish p;
    p.src = counters;
    p.dst = s->dev_view;
    p.seq = q;
    return p;
}

void staging_release(Staging* s, bool synced = false) {
    if (!s) return;
    // a slot dropped before its forward's _end may still have its publication in flight:
    // the next forward to take it must not see that late write land over its own counters
    if (!synced && s->armed) (void)staging_wait(s);
    s->armed = false;
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
    ST_RENDER_BWD, ST_GAUSS_BWD, ST_APPLY_WEIGHTS, ST_GAUSS_LIVE, ST_COUNT
};
// (gauss_live: a batch's live-set pass when it runs apart from the rest of gauss_bwd, gs_views_backward)
const char* kStageNames[ST_COUNT] = {"preprocess", "depth_sort", "scan", "emit", "tile_sort", "ranges",
                                     "render_fwd", "render_bwd", "gauss_bwd", "apply_weights", "gauss_live"};
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
    g.forward_only = 0;
    g.aux_mask = nullptr;
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
    bool ids_ok = true;     // a forward-only render may bin Gaussian ids alone (not apply_weights' binning)
    bool ids_only = false;  // this binning did (EmitArgs::ids_only)
    ~FwdState() { staging_release(st); }
};

// First half of the forward: buffers, preprocess, counter read-back, depth
// sort, instance scan (rasterizer_impl.cu:179-239 up to the num_rendered copy):
// bin_prepare_in (counter memset, the preprocess arguments), the preprocess,
// bin_after_preprocess.
int bin_prepare_in(FwdState& f, int copy_colors, void* geom, void* img, hipStream_t stream) {
    const gs_settings* s = &f.s;
    const Grid& g = f.g;
    const gs_params& gp = f.gp;
    const int P = gp.P;
    const GeomLayout gl = geom_layout(P);
    const ImgLayout il = img_layout(g.W, g.H);
    f.geom = geom;
    f.img = img;

    uint32_t* counters = at<uint32_t>(img, il.counters);
    static_assert(kAlign % 16 == 0, "whole 16-B stores");
    launch_zero16(counters, il.total - il.counters, stream);  // counters, ranges, tile_last, ...
    { const bool debug = s->debug != 0; GS_LAUNCHED("zero image state"); }

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
    pa.aux_mask = gp.forward_only ? nullptr : gp.aux_mask;
    return GS_OK;
}

int bin_prepare(FwdState& f, int copy_colors, gs_alloc_fn alloc, void* ctx, hipStream_t stream) {
    void* geom = alloc(ctx, 0, geom_layout(f.gp.P).total);
    void* img = alloc(ctx, 2, img_layout(f.g.W, f.g.H).total);
    if (!geom || !img) return set_error(GS_ERR_ALLOC, "allocator returned NULL for the geometry/image buffer");
    return bin_prepare_in(f, copy_colors, geom, img, stream);
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
    // (read back by the depth sort's first kernel: against the round-5 D2H copy + event, c2 3217-3243 vs
    // 3208-3230 renders/s and the host's busy time per step 0.46-0.55 vs 0.56-0.68 ms, profiles/r06/queues/)
    const CountPublish pub = staging_publish(f.st, counters);

    // depth order of the Gaussians (stable: ties keep index order), any key range: MSD buckets + local sorts
    int cur = 0;
    { StageScope sc(ST_DEPTH_SORT, stream);
    cur = depth_sort_msd(at<uint32_t>(geom, gl.key0), at<uint32_t>(geom, gl.key1), at<uint2>(geom, gl.val0),
                         at<uint2>(geom, gl.val1), pa.rect, (uint32_t)P, at<uint32_t>(geom, gl.sort_hist),
                         at<uint32_t>(geom, gl.sort_totals), gl.sort_blocks, at<uint2>(geom, gl.msd_ranges),
                         counters + 2, stream, pub); }
    GS_LAUNCHED("depth sort");
    f.st->armed = true;  // (a launch that failed above publishes nothing: its slot is released without a wait)

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
    ea.xhist = two_level(g.gx, g.gy) && pa.rect_packed ? at<uint32_t>(geom, gl.emit_hist) : nullptr;
    // direct emission (k_emit_tiles): the scan also counts each block's instances per tile (in the depth
    // sort's tables, free by then)
    const bool direct = !ea.xhist && direct_emission_grid(g.gx, g.gy) && pa.rect_packed && !tile_sort_unfused();
    ea.thist = direct ? at<uint32_t>(geom, gl.sort_hist) : nullptr;
    // region emission (grids of 2049..kRegionMaxTiles tiles): chosen in bin_emit when its count table fits the
    // binning buffer (the two-level binning's column counts above stay the fallback)
    ea.chunks = pa.rect_packed && region_emission(g.gx, g.gy) ? region_chunks(P) : 0;
    ea.region_rows = region_rows(g.gx, g.gy);
    ea.ttotals = direct ? at<uint32_t>(geom, gl.sort_totals) : nullptr;
    ea.ntiles = g.tiles;
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

// Instance counts seen per (P, W, H): the capacity a speculative forward sizes
// its binning buffer by (gs_views_forward), and the configurations whose depth
// keys needed the 32-bit sort (never speculated).
struct CountHistory {
    std::mutex mu;
    std::unordered_map<uint64_t, uint32_t> max_k;
    std::unordered_map<uint64_t, bool> wide;
};
CountHistory& count_history() {
    static CountHistory h;
    return h;
}
uint64_t config_key(int P, int W, int H) {
    return ((uint64_t)(uint32_t)P << 32) ^ ((uint64_t)(uint32_t)W << 16) ^ (uint64_t)(uint32_t)H;
}
void note_count(int P, int W, int H, uint64_t K, bool wide) {
    CountHistory& h = count_history();
    std::lock_guard<std::mutex> g(h.mu);
    uint32_t& m = h.max_k[config_key(P, W, H)];
    const uint32_t k = K > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)K;
    m = k > m ? k : m;
    if (wide) h.wide[config_key(P, W, H)] = true;
}
// a speculative binning buffer's capacity: the largest count seen x 1.25 + 64k (0: no history, or
// a configuration that needed the 32-bit depth sort)
uint32_t spec_capacity(int P, int W, int H) {
    CountHistory& h = count_history();
    std::lock_guard<std::mutex> g(h.mu);
    const uint64_t k = config_key(P, W, H);
    auto it = h.max_k.find(k);
    if (it == h.max_k.end() || h.wide.count(k)) return 0;
    const uint64_t c = (uint64_t)it->second + it->second / 4 + 65536;
    return c > (uint64_t)std::numeric_limits<int>::max() ? 0u : (uint32_t)c;
}

// The host's copy of a forward's preprocess counters, after its event: the
// instance count, whether the visible depth keys span more bits than the short
// depth sort orders, the prefiltered error.  Releases the staging slot.
struct Counts {
    uint64_t K = 0;
    bool wide = false, prefilter_fail = false;
};
int read_counts(FwdState& f, Counts& c) {
    Staging* st = f.st;
    const auto t0 = std::chrono::steady_clock::now();
    if (!st->armed || !staging_wait(st))
        return set_error(GS_ERR_HIP, "the preprocess counters were not published (within 60 s)");
    std::atomic_thread_fence(std::memory_order_acquire);
    g_host_wait_ns.fetch_add(
        (long long)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0).count(),
        std::memory_order_relaxed);
    uint64_t K64 = 0;
    uint32_t kmax = 0, kmin_not = 0;
    for (int i = 0; i < kCounterSlots; ++i) {
        const uint32_t* q = st->host + kCounterStride * i;
        K64 += q[0];
        kmax = q[1] > kmax ? q[1] : kmax;
        kmin_not = q[2] > kmin_not ? q[2] : kmin_not;
    }
    c.K = K64;
    c.prefilter_fail = st->host[3] != 0;
    // (the MSD depth sort orders any key range: no 32-bit redo; `wide` stays for the forced fallback test)
    c.wide = false;
    (void)kmax;
    (void)kmin_not;
    staging_release(st, true);
    f.st = nullptr;
    note_count(f.gp.P, f.g.W, f.g.H, c.K, c.wide);
    return GS_OK;
}

// The emission, tile sort and tile ranges into the binning buffer `bin`, laid out for `K_layout`
// instances.  n_dev == nullptr: K_layout is the instance count; else (a speculative forward) the
// count is read on the device from the preprocess counters and capped at K_layout.
int bin_emit(FwdState& f, void* bin, uint32_t K_layout, const uint32_t* n_dev, hipStream_t stream) {
    const Grid& g = f.g;
    const bool debug = f.s.debug != 0;
    const ImgLayout il = img_layout(g.W, g.H);
    void* img = f.img;
    EmitArgs& ea = f.ea;
    const bool bwd = !f.gp.forward_only;
    const BinLayout bl = bin_layout((int)K_layout, g.tiles, bwd);
    ea.cap = n_dev ? K_layout : 0xFFFFFFFFu;
    const TileSortPlan plan = tile_sort_plan(g.tiles);
    if (ea.chunks && region_table_fits(bl, f.gp.P, g.tiles)) {
        // region emission: count table, scan, ranges + dispatch order, the lists (every store bounded by the
        // layout's instance count, exact binning or not: the counts come from the rects, not from K)
        ea.cap = K_layout;
        ea.ids_only = f.ids_only = !bwd && f.ids_ok;
        ea.pairs_out = at<uint2>(bin, bl.point_pairs);
        ea.rec_flags32 = bwd ? at<uint32_t>(bin, bl.rec_flags) : nullptr;
        ea.chunk_hist = at<uint32_t>(bin, bl.key0);
        ea.tile_start = at<uint32_t>(bin, bl.slot_gauss);
        ea.ttotals = at<uint32_t>(bin, bl.tile_count);
        ea.ranges = at<uint2>(img, il.ranges);
        ea.tile_order = at<uint32_t>(img, il.tile_order);
        { StageScope sc(ST_EMIT, stream); launch_region_emit(ea, stream); }
        GS_LAUNCHED("region emission");
        return GS_OK;
    }
    if (ea.xhist) {  // two-level binning (tile_sort_fused): column-ordered emission, row pass, ranges
        ea.ids_only = f.ids_only = !bwd && f.ids_ok;
        ea.tile_key = at<uint32_t>(bin, bl.key1);
        ea.pairs_out = at<uint2>(bin, bl.point_pairs == bl.pair1 ? bl.pair0 : bl.pair1);  // (not the row pass's output)
        ea.xtotals = at<uint32_t>(bin, bl.sort_totals);
        ea.tile_count = at<uint32_t>(bin, bl.tile_count);
        ea.ntiles = g.tiles;
        ea.rec_flags32 = bwd ? at<uint32_t>(bin, bl.rec_flags) : nullptr;
        { StageScope sc(ST_EMIT, stream); launch_emit_fused(ea, stream); }
        { StageScope sc(ST_TILE_SORT, stream);
        launch_row_pass(ea, K_layout, at<uint2>(bin, bl.point_pairs), at<uint32_t>(bin, bl.sort_hist), bl.sort_blocks,
                        at<uint2>(img, il.ranges), at<uint32_t>(img, il.tile_order), stream, n_dev); }
        GS_LAUNCHED("two-level binning");
        return GS_OK;
    }
    if (ea.thist) {  // direct emission: the lists, the tile ranges and the dispatch order in one launch
        ea.ids_only = f.ids_only = !bwd && f.ids_ok;
        ea.pairs_out = at<uint2>(bin, bl.point_pairs);
        ea.rec_flags32 = bwd ? at<uint32_t>(bin, bl.rec_flags) : nullptr;
        ea.ranges = at<uint2>(img, il.ranges);
        ea.tile_order = at<uint32_t>(img, il.tile_order);
        { StageScope sc(ST_EMIT, stream); launch_emit_tiles(ea, stream); }
        GS_LAUNCHED("direct emission");
        return GS_OK;
    }
    ea.tile_key = at<uint32_t>(bin, bl.key0);
    ea.slot_gauss = at<uint32_t>(bin, bl.slot_gauss);
    ea.rec_flags32 = bwd ? at<uint32_t>(bin, bl.rec_flags) : nullptr;
    { StageScope sc(ST_EMIT, stream); launch_scan_emit(ea, stream); }
    GS_LAUNCHED("emit");

    int tc;
    { StageScope sc(ST_TILE_SORT, stream);
    tc = tile_sort(at<uint32_t>(bin, bl.key0), at<uint32_t>(bin, bl.key1), at<uint2>(bin, bl.pair0),
                   at<uint2>(bin, bl.pair1), at<uint32_t>(bin, bl.slot_gauss), K_layout, plan.bits,
                   at<uint32_t>(bin, bl.sort_hist), at<uint32_t>(bin, bl.sort_totals), bl.sort_blocks, stream,
                   at<uint2>(img, il.ranges), at<uint32_t>(img, il.tile_order), g.tiles, n_dev); }
    GS_LAUNCHED("tile sort");
    if (!tile_sort_writes_ranges(g.tiles)) {
        StageScope sc(ST_RANGES, stream);
        launch_ranges(at<uint32_t>(bin, tc ? bl.key1 : bl.key0), (int)K_layout, at<uint2>(img, il.ranges), nullptr,
                      stream);
        GS_LAUNCHED("ranges");
    }
    return GS_OK;
}

// Second half: wait for the instance count (the reference's one host sync,
// rasterizer_impl.cu:236-239), then emission, tile sort and tile ranges.  On
// success *bin_out holds the binning buffer and *K_out the instance count.
// which_bin: the allocator's `which` for the binning buffer.
int bin_end(FwdState& f, gs_alloc_fn alloc, void* ctx, hipStream_t stream, void** bin_out, int* K_out,
            int which_bin = 1) {
    const Grid& g = f.g;
    const int P = f.gp.P;
    const bool debug = f.s.debug != 0;
    const GeomLayout gl = geom_layout(P);
    void* geom = f.geom;
    PreprocessArgs& pa = f.pa;
    EmitArgs& ea = f.ea;

    Counts c;
    int rc = read_counts(f, c);
    if (rc) return rc;
    if (c.prefilter_fail)
        return set_error(GS_ERR_PREFILTERED, "Point is filtered although prefiltered is set. This shouldn't happen!");
    if (c.K > (uint64_t)std::numeric_limits<int>::max())
        return set_error(GS_ERR_INVALID_ARG, "too many tile instances (%llu)", (unsigned long long)c.K);
    const uint32_t K = (uint32_t)c.K;
    if (c.wide || force_depth_keys32()) {
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

    void* bin = alloc(ctx, which_bin, bin_layout((int)K, g.tiles, !f.gp.forward_only).total);
    if (!bin) return set_error(GS_ERR_ALLOC, "allocator returned NULL for the binning buffer");
    *bin_out = bin;
    if (K == 0) return GS_OK;
    return bin_emit(f, bin, K, nullptr, stream);
}

// The blend (k_render_fwd) over a finished binning laid out for K_layout instances.
int render_launch(FwdState& f, void* bin, uint32_t K_layout, int order_ready, float* out_color, float* out_depth,
                  hipStream_t stream) {
    const Grid& g = f.g;
    const bool debug = f.s.debug != 0;
    const GeomLayout gl = geom_layout(f.gp.P);
    const ImgLayout il = img_layout(g.W, g.H);
    const BinLayout bl = bin_layout((int)K_layout, g.tiles, !f.gp.forward_only);
    void* geom = f.geom;
    void* img = f.img;
    RenderArgs ra;
    ra.bwd = f.gp.forward_only ? 0 : 1;
    ra.W = g.W; ra.H = g.H; ra.gx = g.gx; ra.gy = g.gy;
    ra.ranges = at<uint2>(img, il.ranges);
    ra.tile_order = at<uint32_t>(img, il.tile_order);
    ra.order_ready = order_ready;
    ra.point_pairs = at<uint2>(bin, bl.point_pairs);
    ra.point_ids = f.ids_only ? at<uint32_t>(bin, bl.point_pairs) : nullptr;
    ra.bwd_items = at<uint2>(bin, bl.bwd_items);
    ra.bwd_count = at<uint32_t>(img, il.bwd_count);
    ra.item_cap = (uint32_t)(4 * bl.nslots);
    ra.splat = at<Splat>(geom, gl.splat);
    ra.bg = f.s.bg;
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
    // (gs_params.aux_mask: the grey composited beside the colour, for a later gs_render_recolor)
    ra.aux_out = f.gp.aux_mask && !f.gp.forward_only ? at<float2>(img, il.aux) : nullptr;
    { StageScope sc(ST_RENDER_FWD, stream); launch_render_forward(ra, stream); }
    GS_LAUNCHED("render");
    return GS_OK;
}

// Everything of the forward up to (and including) tile ranges, in one call.
int bin_forward(const gs_settings* s, const Grid& g, const gs_params& gp, int* radii_out, int copy_colors,
                gs_alloc_fn alloc, void* ctx, hipStream_t stream, void** geom_out, void** img_out, void** bin_out,
                int* K_out) {
    FwdState f;
    f.ids_ok = false;  // (apply_weights reads the (Gaussian, slot) lists)
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

// One view's backward, in two parts: the gradient replay (k_render_bwd: the per-(slot, quadrant)
// records), then the per-Gaussian pass over those records, whose accumulated writes wait for
// writes_after.  R: the binning layout's instance count; slot_cap: a speculative forward's capacity
// (its slots end there), else ~0.
RenderBwdArgs replay_args(const gs_settings* s, const gs_params* gp, int R, const void* geom, const void* binning,
                          const void* img, const float* dL_dpix) {
    const int P = gp->P;
    const Grid g = make_grid(s);
    const GeomLayout gl = geom_layout(P);
    const ImgLayout il = img_layout(g.W, g.H);
    const BinLayout bl = bin_layout(R, g.tiles);
    RenderBwdArgs rb;
    rb.W = g.W; rb.H = g.H; rb.gx = g.gx; rb.gy = g.gy;
    rb.ranges = at<uint2>(img, il.ranges);
    rb.point_pairs = at<uint2>(binning, bl.point_pairs);
    rb.bwd_items = at<uint2>(binning, bl.bwd_items);
    rb.bwd_count = at<uint32_t>(const_cast<void*>(img), il.bwd_count);
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
    rb.records = at<float4>(const_cast<void*>(binning), bl.records);
    rb.rec_flags = at<uint8_t>(const_cast<void*>(binning), bl.rec_flags);
    rb.diag = diag_buffer(1, kDiagWords * 4 * bl.nslots);
    return rb;
}

int replay_view(const gs_settings* s, const gs_params* gp, int R, const void* geom, const void* binning,
                const void* img, const float* dL_dpix, hipStream_t stream) {
    if (gp->P == 0 || R <= 0) return GS_OK;
    const bool debug = s->debug != 0;
    const RenderBwdArgs rb = replay_args(s, gp, R, geom, binning, img, dL_dpix);
    { StageScope sc(ST_RENDER_BWD, stream); launch_render_backward(rb, stream); }
    GS_LAUNCHED("render backward");
    return GS_OK;
}

// the per-Gaussian pass's arguments for one view
// (the per-Gaussian "has a record" bytes: k_gauss_bwd skips every Gaussian without one (all of
// its gradients are zero), which is most of them (occluded behind saturated pixels); both zeroed by
// the forward: `touched` in preprocess, the flags with the tile ranges.  A second backward of the
// same forward finds the bytes of the first, which it sets again: the entries that get records
// depend on the forward alone)
GaussBwdArgs gauss_args(const gs_settings* s, const gs_params* gp, int R, const int* radii, const void* geom,
                        const void* binning, const gs_grads* o, uint32_t slot_cap) {
    const int P = gp->P;
    const Grid g = make_grid(s);
    const GeomLayout gl = geom_layout(P);
    const BinLayout bl = bin_layout(R, g.tiles);
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
    ga.rec_flags = R > 0 ? at<uint8_t>(const_cast<void*>(binning), bl.rec_flags) : nullptr;
    ga.touched = at<uint8_t>(const_cast<void*>(geom), gl.touched);
    ga.live_count = at<uint32_t>(const_cast<void*>(geom), gl.live_count);
    ga.live_list = at<uint32_t>(const_cast<void*>(geom), gl.live_list);
    ga.records = R > 0 ? at<float4>(const_cast<void*>(binning), bl.records) : nullptr;
    ga.dL_dmeans2D = o->dL_dmeans2D; ga.dL_dcolors = o->dL_dcolors; ga.dL_dopacity = o->dL_dopacity;
    ga.dL_dmeans3D = o->dL_dmeans3D; ga.dL_dcov3D = o->dL_dcov3D;
    ga.dL_dscales = o->dL_dscales; ga.dL_drot = o->dL_drotations;
    ga.pm3 = o->pitch_means3D > 0 ? o->pitch_means3D : 3;
    ga.pop = o->pitch_opacity > 0 ? o->pitch_opacity : 1;
    ga.psc = o->pitch_scales > 0 ? o->pitch_scales : 3;
    ga.prot = o->pitch_rotations > 0 ? o->pitch_rotations : 4;
    ga.acc = o->accumulate;
    ga.zeroed = o->zeroed & o->accumulate;
    ga.slot_cap = slot_cap;
    ga.grad_mask = o->grad_mask;
    ga.mask_bits = o->grad_mask ? o->mask_bits : 0u;
    ga.dirty = o->dirty_rows;
    ga.dL_dconic = o->dL_dconic;
    ga.diag = diag_buffer(2, kDiagWords * 4 * (size_t)(P / 256 + 1));
    return ga;
}

int backward_view(const gs_settings* s, const gs_params* gp, int R, const int* radii, const void* geom,
                  const void* binning, const void* img, const float* dL_dpix, const gs_grads* o, hipStream_t stream,
                  hipEvent_t writes_after, uint32_t slot_cap) {
    if (gp->P == 0) return GS_OK;
    const bool debug = s->debug != 0;
    int rc = replay_view(s, gp, R, geom, binning, img, dL_dpix, stream);
    if (rc) return rc;
    const GaussBwdArgs ga = gauss_args(s, gp, R, radii, geom, binning, o, slot_cap);
    { StageScope sc(ST_GAUSS_BWD, stream); launch_gauss_backward(ga, stream, writes_after); }
    GS_LAUNCHED("gaussian backward");
    return GS_OK;
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

int gs_timer_create(void** event) {
    if (!event) return set_error(GS_ERR_INVALID_ARG, "gs_timer_create: event is required");
    hipEvent_t e = nullptr;
    GS_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
    *event = e;
    return GS_OK;
}
int gs_timer_record(void* event, gs_stream_t stream) {
    if (!event) return set_error(GS_ERR_INVALID_ARG, "gs_timer_record: event is required");
    GS_HIP(hipEventRecord((hipEvent_t)event, (hipStream_t)stream));
    return GS_OK;
}
int gs_timer_elapsed_ms(void* start, void* end, float* ms) {
    if (!start || !end || !ms) return set_error(GS_ERR_INVALID_ARG, "gs_timer_elapsed_ms: start, end and ms are required");
    GS_HIP(hipEventSynchronize((hipEvent_t)end));
    GS_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)end));
    return GS_OK;
}
int gs_timer_destroy(void* event) {
    if (event) GS_HIP(hipEventDestroy((hipEvent_t)event));
    return GS_OK;
}

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

long long gs_host_wait_ns(void) { return g_host_wait_ns.load(std::memory_order_relaxed); }

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

int gs_activate_params(int P, const float* raw_opacity, const float* raw_scaling, const float* raw_rotation,
                       float* opacity, float* scaling, float* rotation, gs_stream_t stream) {
    if (P < 0 || (opacity && !raw_opacity) || (scaling && !raw_scaling) || (rotation && !raw_rotation))
        return set_error(GS_ERR_INVALID_ARG, "gs_activate_params: bad arguments");
    if (P == 0) return GS_OK;
    gs::launch_activate_params(P, raw_opacity, raw_scaling, raw_rotation, opacity, scaling, rotation,
                               (hipStream_t)stream);
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GS_OK : set_error(GS_ERR_HIP, "gs_activate_params launch failed: %s", hipGetErrorString(e));
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
        const Grid g = f.g;
        if (f.gp.P == 0) {  // rasterize_points.cu:57-72: zero outputs, empty buffers, no render
            alloc(alloc_ctx, 1, 0);
            GS_HIP(hipMemsetAsync(out_color, 0, sizeof(float) * 3 * (size_t)g.W * g.H, stream));
            GS_HIP(hipMemsetAsync(out_depth, 0, sizeof(float) * (size_t)g.W * g.H, stream));
            return GS_OK;
        }
        void* bin = nullptr;
        int K = 0;
        int rc = bin_end(f, alloc, alloc_ctx, stream, &bin, &K);
        if (rc) return rc;
        rc = render_launch(f, bin, (uint32_t)K, K > 0 && (tile_sort_writes_ranges(g.tiles) || f.ea.xhist) ? 1 : 0,
                           out_color, out_depth, stream);
        if (rc) return rc;
        *num_rendered = K;
        return GS_OK;
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

void gs_rasterize_forward_release(gs_forward_state* state) { delete state; }

int gs_render_recolor(const gs_settings* s, int P, int num_rendered, const void* geom, const void* binning,
                      const void* img, const float* colors, void* img_out, float* out_color, float* out_depth,
                      const uint8_t* src_aux_mask, gs_stream_t stream_) {
    try {
        hipStream_t stream = (hipStream_t)stream_;
        if (!s || P < 0 || num_rendered < 0 || !geom || !img || !img_out || !out_color || !out_depth ||
            (P > 0 && !colors) || (num_rendered > 0 && !binning))
            return set_error(GS_ERR_INVALID_ARG, "gs_render_recolor: bad arguments");
        const bool debug = s->debug != 0;
        const Grid g = make_grid(s);
        if (g.W <= 0 || g.H <= 0) return set_error(GS_ERR_INVALID_ARG, "gs_render_recolor: bad image size");
        const ImgLayout il = img_layout(g.W, g.H);
        // the blend's per-pixel/per-tile outputs into img_out (the source render's backward still reads
        // its own); tile_last is accumulated by atomicMax: zeroed with the rest of the tail
        GS_HIP(hipMemsetAsync(at<uint8_t>(img_out, il.counters), 0, il.total - il.counters, stream));
        if (P == 0 || num_rendered == 0) {
            // no list: every pixel is T = 1 over the background (the blend of empty ranges)
            GS_HIP(hipMemsetAsync(at<uint8_t>(img_out, il.ranges), 0, 8 * (size_t)g.tiles, stream));
        }
        const GeomLayout gl = geom_layout(P);
        const BinLayout bl = bin_layout(num_rendered, g.tiles, true);
        RenderArgs ra;
        ra.bwd = 0;
        ra.W = g.W; ra.H = g.H; ra.gx = g.gx; ra.gy = g.gy;
        const bool empty = P == 0 || num_rendered == 0;
        ra.ranges = at<uint2>(empty ? img_out : img, il.ranges);
        // (read only: the empty case's own order goes to img_out)
        ra.tile_order = at<uint32_t>(empty ? img_out : const_cast<void*>(img), il.tile_order);
        ra.order_ready = empty ? 0 : 1;  // (the source forward left its dispatch order; an empty one gets one)
        ra.point_pairs = empty ? nullptr : at<uint2>(binning, bl.point_pairs);
        ra.point_ids = nullptr;
        ra.splat = at<Splat>(geom, gl.splat);
        ra.bg = s->bg;
        ra.final_T = at<float>(img_out, il.final_T);
        ra.n_contrib = at<uint32_t>(img_out, il.n_contrib);
        ra.tile_last = at<uint32_t>(img_out, il.tile_last);
        ra.quad_last = at<uint32_t>(img_out, il.quad_last);
        ra.ckpt = nullptr; ra.used = nullptr; ra.bwd_items = nullptr; ra.bwd_count = nullptr; ra.item_cap = 0;
        ra.out_color = out_color;
        ra.out_depth = out_depth;
        ra.touched = nullptr;
        ra.diag = nullptr;
        ra.colors = colors;
        if (src_aux_mask && !empty) {
            // the colours against the source forward's aux grey, on the device (a flag word of img_out's
            // counters, zeroed above); equal: the blend composes the image from that forward's sums
            uint32_t* flag = at<uint32_t>(img_out, il.counters);
            launch_aux_match(P, colors, src_aux_mask, flag, stream);
            GS_LAUNCHED("recolor aux check");
            ra.aux_match = flag;
            ra.aux_src = at<float2>(const_cast<void*>(img), il.aux);
            ra.final_T_src = at<float>(const_cast<void*>(img), il.final_T);
        }
        { StageScope sc(ST_RENDER_FWD, stream); launch_render_forward(ra, stream); }
        GS_LAUNCHED("recolor render");
        return GS_OK;
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

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
    o.zeroed = 0;
    o.pitch_means3D = o.pitch_opacity = o.pitch_scales = o.pitch_rotations = 0;
    o.dirty_rows = nullptr;
    gs_params g2 = g;
    g2.M = M;  // dL_dsh is [P,M,3] even when shs is absent (then all zero)
    return gs_rasterize_backward_ex(s, &g2, R, radii, geom, binning, img, dL_dpix, &o, stream);
}

// the views' per-Gaussian passes can run as one (launch_gauss_backward_views): one scene (same P, rows,
// SH layout), the same parameter-shaped outputs, every view after the first adding into all of them
static bool passes_mergeable(int n, const gs_settings* const* s, const gs_params* const* gpv, const gs_grads* const* o) {
    const uint32_t params = GS_ACC_OPACITY | GS_ACC_MEANS3D | GS_ACC_SCALES | GS_ACC_ROTATIONS;
    const gs_params& p0 = *gpv[0];
    const gs_grads* g0 = o[0];
    if (p0.P == 0 || g0->dL_dcov3D || p0.cov3D_precomp) return false;
    for (int v = 1; v < n; ++v) {
        const gs_params& p = *gpv[v];
        const gs_grads* g = o[v];
        if (p.P != p0.P || p.index != p0.index || p.M != p0.M || p.sh_dc != p0.sh_dc || p.sh_rest != p0.sh_rest ||
            p.means3D != p0.means3D || p.opacities != p0.opacities || p.scales != p0.scales ||
            p.rotations != p0.rotations || p.activation != p0.activation || p.sh_half != p0.sh_half ||
            s[v]->sh_degree != s[0]->sh_degree)
            return false;
        if (g->dL_dopacity != g0->dL_dopacity || g->dL_dmeans3D != g0->dL_dmeans3D ||
            g->dL_dscales != g0->dL_dscales || g->dL_drotations != g0->dL_drotations ||
            g->dL_dsh_dc != g0->dL_dsh_dc || g->dL_dsh_rest != g0->dL_dsh_rest || g->dL_dcov3D || g->grad_mask != g0->grad_mask ||
            g->mask_bits != g0->mask_bits || g->pitch_means3D != g0->pitch_means3D ||
            g->pitch_opacity != g0->pitch_opacity || g->pitch_scales != g0->pitch_scales ||
            g->pitch_rotations != g0->pitch_rotations || g->dsh_dc_stride != g0->dsh_dc_stride ||
            g->dsh_rest_stride != g0->dsh_rest_stride)
            return false;
        if ((g->accumulate & params) != params || (g0->dL_dsh_dc && !(g->accumulate & GS_ACC_SH))) return false;
    }
    return true;
}

// the argument checks of a backward (gs_rasterize_backward_ex, gs_views_backward)
static int validate_backward(const gs_settings* s, const gs_params* gp, int R, const int* radii, const void* geom,
                      const void* binning, const void* img, const float* dL_dpix, const gs_grads* o) {
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
    if (!o->dL_dmeans2D || !o->dL_dopacity || !o->dL_dmeans3D || !o->dL_dscales || !o->dL_drotations ||
        (gp->M > 1 && o->dL_dsh_dc && !o->dL_dsh_rest))
        return set_error(GS_ERR_INVALID_ARG, "gradient outputs are required");
    if (R > 0 && !binning) return set_error(GS_ERR_INVALID_ARG, "binning buffer is required when num_rendered > 0");
    if (o->pitch_means3D < 0 || o->pitch_opacity < 0 || o->pitch_scales < 0 || o->pitch_rotations < 0 ||
        (o->pitch_means3D > 0 && o->pitch_means3D < 3) || (o->pitch_scales > 0 && o->pitch_scales < 3) ||
        (o->pitch_rotations > 0 && (o->pitch_rotations < 4 || o->pitch_rotations % 4)) ||
        (reinterpret_cast<uintptr_t>(o->dL_drotations) & 15))
        return set_error(GS_ERR_INVALID_ARG, "gradient row pitches: >= the row width, dL_drotations rows 16-B aligned");
    return GS_OK;
}

int gs_rasterize_backward_ex(const gs_settings* s, const gs_params* gp, int R, const int* radii, const void* geom,
                             const void* binning, const void* img, const float* dL_dpix, const gs_grads* o,
                             gs_stream_t stream_) {
    try {
        const int rc = validate_backward(s, gp, R, radii, geom, binning, img, dL_dpix, o);
        if (rc || gp->P == 0) return rc;
        return backward_view(s, gp, R, radii, geom, binning, img, dL_dpix, o, (hipStream_t)stream_,
                             (hipEvent_t)o->writes_after, 0xFFFFFFFFu);
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

int gs_rasterize_backward_replay(const gs_settings* s, const gs_params* gp, int R, const int* radii,
                                 const void* geom, const void* binning, const void* img, const float* dL_dpix,
                                 const gs_grads* o, gs_stream_t stream_) {
    try {
        const int rc = validate_backward(s, gp, R, radii, geom, binning, img, dL_dpix, o);
        if (rc || gp->P == 0) return rc;
        return replay_view(s, gp, R, geom, binning, img, dL_dpix, (hipStream_t)stream_);
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

int gs_rasterize_backward_passes(int n, const gs_settings* const* s, const gs_params* const* gp, const int* R,
                                 const int* const* radii, const void* const* geom, const void* const* binning,
                                 const gs_grads* const* o, gs_stream_t stream_) {
    try {
        if (n < 1 || n > GS_MAX_VIEWS || !s || !gp || !R || !radii || !geom || !binning || !o)
            return set_error(GS_ERR_INVALID_ARG, "gs_rasterize_backward_passes: 1 <= n <= %d views and every array "
                             "are required", GS_MAX_VIEWS);
        for (int v = 0; v < n; ++v) {
            if (!s[v] || !gp[v] || !o[v]) return set_error(GS_ERR_INVALID_ARG, "view %d: settings, params, grads", v);
            if (gp[v]->P > 0 && (!geom[v] || !radii[v] || (R[v] > 0 && !binning[v])))
                return set_error(GS_ERR_INVALID_ARG, "view %d: buffers and radii are required", v);
        }
        hipStream_t stream = (hipStream_t)stream_;
        const bool debug = s[0]->debug != 0;
        GaussBwdArgs ga[GS_MAX_VIEWS];
        for (int v = 0; v < n; ++v)
            ga[v] = gauss_args(s[v], gp[v], R[v], radii[v], geom[v], binning[v], o[v], 0xFFFFFFFFu);
        if (n > 1 && passes_mergeable(n, s, gp, o)) {
            const int chunk = gauss_backward_max_views();
            for (int v0 = 0; v0 < n; v0 += chunk) {
                const int nv = std::min(chunk, n - v0);
                { StageScope sc(ST_GAUSS_BWD, stream);
                launch_gauss_backward_views(ga + v0, nv, stream, v0 == 0 ? (hipEvent_t)o[0]->writes_after : nullptr); }
                GS_LAUNCHED("gaussian backward (views)");
            }
            return GS_OK;
        }
        for (int v = 0; v < n; ++v) {  // one pass per view, in order
            if (gp[v]->P == 0) continue;
            { StageScope sc(ST_GAUSS_BWD, stream);
            launch_gauss_backward(ga[v], stream, (hipEvent_t)o[v]->writes_after); }
            GS_LAUNCHED("gaussian backward");
        }
        return GS_OK;
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

}  // extern "C"

// ---------------------------------------------------------------------
// gs_views: the forwards and backwards of a batch of views of one scene
// (DGE renders a batch of edited views per step, threestudio/systems/DGE.py:170-239)
// ---------------------------------------------------------------------
namespace {
// ordering events of the views' backward calls, reused across batches
// The pool's events only order streams on the device (hipStreamWaitEvent; the host never waits on them):
// no system-scope fence, which a record otherwise pays with an L2 writeback for the host's view
#ifndef GS_POOL_EVENT_FLAGS
#define GS_POOL_EVENT_FLAGS (hipEventDisableTiming | hipEventDisableSystemFence)
#endif
struct EventPool {
    std::mutex mu;
    std::vector<hipEvent_t> free;
    hipEvent_t get() {
        {
            std::lock_guard<std::mutex> g(mu);
            if (!free.empty()) {
                hipEvent_t e = free.back();
                free.pop_back();
                return e;
            }
        }
        hipEvent_t e = nullptr;
        if (hipEventCreateWithFlags(&e, GS_POOL_EVENT_FLAGS) != hipSuccess) return nullptr;
        return e;
    }
    void put(hipEvent_t e) {
        if (!e) return;
        std::lock_guard<std::mutex> g(mu);
        free.push_back(e);
    }
};
EventPool& event_pool() {
    static EventPool p;
    return p;
}

bool can_speculate(const FwdState& f) {
    const Grid& g = f.g;
    if (f.s.debug || force_depth_keys32()) return false;
    if (tile_sort_writes_ranges(g.tiles)) return true;  // single-pass tile sort
    return two_level(g.gx, g.gy);  // two-level binning
}
}  // namespace

struct gs_views {
    int n = 0;
    FwdState f[GS_MAX_VIEWS];
    void* bin[GS_MAX_VIEWS] = {};
    uint32_t layout[GS_MAX_VIEWS] = {};  // instances the binning buffer is laid out for
    int spec[GS_MAX_VIEWS] = {};         // 1: capacity-sized, count checked by gs_views_check
    long long K[GS_MAX_VIEWS] = {};      // instance count, -1 until the host knows it
    hipEvent_t ev[GS_MAX_VIEWS] = {};    // the end of each view's work (forward, or per-Gaussian backward pass)
    hipEvent_t fork = nullptr;           // the caller's stream, before the views' work
    ~gs_views() {
        for (int v = 0; v < GS_MAX_VIEWS; ++v) event_pool().put(ev[v]);
        event_pool().put(fork);
    }
};

namespace {
// the views' streams wait for the caller's stream `join` (a null handle is the legacy default stream)
int fork_from(gs_views* h, hipStream_t join, const gs_stream_t* streams) {
    bool other = false;
    for (int v = 0; v < h->n; ++v) other |= (hipStream_t)streams[v] != join;
    if (!other) return GS_OK;
    if (!h->fork && !(h->fork = event_pool().get())) return set_error(GS_ERR_HIP, "could not create an event");
    GS_HIP(hipEventRecord(h->fork, join));
    for (int v = 0; v < h->n; ++v) {
        bool seen = (hipStream_t)streams[v] == join;
        for (int u = 0; u < v && !seen; ++u) seen = streams[u] == streams[v];
        if (!seen) GS_HIP(hipStreamWaitEvent((hipStream_t)streams[v], h->fork, 0));
    }
    return GS_OK;
}
// `join` waits for every view stream's work so far
int join_into(gs_views* h, hipStream_t join, const gs_stream_t* streams) {
    for (int v = 0; v < h->n; ++v) {
        bool seen = (hipStream_t)streams[v] == join;
        for (int u = 0; u < v && !seen; ++u) seen = streams[u] == streams[v];
        if (seen) continue;
        if (!h->ev[v] && !(h->ev[v] = event_pool().get())) return set_error(GS_ERR_HIP, "could not create an event");
        GS_HIP(hipEventRecord(h->ev[v], (hipStream_t)streams[v]));
        GS_HIP(hipStreamWaitEvent(join, h->ev[v], 0));
    }
    return GS_OK;
}
}  // namespace

extern "C" {

int gs_views_forward(int n, const gs_settings* const* s, const gs_params* const* gp, float* const* out_color,
                     float* const* out_depth, int* const* radii, int mode, gs_alloc_fn alloc, void* alloc_ctx,
                     const gs_stream_t* streams, gs_stream_t join_, gs_views** out) {
    try {
        if (!out) return set_error(GS_ERR_INVALID_ARG, "out is required");
        *out = nullptr;
        if (n < 1 || n > GS_MAX_VIEWS || !s || !gp || !out_color || !out_depth || !radii || !alloc || !streams)
            return set_error(GS_ERR_INVALID_ARG, "gs_views_forward: 1 <= n <= %d views and every array are required",
                             GS_MAX_VIEWS);
        if (mode != GS_VIEWS_EXACT && mode != GS_VIEWS_SPECULATE)
            return set_error(GS_ERR_INVALID_ARG, "gs_views_forward: unknown mode %d", mode);
        std::unique_ptr<gs_views> h(new gs_views());
        h->n = n;
        // one buffer for every view's geometry and image state (and the binning of the speculated views)
        size_t off_geom[GS_MAX_VIEWS] = {}, off_img[GS_MAX_VIEWS] = {}, off_bin[GS_MAX_VIEWS] = {};
        size_t total = 0;
        for (int v = 0; v < n; ++v) {
            int rc = validate_params(s[v], gp[v]);
            if (rc) return rc;
            if (!out_color[v] || !out_depth[v]) return set_error(GS_ERR_INVALID_ARG, "out_color/out_depth are required");
            FwdState& f = h->f[v];
            f.s = *s[v];
            f.gp = *gp[v];
            f.g = make_grid(s[v]);
            f.radii = radii[v];
            h->K[v] = -1;
            const int P = f.gp.P;
            if (P == 0) continue;
            off_geom[v] = total;
            total = align_up(total + geom_layout(P).total);
            off_img[v] = total;
            total = align_up(total + img_layout(f.g.W, f.g.H).total);
            const uint32_t cap = mode == GS_VIEWS_SPECULATE && can_speculate(f) ? spec_capacity(P, f.g.W, f.g.H) : 0u;
            if (cap) {
                h->spec[v] = 1;
                h->layout[v] = cap;
                off_bin[v] = total;
                total = align_up(total + bin_layout((int)cap, f.g.tiles, !f.gp.forward_only).total);
            }
        }
        char* base = static_cast<char*>(alloc(alloc_ctx, 0, total));
        if (total && !base) return set_error(GS_ERR_ALLOC, "allocator returned NULL for the views' buffers");
        hipStream_t join = (hipStream_t)join_;
        int rc = fork_from(h.get(), join, streams);  // the views' streams start after the caller's work
        if (rc) return rc;
        // first halves on every view's stream: nothing waits for any count yet.  Breadth first: every
        // view's preprocess is enqueued before any view's depth sort, so the views' chains start together
        // (view by view, the last view's preprocess started ~200 us of host issue after the first's and
        // the forward phase ended with that view).  The preprocesses run concurrently on purpose: they read
        // the same parameters (one HBM read serves the views from the caches) — each view's preprocess
        // waiting for the previous one's measured 2616 vs 2925 renders/s (profiles/r05/ab_views_stagger.txt)
        for (int v = 0; v < n; ++v) {
            FwdState& f = h->f[v];
            if (f.gp.P == 0) continue;
            hipStream_t stream = (hipStream_t)streams[v];
            const bool debug = f.s.debug != 0;
            rc = bin_prepare_in(f, 1, base + off_geom[v], base + off_img[v], stream);
            if (rc) return rc;
            { StageScope sc(ST_PREPROCESS, stream); launch_preprocess(f.pa, stream); }
            GS_LAUNCHED("preprocess");
        }
        for (int v = 0; v < n; ++v) {
            FwdState& f = h->f[v];
            if (f.gp.P == 0) continue;
            rc = bin_after_preprocess(f, (hipStream_t)streams[v]);
            if (rc) return rc;
        }
        // second halves: a speculated view's binning runs on the device count, capped at its capacity;
        // the others wait for their count here (the reference's sync, rasterizer_impl.cu:236-239)
        for (int v = 0; v < n; ++v) {
            FwdState& f = h->f[v];
            hipStream_t stream = (hipStream_t)streams[v];
            const Grid& g = f.g;
            if (f.gp.P == 0) {  // rasterize_points.cu:57-72
                GS_HIP(hipMemsetAsync(out_color[v], 0, sizeof(float) * 3 * (size_t)g.W * g.H, stream));
                GS_HIP(hipMemsetAsync(out_depth[v], 0, sizeof(float) * (size_t)g.W * g.H, stream));
                h->K[v] = 0;
                continue;
            }
            if (h->spec[v]) {
                h->bin[v] = base + off_bin[v];
                const uint32_t* counters = at<uint32_t>(f.img, img_layout(g.W, g.H).counters);
                rc = bin_emit(f, h->bin[v], h->layout[v], counters, stream);
                if (rc) return rc;
                rc = render_launch(f, h->bin[v], h->layout[v], tile_sort_writes_ranges(g.tiles) || f.ea.xhist ? 1 : 0,
                                   out_color[v], out_depth[v], stream);
            } else {
                int K = 0;
                rc = bin_end(f, alloc, alloc_ctx, stream, &h->bin[v], &K, 16 + v);
                if (rc) return rc;
                h->K[v] = K;
                h->layout[v] = (uint32_t)K;
                rc = render_launch(f, h->bin[v], (uint32_t)K,
                                   K > 0 && (tile_sort_writes_ranges(g.tiles) || f.ea.xhist) ? 1 : 0, out_color[v],
                                   out_depth[v], stream);
            }
            if (rc) return rc;
        }
        rc = join_into(h.get(), join, streams);
        if (rc) return rc;
        *out = h.release();
        return GS_OK;
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

int gs_views_check(gs_views* h, int* num_rendered) {
    if (!h) return set_error(GS_ERR_INVALID_ARG, "gs_views_check: handle is NULL");
    int rc = GS_OK;
    int first_bad = -1;
    for (int v = 0; v < h->n; ++v) {
        FwdState& f = h->f[v];
        if (h->K[v] < 0 && f.st) {
            Counts c;
            const int r = read_counts(f, c);
            if (r) return r;
            h->K[v] = (long long)c.K;
            if (c.prefilter_fail && rc != GS_ERR_PREFILTERED)
                rc = set_error(GS_ERR_PREFILTERED, "Point is filtered although prefiltered is set. This shouldn't happen!");
            if ((c.K > h->layout[v] || c.wide) && first_bad < 0) first_bad = v;
        }
        if (num_rendered) num_rendered[v] = (int)(h->K[v] < 0 ? 0 : std::min<long long>(h->K[v], 0x7FFFFFFF));
    }
    if (rc) return rc;
    if (first_bad >= 0)
        return set_error(GS_ERR_RETRY, "view %d: %lld tile instances exceed the speculative binning capacity %u (or "
                         "its depth keys need the 32-bit sort): render the views again", first_bad,
                         h->K[first_bad], h->layout[first_bad]);
    return GS_OK;
}

bool views_mergeable(const gs_views* h, const gs_grads* const* o) {
    const gs_settings* s[GS_MAX_VIEWS];
    const gs_params* gp[GS_MAX_VIEWS];
    for (int v = 0; v < h->n; ++v) {
        s[v] = &h->f[v].s;
        gp[v] = &h->f[v].gp;
    }
    return passes_mergeable(h->n, s, gp, o);
}

int gs_views_backward(gs_views* h, const float* const* dL_dpix, const gs_grads* const* grads,
                      const gs_stream_t* streams, void* writes_after, gs_stream_t join_) {
    try {
        if (!h || !dL_dpix || !grads || !streams)
            return set_error(GS_ERR_INVALID_ARG, "gs_views_backward: handle, dL_dpix, grads and streams are required");
        hipStream_t join = (hipStream_t)join_;
        for (int v = 0; v < h->n; ++v) {
            FwdState& f = h->f[v];
            if (f.gp.forward_only && f.gp.P > 0)
                return set_error(GS_ERR_INVALID_ARG, "gs_views_backward: view %d was rendered forward_only", v);
            const int rc = validate_backward(&f.s, &f.gp, (int)h->layout[v], f.radii, f.geom, h->bin[v], f.img,
                                             dL_dpix[v], grads[v]);
            if (rc) return rc;
        }
        if (h->n > 1 && views_mergeable(h, grads)) {
            // every view's replay, then ONE per-Gaussian pass over all of them (chunks of
            // gauss_backward_max_views() views, in view order) on the first view's stream
            hipStream_t s0 = (hipStream_t)streams[0];
            const bool debug = h->f[0].s.debug != 0;
            hipStream_t stream = s0;  // (GS_LAUNCHED)
            const int chunk = gauss_backward_max_views();
            // one pass for the batch: its first half (the live set from the forwards' touched bytes) runs
            // on s0 right behind view 0's replay (or the merged replay)
            const bool split = h->n <= chunk;
            GaussBwdArgs ga[GS_MAX_VIEWS];
            if (split)
                for (int v = 0; v < h->n; ++v) {
                    FwdState& f = h->f[v];
                    ga[v] = gauss_args(&f.s, &f.gp, (int)h->layout[v], f.radii, f.geom, h->bin[v], grads[v],
                                       h->spec[v] ? h->layout[v] : 0xFFFFFFFFu);
                }
            // Views on several streams: every replay in ONE launch on s0 (k_render_bwd_views), so the backward
            // makes no cross-stream hop — the fork to the views' streams and their join back before the
            // per-Gaussian pass each cost ~10 us of queue time (tools/probes/queue_gap.hip).  Views on one
            // stream keep one launch per view (no hop either way; the per-launch stage times stay per view).
            // Off with the per-wave diagnostics (their buffer is per launch) or DGE_AMD_REPLAY_MERGE=0.
            bool merge = false;
            for (int v = 1; v < h->n; ++v) merge |= streams[v] != streams[0];
            if (merge) {
                const char* e = getenv("DGE_AMD_REPLAY_MERGE");
                merge = !(e && !strcmp(e, "0"));
            }
            RenderBwdArgs rbs[GS_MAX_VIEWS];
            int nr = 0;
            for (int v = 0; merge && v < h->n; ++v) {
                FwdState& f = h->f[v];
                if (f.gp.P == 0 || h->layout[v] == 0) continue;
                rbs[nr] = replay_args(&f.s, &f.gp, (int)h->layout[v], f.geom, h->bin[v], f.img, dL_dpix[v]);
                merge = rbs[nr++].diag == nullptr;
            }
            if (merge) {
                if (s0 != join) {  // (only s0 starts after the caller's work)
                    if (!h->fork && !(h->fork = event_pool().get())) return set_error(GS_ERR_HIP, "could not create an event");
                    GS_HIP(hipEventRecord(h->fork, join));
                    GS_HIP(hipStreamWaitEvent(s0, h->fork, 0));
                }
                // the live-set pass (it reads the forwards' outputs only) on the first other view stream, beside the
                // merged replay instead of after it on s0: c2 3089 -> 3181 renders/s with the merge
                // (profiles/r06/queues/ab_merged_replay.txt); DGE_AMD_LIVE_SIDE=0: after it
                int side = -1;
                if (split) {
                    const char* e = getenv("DGE_AMD_LIVE_SIDE");
                    for (int v = 1; !(e && !strcmp(e, "0")) && side < 0 && v < h->n; ++v)
                        if (streams[v] != streams[0]) side = v;
                }
                if (side > 0) {
                    hipStream_t ss = (hipStream_t)streams[side];
                    if (!h->ev[0] && !(h->ev[0] = event_pool().get())) return set_error(GS_ERR_HIP, "could not create an event");
                    GS_HIP(hipEventRecord(h->ev[0], s0));
                    GS_HIP(hipStreamWaitEvent(ss, h->ev[0], 0));
                    { StageScope sc(ST_GAUSS_LIVE, ss); launch_gauss_live_views(ga, h->n, ss, (hipEvent_t)writes_after); }
                    hipStream_t stream = ss;  // (GS_LAUNCHED)
                    GS_LAUNCHED("gaussian live set (views, side stream)");
                    if (!h->ev[side] && !(h->ev[side] = event_pool().get())) return set_error(GS_ERR_HIP, "could not create an event");
                    GS_HIP(hipEventRecord(h->ev[side], ss));
                }
                if (nr) {
                    // (the grids a quarter of the item bounds: ~3.7x the real items at c2; DGE_AMD_REPLAY_GRID_DIV
                    // forces smaller ones, so the tests run the blocks' item loop)
                    const char* d = getenv("DGE_AMD_REPLAY_GRID_DIV");
                    const uint32_t div = d ? (uint32_t)std::max(1, atoi(d)) : 4u;
                    { StageScope sc(ST_RENDER_BWD, s0); launch_render_backward_views(rbs, nr, div, s0); }
                    GS_LAUNCHED("render backward (views)");
                }
                if (side > 0) {
                    GS_HIP(hipStreamWaitEvent(s0, h->ev[side], 0));
                } else if (split) {
                    { StageScope sc(ST_GAUSS_LIVE, s0); launch_gauss_live_views(ga, h->n, s0, (hipEvent_t)writes_after); }
                    GS_LAUNCHED("gaussian live set (views)");
                }
            } else {
                int rc0 = fork_from(h, join, streams);  // (the image gradients come from the caller's stream)
                if (rc0) return rc0;
            }
            for (int v = 0; !merge && v < h->n; ++v) {
                FwdState& f = h->f[v];
                hipStream_t sv = (hipStream_t)streams[v];
                int rc = replay_view(&f.s, &f.gp, (int)h->layout[v], f.geom, h->bin[v], f.img, dL_dpix[v], sv);
                if (rc) return rc;
                // (before view 0's replay instead, beside the others' replays: 2861-2877 vs 2882-2898
                // renders/s, profiles/r05/ab_scan_shape_live_first.txt)
                if (split && v == 0) {
                    { StageScope sc(ST_GAUSS_LIVE, s0); launch_gauss_live_views(ga, h->n, s0, (hipEvent_t)writes_after); }
                    GS_LAUNCHED("gaussian live set (views)");
                }
                if (sv != s0) {
                    if (!h->ev[v] && !(h->ev[v] = event_pool().get())) return set_error(GS_ERR_HIP, "could not create an event");
                    GS_HIP(hipEventRecord(h->ev[v], sv));
                    GS_HIP(hipStreamWaitEvent(s0, h->ev[v], 0));
                }
            }
            if (split) {
                { StageScope sc(ST_GAUSS_BWD, s0);
                launch_gauss_bwd_live_views(ga, h->n, s0, ga[0].dirty ? nullptr : (hipEvent_t)writes_after); }
                GS_LAUNCHED("gaussian backward (views)");
            }
            for (int v0 = 0; !split && v0 < h->n; v0 += chunk) {
                const int nv = std::min(chunk, h->n - v0);
                for (int v = 0; v < nv; ++v) {
                    FwdState& f = h->f[v0 + v];
                    ga[v] = gauss_args(&f.s, &f.gp, (int)h->layout[v0 + v], f.radii, f.geom, h->bin[v0 + v],
                                       grads[v0 + v], h->spec[v0 + v] ? h->layout[v0 + v] : 0xFFFFFFFFu);
                }
                { StageScope sc(ST_GAUSS_BWD, s0);
                launch_gauss_backward_views(ga, nv, s0, v0 == 0 ? (hipEvent_t)writes_after : nullptr); }
                GS_LAUNCHED("gaussian backward (views)");
            }
            if (s0 != join) {
                if (!h->ev[0] && !(h->ev[0] = event_pool().get())) return set_error(GS_ERR_HIP, "could not create an event");
                GS_HIP(hipEventRecord(h->ev[0], s0));
                GS_HIP(hipStreamWaitEvent(join, h->ev[0], 0));
            }
            return GS_OK;
        }
        int rc0 = fork_from(h, join, streams);  // (the image gradients come from the caller's stream)
        if (rc0) return rc0;
        int prev = -1;
        for (int v = 0; v < h->n; ++v) {
            FwdState& f = h->f[v];
            if (f.gp.P == 0) continue;
            hipStream_t sv = (hipStream_t)streams[v];
            // accumulated writes in view order: view v's per-Gaussian pass after view prev's
            hipEvent_t wa = prev < 0 ? (hipEvent_t)writes_after
                                     : (streams[prev] != streams[v] ? h->ev[prev] : nullptr);
            int rc = backward_view(&f.s, &f.gp, (int)h->layout[v], f.radii, f.geom, h->bin[v], f.img, dL_dpix[v],
                                   grads[v], sv, wa, h->spec[v] ? h->layout[v] : 0xFFFFFFFFu);
            if (rc) return rc;
            if (!h->ev[v] && !(h->ev[v] = event_pool().get())) return set_error(GS_ERR_HIP, "could not create an event");
            GS_HIP(hipEventRecord(h->ev[v], sv));
            prev = v;
        }
        for (int v = 0; v < h->n; ++v)
            if (h->ev[v] && streams[v] != join_) GS_HIP(hipStreamWaitEvent(join, h->ev[v], 0));
        return GS_OK;
    } catch (const std::exception& e) {
        return set_error(GS_ERR_INVALID_ARG, "exception: %s", e.what());
    } catch (...) {
        return set_error(GS_ERR_INVALID_ARG, "unknown exception");
    }
}

int gs_views_overflow(const gs_views* h, uint8_t* flag, gs_stream_t stream_) {
    hipStream_t stream = (hipStream_t)stream_;
    if (!h || !flag) return set_error(GS_ERR_INVALID_ARG, "gs_views_overflow: handle and flag are required");
    OverflowArgs a;
    a.n = h->n;
    for (int v = 0; v < h->n; ++v) {
        const FwdState& f = h->f[v];
        if (!h->spec[v] || f.gp.P == 0) continue;
        a.counters[v] = at<uint32_t>(f.img, img_layout(f.g.W, f.g.H).counters);
        a.cap[v] = h->layout[v];
    }
    launch_views_overflow(a, flag, stream);
    const bool debug = false;
    GS_LAUNCHED("views overflow flag");
    return GS_OK;
}

void* gs_views_buffer(const gs_views* h, int v, int which) {
    if (!h || v < 0 || v >= h->n) return nullptr;
    switch (which) {
        case 0: return h->f[v].geom;
        case 1: return h->bin[v];
        case 2: return h->f[v].img;
        default: return nullptr;
    }
}

long long gs_views_layout(const gs_views* h, int v) { return (!h || v < 0 || v >= h->n) ? -1 : (long long)h->layout[v]; }

void gs_views_release(gs_views* h) { delete h; }

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
        gs_params gp = make_params(P, M, means3D, shs, weights, opacities, scales, rotations, cov3D_precomp);
        gp.forward_only = 1;  // (no blend, no backward: the binning only)
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
        const BinLayout bl = bin_layout(K, g.tiles, false);
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
