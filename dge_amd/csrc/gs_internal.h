// gs_internal.h — buffer layouts and kernel launchers shared by the HIP
// translation units of libgs_raster.so.  Not part of the C ABI.
//
// Buffer design (MI355X-first; the reference's GeometryState / BinningState /
// ImageState live in rasterizer_impl.h:21-73 and are NOT mirrored):
//   geometry (per Gaussian, SoA, 256-B aligned arrays):
//     splat (64-B record: means2D, conic + opacity, colour + depth — one
//     cache-line half per gather in the blend loops), tiles_touched u32, clamped u8 (3 bits),
//     radii i32, first_slot u32 (first binning slot of the Gaussian),
//     depth sort ping-pong (key u32 = depth bits, val u32 = index) and scratch.
//   binning (per tile instance): slot_gauss (emitted Gaussian per slot), the
//     tile sort's ping-pong keys (tile) and uint2 values (Gaussian, slot) —
//     the result, point_pairs, is the per-tile list (x: Gaussian, y: slot, the
//     gradient-record index) — and the
//     gradient records written by the backward blend, one 48-B record per
//     (binning slot, 8x8 quadrant) at 4*slot+q, written only for entries the
//     quadrant's cull kept (sized for HBM capacity, not touched otherwise),
//     plus one flag byte per record (zeroed by each backward).
//   image (per pixel / tile): final_T, n_contrib, ranges uint2, tile_last
//     (max n_contrib over the tile) and quad_last (max n_contrib over each
//     quadrant: the backward wave's start position).
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace gs {

constexpr int kSortIPT = 16;                    // keys per thread in the tile-key radix kernels
constexpr int kSortTile = 256 * kSortIPT;       // keys per workgroup
constexpr int kDepthSortIPT = 8;                // depth sort: smaller tiles, >= 2 workgroups per CU at 1M
constexpr int kDepthSortTile = 256 * kDepthSortIPT;
constexpr int kScanIPT = 4;
constexpr int kScanTile = 256 * kScanIPT;
// Depth sort: keys are the bits of the view depth (d > 0.2), relative to the visible minimum; since round 5
// one MSD bucketing pass + a per-bucket local sort (depth_sort_msd) orders any range.  The 3-pass LSD form
// (kDepthSortBits) is kept as the 32-bit fallback's pass width only (DGE_AMD_DEPTH_KEYS32, a test switch).
constexpr int kCounterSlots = 16;   // preprocess counters: copies in separate 64-B lines
constexpr int kCounterStride = 16;  // u32 per slot
constexpr int kDepthPassBits = 9;
constexpr int kDepthSortBits = 3 * kDepthPassBits;
constexpr int kMaxSinglePassBits = 11;          // tile keys up to 2048 tiles sort in one pass
constexpr int kMsdBits = 11, kMsdBuckets = 1 << kMsdBits, kMsdCulled = kMsdBuckets - 1;  // depth_sort_msd
#ifndef GS_MSD_IPT
#define GS_MSD_IPT 16  // keys per thread of the MSD pass's blocks (8: 2648-2736 vs 16: 2754-2760 renders/s)
#endif
constexpr int kMsdIPT = GS_MSD_IPT;
static_assert(kMsdIPT >= kDepthSortIPT, "the depth sort's tables are sized for kDepthSortTile-key blocks");
constexpr size_t kAlign = 256;

__host__ __device__ inline size_t align_up(size_t x, size_t a = kAlign) { return (x + a - 1) / a * a; }
inline int div_up(long long a, long long b) { return (int)((a + b - 1) / b); }
__host__ __device__ inline uint32_t div_up_u(uint32_t a, uint32_t b) { return (a + b - 1) / b; }

inline int ceil_log2(uint32_t n) {
    int b = 0;
    while ((1u << b) < n) ++b;
    return b;
}

// Two-level binning for grids of more than 2048 tiles and at most 128 x 128 (c4: 120 x 68): the
// emission itself does the first, column pass (k_scan_emit_x: instances written ordered by tile
// column, stable, with the key y << 7 | x), one 7-bit row pass follows, and the tile ranges come
// from per-tile counts taken during that pass — instead of an emission, two full sort passes and a
// ranges pass over the K instances.
constexpr int kXBits = 7, kXDigits = 1 << kXBits;
inline bool tile_sort_fused(int gx, int gy) { return gx * gy > (1 << 11) && gx <= kXDigits && gy <= kXDigits; }

// Radix pass plan for the tile-key sort.
struct TileSortPlan {
    int bits;          // total key bits
    int passes;        // 1 or 2
    int bits0, bits1;  // digit width of each pass
};
inline TileSortPlan tile_sort_plan(int num_tiles) {
    TileSortPlan p;
    p.bits = ceil_log2((uint32_t)(num_tiles > 1 ? num_tiles : 2));
    if (p.bits <= kMaxSinglePassBits) {
        p.passes = 1; p.bits0 = p.bits; p.bits1 = 0;
    } else {
        p.passes = 2; p.bits0 = (p.bits + 1) / 2; p.bits1 = p.bits - p.bits0;
    }
    return p;
}

// What the blend kernels gather per list entry, one 64-B record per Gaussian
// (one cache-line half per gather instead of three lines from three arrays):
// 2D mean, conic + opacity, colour + depth (forward.cu:251-255 outputs).
struct alignas(64) Splat {
    float2 xy;
    float2 pad0;
    float4 co;    // conic (a, b, c) + opacity
    // colour + view depth; the depth NEGATED where gs_params.aux_mask marks the Gaussian (the grey value 1 the
    // blend composites beside the colour): a touched Gaussian's depth is > 0.2, so its sign is a free bit the
    // gather brings along, and every reader takes |w|
    float4 rgbd;
    float4 pad1;
};

struct GeomLayout {
    size_t splat, tiles_touched, clamped, touched, live_count, live_list, radii, first_slot;
    // live_count: one u32 per 256-Gaussian block (k_gauss_live); live_list: block-local compacted ids
    size_t key0, key1, val0, val1, rect, sort_hist, sort_totals, scan_sums, emit_hist, msd_ranges, total;
    int sort_blocks, scan_blocks;
};
inline GeomLayout geom_layout(int P) {
    GeomLayout L;
    size_t o = 0;
    size_t p = (size_t)(P > 0 ? P : 1);
    L.sort_blocks = div_up((long long)p, kDepthSortTile);
    L.scan_blocks = div_up((long long)p, kScanTile);
    L.splat = o; o = align_up(o + sizeof(Splat) * p);
    L.tiles_touched = o; o = align_up(o + 4 * p);
    L.clamped = o; o = align_up(o + 1 * p);
    L.touched = o; o = align_up(o + 1 * p);
    L.live_count = o; o = align_up(o + 4 * (size_t)div_up((long long)p, 256));
    L.live_list = o; o = align_up(o + 4 * p);
    L.radii = o; o = align_up(o + 4 * p);
    L.first_slot = o; o = align_up(o + 4 * p);
    L.key0 = o; o = align_up(o + 4 * p);
    L.key1 = o; o = align_up(o + 4 * p);
    L.val0 = o; o = align_up(o + 8 * p);  // depth sort values: uint2 (rect-or-count, Gaussian)
    L.val1 = o; o = align_up(o + 8 * p);
    L.rect = o; o = align_up(o + 4 * p);  // packed tile rect (pack_rect) or tiles_touched
    // any digit width; also the direct emission's per-block tile counts (scan_blocks rows of up to 2048 tiles)
    const size_t hist_rows = (size_t)(L.sort_blocks > L.scan_blocks ? L.sort_blocks : L.scan_blocks);
    L.sort_hist = o; o = align_up(o + 4 * (1u << kMaxSinglePassBits) * hist_rows);
    L.sort_totals = o; o = align_up(o + 4 * (1u << kMaxSinglePassBits));
    L.scan_sums = o; o = align_up(o + 4 * (size_t)(L.scan_blocks + 1));
    L.emit_hist = o; o = align_up(o + 4 * (size_t)kXDigits * L.scan_blocks);  // two-level binning: columns per block
    L.msd_ranges = o; o = align_up(o + 8 * (size_t)kMsdBuckets);  // depth_sort_msd: each bucket's (start, end)
    L.total = o;
    return L;
}

// Segment-parallel backward replay: for every segment k = [k*kSegLen,
// (k+1)*kSegLen) of a tile list it blends, the forward stores per quadrant pixel
// slot k = (T after the segment, S_k), S_k = the segment's own colour sum
// sum f alpha T (a separate accumulator, reset per segment).  The backward
// replays each segment of a quadrant window as its own work item, starting
// from T = slot k.T and the colour composited behind the segment
// D = (S_{k+1} + ... + S_last) / T: a sum of later segments' local sums, so its
// rounding is relative to D itself (a difference of prefix sums,
// (C_final - C_k) / T_k, would carry the whole prefix's rounding / T_k).  Checkpoint slots are allocated per
// tile from its list: tile t owns slots [ckpt_base(t), ckpt_base(t) + ceil(len/kSegLen)),
// ckpt_base(t) = range.x / kSegLen + t (monotone and non-overlapping because
// ranges are a prefix sum), each slot 4 quadrants x 64 pixels x float4.
constexpr int kBlendRound = 256;  // list entries per blend round
// Replay work items are listed by class of their blended-entry count, heaviest first (the hardware
// dispatches workgroups in order: the longest items start first, the short ones fill the end).  Each
// class keeps one list per XCD group of the forward (kItemXcds: the forward's rank & 7, the XCD its
// tile's four quadrant waves ran on): list (c, x) holds up to item_cap items at
// bwd_items[(c * kItemXcds + x) * item_cap ..), counted in bwd_count[item_count_at(c, x)], and the
// replay runs list x on one XCD, so a tile's four quadrants gather its list and Splats into one L2
constexpr int kItemClasses = 4, kItemXcds = 8, kItemCount0 = 32;
// (count (c, x) on XCD group x's 128-B line; each class's longest list on line 0, an atomicMax beside each
// list's atomicAdd: a replay workgroup reads the four maxima and its own list's count, 5 scalar loads —
// the ~100k surplus workgroups of a speculated grid exit after the first four)
__host__ __device__ inline int item_count_at(int c, int x) { return kItemCount0 * (2 + x) + c; }
__host__ __device__ inline int item_max_at(int c) { return kItemCount0 + c; }
// backward segment length: checkpoints at every round boundary and mid-round, so a replay work item
// covers at most 128 positions (half the per-item work of round-long segments: the replay's wave
// durations pack onto the SIMDs instead of leaving a tail of long items)
constexpr int kSegLen = 128;
static_assert(kBlendRound == 2 * kSegLen, "k_render_fwd writes two checkpoints per round");
__host__ __device__ inline uint32_t ckpt_base(uint32_t range_x, int tile) { return range_x / kSegLen + (uint32_t)tile; }
// checkpoint slots / work items for K instances over `tiles` tiles (upper bound)
__host__ __device__ inline size_t ckpt_slots(size_t K, int tiles) { return K / kSegLen + (size_t)tiles + 2; }
// Per (quadrant, list position) "blended by some pixel" bits, written by the forward
// and read by the backward instead of re-running the quadrant cull (exact: the
// backward's per-pixel hits are the forward's).  Tile t's words start at
// used_base(t) (64 positions per word), 4 quadrants interleaved: word w of
// quadrant q is used[(used_base + w) * 4 + q].
__host__ __device__ inline uint32_t used_base(uint32_t range_x, int tile) { return range_x / 64 + (uint32_t)tile; }
__host__ __device__ inline size_t used_words(size_t K, int tiles) { return 4 * (K / 64 + (size_t)tiles + 2); }

struct ImgLayout {
    size_t final_T, n_contrib, tile_order, counters, ranges, tile_last, quad_last, bwd_count, aux, total;
    // counters: kCounterSlots slots of kCounterStride u32: [0] instances, [1] max depth key,
    // [2] ~min depth key (summed / maxed over the slots by the host); slot 0 [3]: prefiltered error
};
inline ImgLayout img_layout(int W, int H) {
    ImgLayout L;
    size_t o = 0;
    size_t n = (size_t)W * H;
    size_t tiles = (size_t)div_up(W, 16) * div_up(H, 16);
    L.final_T = o; o = align_up(o + 4 * n);
    L.n_contrib = o; o = align_up(o + 4 * n);
    L.tile_order = o; o = align_up(o + 4 * tiles);  // tiles by list length, longest first
    // (before the counters: every pixel is written by the blend that fills it, the memset skips its 8 B/pixel)
    L.aux = o; o = align_up(o + 8 * n);  // float2 per pixel: the aux_mask grey sum (before bg), depth
    L.counters = o; o = align_up(o + 4 * kCounterSlots * kCounterStride);  // counters.. zeroed per forward (one memset)
    L.ranges = o; o = align_up(o + 8 * tiles);
    L.tile_last = o; o = align_up(o + 4 * tiles);
    L.quad_last = o; o = align_up(o + 16 * tiles);
    L.bwd_count = o; o = align_up(o + 4 * (size_t)item_count_at(0, kItemXcds));  // [item_max_at(c)], [item_count_at(c, x)]
    L.total = o;
    return L;
}

struct BinLayout {
    size_t key0, key1, pair0, pair1, slot_gauss, point_pairs, records, rec_flags, sort_hist, sort_totals, ckpt,
        bwd_items, used, tile_count, total;
    int sort_blocks;
    size_t nslots;  // checkpoint slots = work-item capacity / 4
};
// bwd: with the backward's scratch (records, flags, checkpoints, work list, blended bits); a forward-only
// binning (gs_params.forward_only) leaves them out (zero-sized, at the end)
inline BinLayout bin_layout(int K, int num_tiles, bool bwd = true) {
    BinLayout L;
    size_t o = 0;
    size_t k = (size_t)(K > 0 ? K : 1);
    TileSortPlan plan = tile_sort_plan(num_tiles);
    int maxbits = plan.bits0 > plan.bits1 ? plan.bits0 : plan.bits1;
    // the two-level binning (grids over 2048 tiles: tile_sort_fused) keeps kXDigits column / row digits in
    // these tables (its column totals, the row pass's histogram): a 2049..4096-tile grid's two 6-bit passes
    // would size them for 64
    if (num_tiles > (1 << kMaxSinglePassBits) && maxbits < kXBits) maxbits = kXBits;
    L.sort_blocks = div_up((long long)k, kSortTile);
    L.key0 = o; o = align_up(o + 4 * k);
    L.key1 = o; o = align_up(o + 4 * k);
    L.pair0 = o; o = align_up(o + 8 * k);
    L.pair1 = o; o = align_up(o + 8 * k);
    L.point_pairs = plan.passes & 1 ? L.pair1 : L.pair0;  // where tile_sort leaves (Gaussian, slot)
    L.slot_gauss = o; o = align_up(o + 4 * k);
    L.sort_hist = o; o = align_up(o + 4 * ((size_t)1 << maxbits) * (size_t)L.sort_blocks);
    L.sort_totals = o; o = align_up(o + 4 * ((size_t)1 << maxbits));
    L.tile_count = o; o = align_up(o + 4 * (size_t)num_tiles);  // two-level binning: instances per tile
    const size_t kb = bwd ? k : 0;
    L.nslots = bwd ? ckpt_slots(k, num_tiles) : 0;
    L.records = o; o = align_up(o + 4 * 48 * kb);  // one record per (slot, quadrant)
    L.rec_flags = o; o = align_up(o + 4 * kb);
    L.ckpt = o; o = align_up(o + 16 * 64 * 4 * L.nslots);  // [slot][quadrant][64] float4 (T, own colour sum)
    L.bwd_items = o; o = align_up(o + 8 * 4 * L.nslots * kItemClasses * kItemXcds);  // uint2 (tile, seg << 2 | quadrant)
    L.used = o; o = align_up(o + (bwd ? 8 * used_words(k, num_tiles) : 0));
    L.total = o;
    return L;
}

// ---------------------------------------------------------------------
// launchers (defined in the .hip translation units)
// ---------------------------------------------------------------------
// SH coefficient k of Gaussian i: k == 0 at sh_dc + i*dc_stride,
// k >= 1 at sh_rest + i*rest_stride + 3*(k-1).  The reference's [P,M,3]
// tensor is dc = shs, rest = shs + 3, both strides 3M; GaussianModel's raw
// _features_dc [P,1,3] / _features_rest [P,M-1,3] are read in place (no cat).
struct ShView {
    const float* dc;    // fp32, or fp16 reinterpreted when `half`
    const float* rest;
    int dc_stride, rest_stride;  // in elements
    int half;
};
struct ShGradView {
    float* dc;
    float* rest;
    int dc_stride, rest_stride;
};

struct PreprocessArgs {
    int P, D, M, W, H, gx, gy;
    const float *means3D, *colors_precomp, *opacities, *scales, *rotations, *cov3D_precomp;
    const int* index;  // gs_params.index: parameter row of Gaussian i (NULL: i)
    ShView sh;         // sh.dc == nullptr: no SH
    int activation;    // 1: opacities/scales/rotations are raw GaussianModel parameters
    const float *view, *proj, *campos;
    float tanfovx, tanfovy, fx, fy, scale_modifier;
    int prefiltered, copy_colors;
    int* radii_out;
    uint8_t* visible_out;  // optional (radii > 0) bytes
    int* radii;
    Splat* splat;
    uint32_t* tiles_touched;
    uint8_t* clamped;
    uint32_t* depth_key;
    uint32_t* rect;          // pack_rect(tile rect) when the grid allows it, else tiles_touched
    int rect_packed;
    uint32_t* counters;  // kCounterSlots x kCounterStride (ImgLayout)
    uint8_t* touched;    // zeroed here: k_render_fwd sets the bytes of Gaussians some pixel blends
    const uint8_t* aux_mask = nullptr;  // gs_params.aux_mask: the sign of the Splat's depth
};
void launch_preprocess(const PreprocessArgs& a, hipStream_t s);
void launch_zero16(void* p, size_t bytes, hipStream_t s);  // bytes: a multiple of 16, p 16-B aligned
void launch_depth_keys32(int P, const uint32_t* rect, const Splat* splat, uint32_t* key, hipStream_t s);
void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t s);
// (test hook gs_activate_params) the fused path's in-kernel activations over P rows
void launch_activate_params(int P, const float* raw_opacity, const float* raw_scaling, const float* raw_rotation,
                            float* opacity, float* scaling, float* rotation, hipStream_t s);

// LSD radix sort of (u32 key, u32 value).  Returns the buffer index (0/1)
// holding the result.  identity_vals: values of the first pass are the
// element indices (val0 is not read).
// Stable LSD sort of (key, (aux[i], i)) pairs on key bits [0, bits), at most
// max_pass_bits per pass; returns the ping-pong index holding the result.
int radix_sort_aux(uint32_t* key0, uint32_t* key1, uint2* pair0, uint2* pair1, const uint32_t* aux, uint32_t n,
                   int bits, int max_pass_bits, int ipt, uint32_t* hist, uint32_t* totals, int nblocks, hipStream_t s,
                   uint2* ranges = nullptr, const uint32_t* key_bias_not = nullptr, uint32_t* tile_order = nullptr,
                   int ntiles = 0, const uint32_t* n_dev = nullptr);
// key_bias_not: the preprocess counter slots' ~min key (kCounterStride apart); the first pass sorts
// (and writes) key - min
// Stable sort of the K emitted instances on their tile id (key0 in slot
// order); the values are (Gaussian, slot) pairs built on the first pass from
// gauss_by_slot.  Returns the buffer index (0/1) holding keys and pairs.
// The depth order (depth bits, index) of the P Gaussians for any key range: one stable 11-bit MSD pass
// into depth buckets (keys relative to the visible minimum, read with the range from the preprocess counters
// at bias_not) and a per-bucket local sort; the (rect, Gaussian) values end in pair0 (returns 0).
// The preprocess counters published to the host by the depth sort's first kernel (block 0, at its end): the
// kCounterSlots x kCounterStride words at src copied to dst (pinned host memory, device view), then after a
// system-scope fence the word dst[kCounterSlots * kCounterStride] = seq — the host polls that word instead of
// an event behind a D2H copy (the copy and the fenced marker cost each view's sort chain ~13 us of queue time)
struct CountPublish {
    const uint32_t* src = nullptr;
    uint32_t* dst = nullptr;
    uint32_t seq = 0;
};
int depth_sort_msd(uint32_t* key0, uint32_t* key1, uint2* pair0, uint2* pair1, const uint32_t* rect, uint32_t n,
                   uint32_t* hist, uint32_t* totals, int nblocks, uint2* bucket_ranges, const uint32_t* bias_not,
                   hipStream_t s, CountPublish pub = CountPublish{});
int tile_sort(uint32_t* key0, uint32_t* key1, uint2* pair0, uint2* pair1, const uint32_t* gauss_by_slot, uint32_t n,
              int bits, uint32_t* hist, uint32_t* totals, int nblocks, hipStream_t s, uint2* ranges,
              uint32_t* tile_order, int ntiles,  // tile_order: the forward's dispatch order (single pass only)
              const uint32_t* n_dev = nullptr);  // n_dev: preprocess counters, n = min(count, n) read on the device
// the single-pass tile sort writes the tile ranges itself (and no sorted keys); two passes need k_ranges
inline bool tile_sort_writes_ranges(int num_tiles) { return tile_sort_plan(num_tiles).passes == 1; }

// Tile rect of a Gaussian in one u32 (x0, y0, x1, y1: 8 bits each, x1/y1
// exclusive) — carried through the depth sort with the Gaussian id, so the
// instance scan and the emission read it in depth order without gathers.
// Grids wider or taller than 255 tiles carry tiles_touched instead and the
// emission gathers the rect (rect_packed = 0).
constexpr int kRectPackMax = 255;
__host__ __device__ inline bool rect_packable(int gx, int gy) { return gx <= kRectPackMax && gy <= kRectPackMax; }
__host__ __device__ inline uint32_t pack_rect(int x0, int y0, int x1, int y1) {
    return (uint32_t)x0 | ((uint32_t)y0 << 8) | ((uint32_t)x1 << 16) | ((uint32_t)y1 << 24);
}

struct EmitArgs {
    int P, gx, gy;
    int rect_packed;
    const uint2* order;          // by depth rank: (packed rect or tiles_touched, Gaussian id)
    const uint32_t* tiles_touched;
    const Splat* splat;
    const int* radii;
    uint32_t* scan_sums;         // [scan_blocks + 1]
    uint32_t* first_slot;
    uint32_t* tile_key;          // K (two-level binning: u16 keys y << 7 | x in the same buffer)
    uint32_t* slot_gauss;        // K
    uint32_t* rec_flags32 = nullptr;  // K: zeroed by the emission (the backward's per-slot record flags)
    int scan_blocks;
    uint32_t cap = 0xFFFFFFFFu;  // binning capacity: slots at or past it are not written (speculative forward)
    // two-level binning (tile_sort_fused): per-block column counts (k_scan_reduce), their scanned
    // form and totals, the column-ordered (Gaussian, slot) pairs, per-tile counts zeroed by block 0
    uint32_t* xhist = nullptr;
    uint32_t* xtotals = nullptr;
    uint2* pairs_out = nullptr;
    uint32_t* tile_count = nullptr;
    int ntiles = 0;
    // ids_only (a forward-only render's two-level binning): the lists carry the Gaussian id alone (u32 at
    // pairs_out / the point list) — the binning slot is only the backward's record address
    int ids_only = 0;
    // direct emission (direct_emission: single-pass grids with packed rects): each scan block's instances
    // per tile (k_scan_reduce), scanned in place over the blocks by launch_scan_reduce, the tile totals;
    // k_emit_tiles writes the lists (pairs_out), the tile ranges and the forward's dispatch order
    uint32_t* thist = nullptr;
    uint32_t* ttotals = nullptr;
    uint2* ranges = nullptr;
    uint32_t* tile_order = nullptr;
    // region emission (region_emission_grid): each depth chunk's instances per tile, scanned in place over the
    // chunks (chunks rows of ntiles, block-major), every tile's first list position (unclamped), the rows of a
    // region
    uint32_t* chunk_hist = nullptr;
    uint32_t* tile_start = nullptr;
    int chunks = 0;
    int region_rows = 0;
};
// The direct emission for a gx x gy grid: at most 2048 tiles (one digit of the tile sort) and rects packed
// in the depth-sort payload
inline bool direct_emission_grid(int gx, int gy) {
    return gx * gy <= (1 << kMaxSinglePassBits) && rect_packable(gx, gy);
}
// The region emission (round 6) for grids of 2049..kRegionMaxTiles tiles with packed rects (c4's 120 x 68): the
// depth order is cut into chunks of kChunkG Gaussians and the grid into regions of region_rows(gx) tile rows.
// Each chunk counts its instances per tile (k_chunk_count), a scan over the chunks gives each chunk's first
// position in every tile's list, and one workgroup per (chunk, region) picks the chunk's Gaussians that reach its
// region, expands their instances there in depth order, ranks them per tile, stages them tile-major in LDS and
// stores each tile's run (about kChunkG x 17 / 8160 = 34 ids at c4) coalesced.  Every instance is written once,
// into its final place — the two-level binning wrote it twice (column emission, row pass) and read it back once.
// Opt-in (DGE_AMD_BINNING=region): it measured slower than the two-level binning at c4, 574 vs 423 us — its
// per-batch ranking, scans and barriers leave the CUs waiting.
#ifndef GS_CHUNK_G
#define GS_CHUNK_G 16384
#endif
constexpr int kChunkG = GS_CHUNK_G, kRegionMaxTiles = 12288;
static_assert(kChunkG % kScanTile == 0, "a chunk is whole scan blocks");
inline int region_chunks(int P) { return div_up((long long)(P > 0 ? P : 1), kChunkG); }
// tile rows per region: about GS_REGION_TILES tiles (a region's per-tile counters fit 10 bits of tile index;
// the emit time at c4 by region size in the comment below)
#ifndef GS_REGION_TILES
#define GS_REGION_TILES 512  // (c4: 1024 -> 764 us, 512 -> 574, 256 -> 621, 128 -> 791)
#endif
static_assert(GS_REGION_TILES <= 1024, "region tiles fit 10 bits");
inline int region_rows(int gx, int gy) {
    const int r = GS_REGION_TILES / (gx > 0 ? gx : 1);
    return r < 1 ? 1 : (r > gy ? gy : r);
}
inline bool region_emission_grid(int gx, int gy) {
    return gx * gy > (1 << kMaxSinglePassBits) && gx * gy <= kRegionMaxTiles && rect_packable(gx, gy);
}
// the count table (chunks x tiles u32) goes where the tile sort's keys would be ([key0, pair0)), the tile starts
// where its slot map would be: both unused by the region emission
inline bool region_table_fits(const BinLayout& L, int P, int tiles) {
    return (size_t)4 * region_chunks(P) * (size_t)tiles <= L.pair0 - L.key0 &&
           (size_t)4 * (size_t)tiles <= L.sort_hist - L.slot_gauss;
}
void launch_region_emit(const EmitArgs& a, hipStream_t s);
void launch_scan_reduce(const EmitArgs& a, hipStream_t s);
void launch_scan_emit(const EmitArgs& a, hipStream_t s);
void launch_emit_tiles(const EmitArgs& a, hipStream_t s);
// two-level binning after the instance count is known: column scan + k_scan_emit_x, the row pass
// (pairs_out/tile_key -> point_pairs, per-tile counts), ranges from the counts
void launch_emit_fused(const EmitArgs& a, hipStream_t s);
// (tile_order: also the forward's longest-list-first dispatch order, from the same counts)
void launch_row_pass(const EmitArgs& a, uint32_t K, uint2* point_pairs, uint32_t* hist, int sort_blocks,
                     uint2* ranges, uint32_t* tile_order, hipStream_t s, const uint32_t* n_dev = nullptr);

// One byte on the device: 1 when some speculated view of a batch overflowed its binning capacity (the
// sum of its preprocess counter slots > cap) or its visible depth keys span more than `bits` bits — the
// host's gs_views_check decision, made where a collective can carry it (GradBucket.allreduce_begin)
struct OverflowArgs {
    int n = 0;
    const uint32_t* counters[8] = {};  // (GS_MAX_VIEWS)
    uint32_t cap[8] = {};  // 0: an exact view (never overflows)
};
void launch_views_overflow(const OverflowArgs& a, uint8_t* flag, hipStream_t s);

// tile ranges; also zeroes the backward's per-slot record flags (u32 per slot)
void launch_ranges(const uint32_t* sorted_tile, int K, uint2* ranges, uint32_t* rec_flags32, hipStream_t s);

struct RenderArgs {
    int W, H, gx, gy;
    const uint2* ranges;
    uint32_t* tile_order;      // tiles longest list first: by the single-pass tile sort, else k_tile_order
    int order_ready;           // tile_order already written (the single-pass tile sort did it)
    const uint2* point_pairs;  // per-tile lists: (Gaussian, binning slot)
    const uint32_t* point_ids = nullptr;  // ... or the Gaussian ids alone (EmitArgs::ids_only)
    const Splat* splat;
    const float* bg;
    float* final_T;
    uint32_t* n_contrib;
    uint32_t* tile_last;
    uint32_t* quad_last;  // [tiles*4] max n_contrib per 8x8 quadrant
    float4* ckpt;         // (T, own colour sum) checkpoints for the segmented backward (see ckpt_base)
    uint64_t* used;       // per (quadrant, position) blended bits (see used_base)
    uint2* bwd_items;     // backward work list (4 * nslots) and its counters
    uint32_t* bwd_count;
    uint32_t item_cap;
    float* out_color;
    float* out_depth;
    uint8_t* touched;     // [P] set to 1 for every Gaussian some pixel blends (zeroed by the preprocess):
                          // exactly the Gaussians the backward gives a record, known after the forward
    uint64_t* diag;       // optional [tiles*4][kDiagWords] (see diag_buffer)
    int bwd = 1;          // 0: a forward-only render (gs_params.forward_only): no backward bookkeeping
    const float* colors = nullptr;  // forward-only: blend these [P,3] colours instead of the Splats' (recolor)
    float2* aux_out = nullptr;      // (bwd) gs_params.aux_mask: per pixel the grey sum and the depth
    // (recolor) *aux_match == 0: the colours are the source forward's aux grey, so the image is composed
    // from its aux sums (aux_src) and transmittance (final_T_src) instead of blended
    const uint32_t* aux_match = nullptr;
    const float2* aux_src = nullptr;
    const float* final_T_src = nullptr;
};
void launch_render_forward(const RenderArgs& a, hipStream_t s);
// flag[0] |= 1 unless colors[i] == (m, m, m) bit for bit, m = aux_mask[i] ? 1 : 0, for every i < P
void launch_aux_match(int P, const float* colors, const uint8_t* aux_mask, uint32_t* flag, hipStream_t s);

struct ApplyWeightsArgs {
    int W, H, gx, gy, C;
    const uint2* ranges;
    const uint2* point_pairs;  // per-tile lists: (Gaussian, binning slot)
    const Splat* splat;
    const float* image_weights;
    float* weights;
    int* cnt;
};
void launch_render_apply_weights(const ApplyWeightsArgs& a, hipStream_t s);
void launch_blend_exp(long long n, const float* x, float* y, hipStream_t s);

struct RenderBwdArgs {
    int W, H, gx, gy;
    const uint2* ranges;
    const uint2* point_pairs;  // per-tile lists: (Gaussian, binning slot)
    const uint32_t* quad_last;  // [tiles*4] the replay window of each quadrant wave
    const float4* ckpt;         // the forward's (T, own colour sum) checkpoints
    const uint64_t* used;       // the forward's blended bits: the backward's exact cull
    const uint2* bwd_items;     // the forward's work list (capacity item_cap)
    const uint32_t* bwd_count;  // [0] multi, [1] single items; [2], [3] the per-tile list's (k_bwd_tile_items)
    const uint32_t* tile_last;  // [tiles] the tile's last contributor (the per-tile replay's window)
    uint32_t item_cap;
    const Splat* splat;
    const float* bg;
    const float* final_T;
    const uint32_t* n_contrib;
    const float* dL_dpix;
    float4* records;     // [4*K][3] float4: one record per (slot, quadrant), kept entries only
    uint8_t* rec_flags;  // [4*K] set to 1 with each record (zeroed before the launch)
    uint64_t* diag;   // optional [item_cap][kDiagWords], by queue position (see diag_buffer)
};
void launch_render_backward(const RenderBwdArgs& a, hipStream_t s);
// n views' replays as one launch per kMaxReplayViews views, on one stream (no diag): view v's grid is
// grid_div-th of its item bound (rounded up to whole runs of 8 blocks), each block looping over the items
// one grid apart
constexpr int kMaxReplayViews = 4;
struct RenderBwdViews {
    int n;
    uint32_t grid[kMaxReplayViews];
    RenderBwdArgs v[kMaxReplayViews];
};
void launch_render_backward_views(const RenderBwdArgs* a, int n, uint32_t grid_div, hipStream_t s);

struct GaussBwdArgs {
    int P, D, M, W, H, gx, gy;
    const float *means3D, *scales, *rotations, *cov3D_precomp, *opacities;
    const int* index;  // gs_params.index: parameter row (inputs and parameter-shaped gradients)
    ShView sh;
    ShGradView dsh;    // dsh.dc == nullptr: no SH gradient output
    int activation;    // 1: chain the gradients through sigmoid / exp / normalize
    const float *view, *proj, *campos;
    float tanfovx, tanfovy, fx, fy, scale_modifier;
    const int* radii;       // caller's radii (the reference's visibility gate)
    const uint32_t* tiles_touched;
    const uint32_t* first_slot;
    const uint8_t* clamped;
    const uint8_t* rec_flags;  // [4*K] nonzero: record (slot, quadrant) was written
    const uint8_t* touched;    // [P] nonzero: the Gaussian has at least one record
    uint32_t* live_list;       // [P] k_gauss_live: block b's live Gaussians at [256 b, 256 b + live_count[b])
    uint32_t* live_count;      // [P/256] live Gaussians per 256-Gaussian block
    const float4* records;     // [4*K][3] float4: (slot, quadrant) record at 3*(4*slot + q), flag byte 4*slot + q
    float *dL_dmeans2D, *dL_dcolors, *dL_dopacity, *dL_dmeans3D, *dL_dcov3D, *dL_dscales, *dL_drot;
    int pm3 = 3, pop = 1, psc = 3, prot = 4;  // row pitches (floats) of the parameter-shaped outputs
    uint32_t acc;  // GS_ACC_* bits: add into the output instead of overwriting
    uint32_t zeroed;  // acc bits whose outputs hold zeros: a Gaussian's first write stores (gs_grads.zeroed)
    uint32_t slot_cap = 0xFFFFFFFFu;  // binning capacity (a speculative forward's slots end there)
    uint8_t* dirty = nullptr;  // optional [rows] (gs_grads.dirty_rows): k_gauss_live marks the live rows
    const uint8_t* grad_mask;  // optional [P]: outputs in mask_bits are multiplied by it
    uint32_t mask_bits;
    float* dL_dconic;          // optional [P,3]: the summed conic gradient (parity tests)
    uint64_t* diag;            // optional per-wave phase stamps of k_gauss_bwd_live (see diag_buffer)
};
void launch_gauss_backward(const GaussBwdArgs& a, hipStream_t s, hipEvent_t writes_after = nullptr);
// n views' per-Gaussian passes as one (views[0] names the live-list scratch; the parameter-shaped
// outputs are shared, GS_ACC_* set on them for every view but the first): at most
// gauss_backward_max_views() views per call
void launch_gauss_backward_views(const GaussBwdArgs* views, int n, hipStream_t s, hipEvent_t writes_after = nullptr);
// the same in its two passes (the first needs only the forwards' outputs)
void launch_gauss_live_views(const GaussBwdArgs* views, int n, hipStream_t s, hipEvent_t writes_after);
void launch_gauss_bwd_live_views(const GaussBwdArgs* views, int n, hipStream_t s, hipEvent_t writes_after);
int gauss_backward_max_views();

// diagnostics (gs_profile_diag_*): per-wave records of the blend kernels,
// kDiagWords u64 each: start, end (s_memrealtime, 100 MHz), kept entries,
// rounds, cycles in the blend/replay loops, total cycles (s_memtime).
constexpr int kDiagWords = 8;
uint64_t* diag_buffer(int which, size_t n_u64);  // which: 0 forward, 1 backward, 2 gauss_bwd; nullptr when off
int report_error(int code, const char* msg);      // sets gs_last_error(), returns code

}  // namespace gs
