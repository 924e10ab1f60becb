// gs_sort.hip — binning for gfx950: depth sort, instance scan + emission,
// tile-key sort, tile ranges.
//
// The reference (rasterizer_impl.cu:227-270) scans tiles_touched in Gaussian
// order, emits a 64-bit (tile << 32 | depth) key per instance
// (duplicateWithKeys, :67-100) and radix-sorts all K instances on 32+log2(tiles)
// bits with cub (:253-261).  Because that sort is stable and emission follows
// Gaussian order, the result is: per tile, instances ordered by (depth bits,
// Gaussian index).  This file produces the identical order with less traffic:
//   1. stable LSD sort of the P visible depth keys (32-bit key, index value);
//   2. exclusive scan of tiles_touched in depth order, then emission of one
//      (tile, slot) instance per overlapped tile — instances are therefore
//      already depth-ordered;
//   3. stable LSD sort of the K instances on the tile id only (one pass for
//      up to 2048 tiles);
//   4. tile ranges from the sorted tile ids; the sort carries the slot (the
//      gradient-record index) and the Gaussian id (the point list) along.
// The radix kernels rank keys inside a workgroup with 64-lane ballots
// (peer-mask match per digit), keep per-wave digit counters in LDS and never
// use global atomics, so every pass is deterministic.
#include <type_traits>

#include "gs_common.h"
#include "gs_internal.h"

namespace gs {

// ---------------------------------------------------------------------
// helpers
// ---------------------------------------------------------------------
template <int BITS>
__device__ __forceinline__ uint64_t match_digit(uint32_t d, uint64_t valid_mask) {
    uint64_t m = valid_mask;
#pragma unroll
    for (int b = 0; b < BITS; ++b) {
        const bool bit = (d >> b) & 1u;
        const uint64_t bal = __ballot(bit);
        m &= bit ? bal : ~bal;
    }
    return m;
}

// k div w for the instance index k < 2^16 inside a rect w <= 255 tiles wide, without a division: a table of
// magic multipliers M[w] = ceil(2^32 / w) (one integer division per thread, filled before the block's first
// barrier), k div w = umulhi(k, M[w]) — exact since k (M - 2^32 / w) < 2^32 / w for k < 2^16 (and w = 1 is k).
// (The IEEE float quotient (k + 0.5) / w it replaces cost ~16 VALU and a reciprocal per instance.)
__device__ __forceinline__ void fill_div_magic(uint32_t* s_magic) {
    const uint32_t w = threadIdx.x;  // (256 threads: one entry each)
    s_magic[w] = w > 1 ? 0xFFFFFFFFu / w + 1u : 0u;
}
__device__ __forceinline__ uint32_t div_small(uint32_t k, uint32_t w, const uint32_t* s_magic) {
    return w == 1 ? k : __umulhi(k, s_magic[w]);
}

// This thread's part of the sum of sums[0 .. n): elements tid, tid + 256, ... loaded four at a time, clamped
// and unconditional, so their loads are in flight together (a loop adding each load as it came waited for
// every one in turn).
__device__ __forceinline__ uint32_t strided_part(const uint32_t* __restrict__ sums, uint32_t n) {
    uint32_t part = 0;
    for (uint32_t j0 = threadIdx.x; j0 < n; j0 += 1024) {
        uint32_t v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = sums[min(j0 + 256u * u, n - 1)];
#pragma unroll
        for (int u = 0; u < 4; ++u) part += j0 + 256u * u < n ? v[u] : 0u;
    }
    return part;
}

// 256-thread exclusive scan; `total` receives the workgroup sum.
__device__ __forceinline__ uint32_t block_exclusive_scan(uint32_t v, uint32_t* lds4, uint32_t& total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) lds4[w] = x;
    __syncthreads();
    uint32_t wbase = 0, t = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const uint32_t c = lds4[i];
        wbase += (i < w) ? c : 0u;
        t += c;
    }
    __syncthreads();
    total = t;
    return wbase + x - v;
}

// 256-thread exclusive max-scan (0 for thread 0).
__device__ __forceinline__ uint32_t block_exclusive_max(uint32_t v, uint32_t* lds4) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    uint32_t x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = (uint32_t)__shfl_up((int)x, o);
        if (lane >= o) x = max(x, y);
    }
    if (lane == 63) lds4[w] = x;
    __syncthreads();
    uint32_t pre = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) pre = i < w ? max(pre, lds4[i]) : pre;
    __syncthreads();
    const uint32_t ex = (uint32_t)__shfl_up((int)x, 1);
    return max(pre, lane > 0 ? ex : 0u);
}

// The depth sort's bias: the minimum visible key, kept as ~min in the preprocess counter slots
// (max over the slots; kCounterStride apart).
__device__ __forceinline__ uint32_t key_bias(const uint32_t* __restrict__ bias_not) {
    if (!bias_not) return 0u;
    uint32_t m = 0u;
#pragma unroll
    for (int i = 0; i < kCounterSlots; ++i) m = max(m, bias_not[i * kCounterStride]);
    return ~m;
}

// The instance count of a forward whose binning was enqueued before the host read it back
// (gs_views_forward, speculative capacity): the sum of the preprocess counter slots, capped at the
// binning buffer's capacity `cap` (an overflow is detected by the host later, gs_views_check).
// n_dev == nullptr: the host-known count `cap` itself.
__device__ __forceinline__ uint32_t dev_count(const uint32_t* __restrict__ n_dev, uint32_t cap) {
    if (!n_dev) return cap;
    uint32_t k = 0;
#pragma unroll
    for (int i = 0; i < kCounterSlots; ++i) k += n_dev[i * kCounterStride];
    return k < cap ? k : cap;
}

// The depth sort's MSD bucketing (depth_sort_msd): the visible keys' range [kmin, kmax] (the preprocess
// counter slots: [1] max key, [2] ~min key) split into at most kMsdBuckets - 1 buckets of 2^s keys each,
// bucket = (key - kmin) >> s with s the smallest shift that keeps the top bucket below kMsdCulled; culled
// keys (0xFFFFFFFF, whose relative key is ~kmin) in bucket kMsdCulled.  Within a bucket only the low s
// bits of key - kmin differ: k_depth_bucket_sort orders them.
struct MsdParams {
    uint32_t kmin, s;
};
__device__ __forceinline__ MsdParams msd_params(const uint32_t* __restrict__ bias_not) {
    uint32_t mn = 0u, mx = 0u;
#pragma unroll
    for (int i = 0; i < kCounterSlots; ++i) {
        mn = max(mn, bias_not[i * kCounterStride]);
        mx = max(mx, bias_not[i * kCounterStride - 1]);
    }
    MsdParams m;
    m.kmin = ~mn;
    const uint32_t range = mx >= m.kmin ? mx - m.kmin : 0u;  // (no visible key: kmin = ~0, range 0)
    const uint32_t q = range / (uint32_t)(kMsdBuckets - 1);
    m.s = q ? 32u - (uint32_t)__clz(q) : 0u;  // range < (kMsdBuckets - 1) << s
    return m;
}
__device__ __forceinline__ uint32_t msd_digit(uint32_t krel, const MsdParams& m) {
    return krel == ~m.kmin ? (uint32_t)kMsdCulled : krel >> m.s;
}

// ---------------------------------------------------------------------
// radix sort: histogram -> per-digit scan -> stable scatter
// ---------------------------------------------------------------------
// Per-block digit counts (integer LDS atomics: the counts do not depend on the order),
// stored block-major (bm: hist[b * NDIG + d], one coalesced row per block; a
// digit-major table makes every block write NDIG scattered words, one cache line
// each) while the column scan stays short — up to kScanBmRows blocks; longer sorts
// (c4's 10k-block tile sort) keep the digit-major table, whose scan is one
// workgroup per digit over a contiguous row.
__host__ __device__ __forceinline__ size_t hist_at(int bm, uint32_t b, uint32_t d, int nb, int ndig) {
    return bm ? (size_t)b * ndig + d : (size_t)d * nb + b;
}
// KT: the key type (u16 for the two-level binning's row pass: its keys are y << 7 | x)
// DM: the digit is the MSD depth bucket (msd_digit) instead of (key >> shift) & mask
template <int BITS, int IPT, class KT = uint32_t, bool DM = false>
__global__ __launch_bounds__(256) void k_radix_hist(const KT* __restrict__ keys, uint32_t n, int shift,
                                                    uint32_t* __restrict__ hist, int nb, int bm,
                                                    const uint32_t* __restrict__ bias_not,
                                                    const uint32_t* __restrict__ n_dev, CountPublish pub) {
    constexpr int NDIG = 1 << BITS;
    __shared__ uint32_t cnt[NDIG];
    const int tid = threadIdx.x;
    n = dev_count(n_dev, n);
    const uint32_t base = blockIdx.x * (uint32_t)(256 * IPT);
    if (base >= n && blockIdx.x) return;  // (a capacity-sized grid: rows past the count are never read)
    for (int i = tid; i < NDIG; i += 256) cnt[i] = 0;
    __syncthreads();
    const uint32_t bias = key_bias(bias_not);
    MsdParams msd{0u, 0u};
    if constexpr (DM) msd = msd_params(bias_not);
    // counts do not depend on which thread sees which key: each thread takes VEC consecutive keys per 16-B
    // load (a wave reads 1 KB per instruction instead of 64 scattered 2-4 B words)
    constexpr int VEC = 16 / (int)sizeof(KT);
    static_assert(IPT % VEC == 0, "whole 16-B loads per thread");
    uint4 raw[IPT / VEC];
#pragma unroll
    for (int j = 0; j < IPT / VEC; ++j) {
        const uint32_t e0 = base + (uint32_t)(j * 256 + tid) * VEC;
        if (e0 + VEC <= n) {
            raw[j] = *reinterpret_cast<const uint4*>(keys + e0);
        } else {  // (the block's tail: key by key)
            KT t[VEC];
#pragma unroll
            for (int u = 0; u < VEC; ++u) t[u] = e0 + u < n ? keys[e0 + u] : KT(0);
            raw[j] = *reinterpret_cast<const uint4*>(t);
        }
    }
#pragma unroll
    for (int j = 0; j < IPT / VEC; ++j) {
        const uint32_t e0 = base + (uint32_t)(j * 256 + tid) * VEC;
        const KT* k = reinterpret_cast<const KT*>(&raw[j]);
#pragma unroll
        for (int u = 0; u < VEC; ++u)
            if (e0 + u < n) {
                const uint32_t kr = (uint32_t)k[u] - bias;
                atomicAdd(&cnt[DM ? msd_digit(kr, msd) : (kr >> shift) & (NDIG - 1)], 1u);
            }
    }
    __syncthreads();
    for (int d = tid; d < NDIG; d += 256) hist[hist_at(bm, blockIdx.x, d, nb, NDIG)] = cnt[d];
    if (pub.dst && blockIdx.x == 0) {  // (CountPublish: vector stores, the sequence word last)
        for (int i = tid; i < kCounterSlots * kCounterStride; i += 256) pub.dst[i] = pub.src[i];
        __threadfence_system();
        __syncthreads();
        if (tid == 0) __hip_atomic_store(pub.dst + kCounterSlots * kCounterStride, pub.seq, __ATOMIC_RELEASE,
                                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Exclusive scan of every digit's column hist[0..nb)[d] in place, totals[d] =
// digit count.  One workgroup per kScanDigits digits: thread (row group g,
// digit dl) sums rows [g*per, (g+1)*per) of its digit (a wave load covers 8 rows
// x 32 B), the kScanGroups row-group sums are scanned in LDS, then the rows are
// rewritten.  (c2: the direct emission's 977 block rows -> 31 per thread.)
// Digits per digit-scan workgroup x row groups = its threads.  256-thread workgroups (8 x 32) find room on
// CUs busy with the other streams' blends, where 1024-thread ones waited up to 70 us for a CU to drain
// (3-stream trace): c2 2883-2898 -> 2943-2945 renders/s (one-stream scan stage 18.0 -> 20.7 us); 4 x 64
// (16-B row segments) measured 2882 (profiles/r05/ab_scan_shape_live_first.txt)
#ifndef GS_SCAN_DIGITS
#define GS_SCAN_DIGITS 8
#endif
#ifndef GS_SCAN_GROUPS
#define GS_SCAN_GROUPS 32
#endif
constexpr int kScanDigits = GS_SCAN_DIGITS, kScanGroups = GS_SCAN_GROUPS, kScanRegs = 32;
constexpr int kScanThreads = kScanDigits * kScanGroups;
constexpr int kScanBmRows = kScanGroups * kScanRegs;  // block-major tables up to this many blocks
__global__ __launch_bounds__(kScanThreads) void k_radix_digit_scan(uint32_t* __restrict__ hist, int nb, int ndig,
                                                           uint32_t* __restrict__ totals,
                                                           const uint32_t* __restrict__ n_dev, uint32_t cap,
                                                           int tile) {
    __shared__ uint32_t part[kScanGroups][kScanDigits];
    if (n_dev) nb = max(1, div_up_u(dev_count(n_dev, cap), (uint32_t)tile));  // rows the histogram wrote
    const int dl = threadIdx.x & (kScanDigits - 1), g = threadIdx.x / kScanDigits;
    const int d = blockIdx.x * kScanDigits + dl;
    const int per = (nb + kScanGroups - 1) / kScanGroups;
    const int r0 = g * per, r1 = min(nb, r0 + per);
    // up to kScanRegs rows per thread are held in registers: every load in flight at once, one
    // read and one write per element (c2: 14 tile-sort rows, 8 depth-sort rows); longer columns loop
    const bool in_regs = per <= kScanRegs;
    uint32_t v[kScanRegs];
    uint32_t s = 0;
    if (d < ndig) {
        if (in_regs) {
#pragma unroll
            for (int i = 0; i < kScanRegs; ++i) {
                v[i] = r0 + i < r1 ? hist[(size_t)(r0 + i) * ndig + d] : 0u;
                s += v[i];
            }
        } else {
#pragma unroll 4
            for (int r = r0; r < r1; ++r) s += hist[(size_t)r * ndig + d];
        }
    }
    part[g][dl] = s;
    __syncthreads();
    uint32_t run = 0, total = 0;
#pragma unroll 8
    for (int i = 0; i < kScanGroups; ++i) {
        const uint32_t pv = part[i][dl];
        run += i < g ? pv : 0u;
        total += pv;
    }
    if (d < ndig) {
        if (in_regs) {
#pragma unroll
            for (int i = 0; i < kScanRegs; ++i) {
                if (r0 + i < r1) hist[(size_t)(r0 + i) * ndig + d] = run;
                run += v[i];
            }
        } else {
#pragma unroll 4
            for (int r = r0; r < r1; ++r) {
                const size_t at = (size_t)r * ndig + d;
                const uint32_t c = hist[at];
                hist[at] = run;
                run += c;
            }
        }
        if (g == 0) totals[d] = total;
    }
}

// One workgroup per digit (digit-major table): exclusive scan of hist[d][0..nb)
// in place, totals[d] = digit count.
__global__ __launch_bounds__(256) void k_radix_digit_scan_dm(uint32_t* __restrict__ hist, int nb,
                                                             uint32_t* __restrict__ totals,
                                                             const uint32_t* __restrict__ n_dev, uint32_t cap,
                                                             int tile) {
    __shared__ uint32_t lds4[4];
    uint32_t* row = hist + (size_t)blockIdx.x * nb;  // (digit-major: the row pitch stays the grid's nb)
    if (n_dev) nb = max(1, div_up_u(dev_count(n_dev, cap), (uint32_t)tile));
    // each wave scans a contiguous quarter of the row in coalesced 64-element chunks (loads issued
    // kB chunks at a time): the wave's sum, the waves' prefix through LDS, then each chunk's
    // 64-lane scan carried from chunk to chunk (c4's row pass: 10.4k rows per digit)
    constexpr int kB = 16;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int nchunk = (nb + 63) / 64, cpw = (nchunk + 3) / 4;  // chunks per wave
    const int c0 = w * cpw, c1 = min(nchunk, c0 + cpw);
    uint32_t s = 0;
    for (int cb = c0; cb < c1; cb += kB) {
        uint32_t v[kB];
#pragma unroll
        for (int i = 0; i < kB; ++i) {
            const int j = (cb + i) * 64 + lane;
            v[i] = cb + i < c1 && j < nb ? row[j] : 0u;
        }
#pragma unroll
        for (int i = 0; i < kB; ++i) s += v[i];
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) s += (uint32_t)__shfl_xor((int)s, o);
    if (lane == 0) lds4[w] = s;
    __syncthreads();
    uint32_t run = 0, total = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        run += i < w ? lds4[i] : 0u;
        total += lds4[i];
    }
    for (int cb = c0; cb < c1; cb += kB) {
        uint32_t v[kB];
#pragma unroll
        for (int i = 0; i < kB; ++i) {
            const int j = (cb + i) * 64 + lane;
            v[i] = cb + i < c1 && j < nb ? row[j] : 0u;
        }
#pragma unroll
        for (int i = 0; i < kB; ++i) {
            uint32_t x = v[i];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t y = (uint32_t)__shfl_up((int)x, o);
                if (lane >= o) x += y;
            }
            const int j = (cb + i) * 64 + lane;
            if (cb + i < c1 && j < nb) row[j] = run + x - v[i];
            run += (uint32_t)__shfl((int)x, 63);
        }
    }
    if (threadIdx.x == 0) totals[blockIdx.x] = total;
}

// What a single-pass tile sort writes besides the permutation: the tile ranges
// (the digit IS the tile) and, when tile_order is set, the forward's dispatch
// order — tiles by list length, longest first (the former k_tile_order launch;
// block 0 has every tile's count in registers when it writes the ranges).
struct RangeOut {
    uint2* ranges;
    uint32_t* tile_order;
    int ntiles;
    // two-level binning's row pass: instances per tile (key y << 7 | x, input ordered by column x),
    // counted in LDS for the block's first kTcCols columns, global atomics beyond
    uint32_t* tile_count = nullptr;
    int gx = 0;
    // the MSD depth pass (DM): the culled bucket's values (already final: index order, nothing to sort)
    // go straight to the sorted output instead of through k_depth_bucket_sort
    uint2* culled_out = nullptr;
};
constexpr int kTcCols = 4;

// Block 0 of a single-pass tile sort (or of the direct emission): each thread holds the counts c of tiles
// [tid * PER, tid * PER + PER), starting at list position `run`.  Writes the tile ranges
// (identifyTileRanges, rasterizer_impl.cu:105-125; empty tiles keep (0, 0)) and, when tile_order is set, the
// forward's dispatch order — tiles by list length, longest first (the former k_tile_order launch).  Every
// thread of the block calls it (barriers).
// cap: the binning capacity of a speculative forward (the direct emission's counts are the full instance
// counts): ranges are clamped to it, so an overflowed binning, redone later, is never read past its end
template <int PER>
__device__ void write_tile_ranges(const uint32_t (&c)[PER], uint32_t run, int ntiles, uint2* __restrict__ ranges,
                                  uint32_t* __restrict__ tile_order, uint32_t cap = 0xFFFFFFFFu) {
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int d = tid * PER + i;
        if (ranges && d < ntiles)
            ranges[d] = c[i] ? make_uint2(min(run, cap), min(run + c[i], cap)) : make_uint2(0u, 0u);
        run += c[i];
    }
    if (!tile_order) return;
    constexpr int kClasses = 64;
    __shared__ uint32_t s_cls[kClasses];
    auto cls = [](uint32_t len) { return min(kClasses - 1, (int)(__log2f((float)len + 1.0f) * 3.0f)); };
    if (tid < kClasses) s_cls[tid] = 0u;
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int d = tid * PER + i;
        if (d < ntiles) atomicAdd(&s_cls[cls(c[i])], 1u);
    }
    __syncthreads();
    if (tid == 0) {  // start of each class, longest class first
        uint32_t acc = 0;
        for (int k = kClasses - 1; k >= 0; --k) {
            const uint32_t m = s_cls[k];
            s_cls[k] = acc;
            acc += m;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < PER; ++i) {
        const int d = tid * PER + i;
        if (d < ntiles) tile_order[atomicAdd(&s_cls[cls(c[i])], 1u)] = (uint32_t)d;
    }
}

// Value modes of the scatter: u32 values (IDV: the element index), or a packed
// (Gaussian, slot) pair: built from the index and a Gaussian-per-slot array on
// the first pass of the tile sort, then carried as one 8-byte value.
enum ValMode { kValU32 = 0, kValPairFirst = 1, kValPair = 2 };

// WK: the sorted keys are written (every pass but the last tile-sort pass).  Without them the block
// stages only the digit (u16), and the per-wave digit counters are u16 throughout (<= 256*IPT), so
// the single-pass tile sort fits three workgroups per CU (52 KB of LDS instead of 68).
#ifndef GS_SCATTER_MINW
#define GS_SCATTER_MINW 1  // minimum waves per SIMD the scatter's registers are fitted for (A/B)
#endif
template <int BITS, int IPT, bool IDV, int VM, bool WK = true, bool TC = false, class KT = uint32_t, bool DM = false>
__global__ __launch_bounds__(256, GS_SCATTER_MINW) void k_radix_scatter(const KT* __restrict__ keys_in,
                                                       const void* __restrict__ vals_in_,
                                                       uint32_t* __restrict__ keys_out, void* __restrict__ vals_out_,
                                                       const uint32_t* __restrict__ gauss_by_slot, uint32_t n,
                                                       int shift, const uint32_t* __restrict__ hist,
                                                       const uint32_t* __restrict__ totals, int nb, int bm,
                                                       RangeOut ro,
                                                       const uint32_t* __restrict__ bias_not,
                                                       const uint32_t* __restrict__ n_dev) {
    using V = typename std::conditional<VM == kValU32, uint32_t, uint2>::type;
    n = dev_count(n_dev, n);
    const uint32_t* vals_in = static_cast<const uint32_t*>(vals_in_);
    const uint2* pairs_in = static_cast<const uint2*>(vals_in_);
    V* vals_out = static_cast<V*>(vals_out_);
    constexpr int NDIG = 1 << BITS;
    constexpr int PER = NDIG >= 256 ? NDIG / 256 : 1;
    using C = uint16_t;
    static_assert(256 * IPT <= 65535, "u16 digit counters");
    __shared__ C cnt[4][NDIG];
    __shared__ uint32_t dbase[NDIG];
    __shared__ uint32_t lds4[4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int i = tid; i < 4 * NDIG; i += 256) (&cnt[0][0])[i] = 0;
    __shared__ uint32_t s_tc[TC ? kTcCols * kXDigits : 1];  // TC: the row pass's tile counts
    if (TC)
        for (int i = tid; i < kTcCols * kXDigits; i += 256) s_tc[i] = 0u;
    {  // dbase = exclusive scan of the digit totals
        uint32_t loc[PER];
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int d = tid * PER + i;
            loc[i] = d < NDIG ? totals[d] : 0u;
            s += loc[i];
        }
        uint32_t tot;
        const uint32_t run0 = block_exclusive_scan(s, lds4, tot);
        uint32_t run = run0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int d = tid * PER + i;
            if (d < NDIG) dbase[d] = run;
            run += loc[i];
        }
        // single-pass tile sort: the digit is the tile, so its run is the tile's range
        if (blockIdx.x == 0 && (ro.ranges || ro.tile_order))  // (uniform per block: its barriers are safe)
            write_tile_ranges<PER>(loc, run0, ro.ntiles, ro.ranges, ro.tile_order);
    }
    __syncthreads();
    // a capacity-sized grid (n_dev): blocks past the count leave after block 0 wrote the ranges
    if (blockIdx.x * (uint32_t)(256 * IPT) >= n) return;
    const uint32_t base = blockIdx.x * (uint32_t)(256 * IPT) + w * 64u * IPT;
    const uint32_t bias = key_bias(bias_not);
    MsdParams msd{0u, 0u};
    if constexpr (DM) msd = msd_params(bias_not);
    auto digit = [&](uint32_t k) { return DM ? msd_digit(k, msd) : (k >> shift) & (NDIG - 1); };
    uint32_t key[IPT], loc[IPT];
    V val[IPT];
    // unconditional loads, clamped into the array (base < n here): all of them in flight at once.  (Loads
    // under `valid` with the bias applied in the same branch waited for each key in turn — 16 memory round
    // trips per block: c4's row pass 221 us.)
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
        const uint32_t idx = base + it * 64 + lane;
        const uint32_t ci = idx < n ? idx : n - 1;
        key[it] = (uint32_t)keys_in[ci];
        if constexpr (VM == kValU32) val[it] = IDV ? idx : vals_in[ci];
        else if constexpr (VM == kValPairFirst) val[it] = make_uint2(0u, idx);  // (aux re-read at the store)
        else val[it] = pairs_in[ci];
    }
    __builtin_amdgcn_sched_barrier(0);  // (keeps the bias below from being hoisted between the loads)
#pragma unroll
    for (int it = 0; it < IPT; ++it) key[it] = base + it * 64 + lane < n ? key[it] - bias : 0u;
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
        const uint32_t idx = base + it * 64 + lane;
        const bool valid = idx < n;
        const uint64_t vm = __ballot(valid);
        if (vm == 0) break;
        const uint32_t d = digit(key[it]);
        const uint64_t peers = match_digit<BITS>(d, vm);
        const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
        const uint32_t old = cnt[w][d];
        loc[it] = old + rank;
        if (valid && rank == 0) cnt[w][d] = (C)(old + (uint32_t)__popcll(peers));
    }
    __syncthreads();
    // block-local digit-major order: run of digit d starts at bstart[d] (scan of the block's digit
    // totals); wave w's elements of digit d follow those of waves < w.  cnt[w][d] <- that start,
    // dbase[d] <- global position of the block's run minus bstart[d].
    {
        uint32_t tot[PER];
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int d = tid * PER + i;
            tot[i] = d < NDIG ? cnt[0][d] + cnt[1][d] + cnt[2][d] + cnt[3][d] : 0u;
            s += tot[i];
        }
        uint32_t all;
        uint32_t run = block_exclusive_scan(s, lds4, all);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int d = tid * PER + i;
            if (d < NDIG) {
                const uint32_t c0 = cnt[0][d], c1 = cnt[1][d], c2 = cnt[2][d];
                cnt[0][d] = (C)run;
                cnt[1][d] = (C)(run + c0);
                cnt[2][d] = (C)(run + c0 + c1);
                cnt[3][d] = (C)(run + c0 + c1 + c2);
                dbase[d] = dbase[d] + hist[hist_at(bm, blockIdx.x, d, nb, NDIG)] - run;
            }
            run += tot[i];
        }
    }
    __syncthreads();
    // stage the block in digit-major order, then store it with consecutive lanes on consecutive
    // positions of each digit run (coalesced) instead of one scattered element per lane
    using SK = typename std::conditional<WK, uint32_t, uint16_t>::type;  // staged key, or its digit
    // kValPairFirst stages the element's position in the block (u16) instead of its 8-B (aux, index) pair and
    // gathers aux again at the store (from L1/L2: the block's slice was just read): a quarter of the staging
    // LDS, so more workgroups per CU (c2's single-pass tile sort: 52 -> 28 KB, 3 -> 5 per CU)
    using SV = typename std::conditional<VM == kValPairFirst, uint16_t, V>::type;
    __shared__ SK s_key[256 * IPT];
    __shared__ SV s_val[256 * IPT];
    const uint32_t b0 = blockIdx.x * (uint32_t)(256 * IPT);
    const uint32_t x_first = TC ? (uint32_t)keys_in[b0] & (kXDigits - 1) : 0u;  // the block's first column
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
        const uint32_t idx = base + it * 64 + lane;
        if (idx < n) {
            const uint32_t d = digit(key[it]);
            const uint32_t lp = cnt[w][d] + loc[it];
            s_key[lp] = WK ? (SK)key[it] : (SK)d;
            if constexpr (VM == kValPairFirst) s_val[lp] = (uint16_t)(idx - b0);
            else s_val[lp] = val[it];
            if (TC) {
                const uint32_t x = key[it] & (kXDigits - 1), y = key[it] >> kXBits, c = x - x_first;
                if (c < (uint32_t)kTcCols) atomicAdd(&s_tc[c * kXDigits + y], 1u);
                else atomicAdd(&ro.tile_count[y * (uint32_t)ro.gx + x], 1u);
            }
        }
    }
    __syncthreads();
    if (TC) {  // integer sums: the counts do not depend on the order
        for (int i = tid; i < kTcCols * kXDigits; i += 256) {
            const uint32_t v = s_tc[i];
            if (v) atomicAdd(&ro.tile_count[(uint32_t)(i % kXDigits) * ro.gx + x_first + i / kXDigits], v);
        }
    }
    const int nvalid = n - b0 < (uint32_t)(256 * IPT) ? (int)(n - b0) : 256 * IPT;
    for (int i = tid; i < nvalid; i += 256) {
        const uint32_t k = s_key[i];
        const uint32_t dd = WK ? digit(k) : k;
        const uint32_t pos = dbase[dd] + (uint32_t)i;
        if (WK) keys_out[pos] = k;
        if constexpr (VM == kValPairFirst) {
            const uint32_t e = b0 + (uint32_t)s_val[i];
            V* dst = vals_out;
            if constexpr (DM) dst = dd == (uint32_t)kMsdCulled && ro.culled_out ? ro.culled_out : vals_out;
            dst[pos] = make_uint2(gauss_by_slot[e], e);
        } else {
            vals_out[pos] = s_val[i];
        }
    }
}

template <int BITS, int IPT>
static void radix_pass(const uint32_t* kin, const void* vin, uint32_t* kout, void* vout, const uint32_t* gauss_by_slot,
                       uint32_t n, int shift, bool idv, int vm, uint32_t* hist, uint32_t* totals, int nb,
                       RangeOut ro, const uint32_t* bias_not, hipStream_t s, const uint32_t* n_dev = nullptr) {
    // n_dev: the element count is read on the device (capped at n, the capacity the grid nb covers)
    constexpr int NDIG = 1 << BITS;
    const int bm = nb <= kScanBmRows ? 1 : 0;
    hipLaunchKernelGGL((k_radix_hist<BITS, IPT>), dim3(nb), dim3(256), 0, s, kin, n, shift, hist, nb, bm, bias_not,
                       n_dev, CountPublish{});
    if (bm)
        hipLaunchKernelGGL(k_radix_digit_scan, dim3(div_up(NDIG, kScanDigits)), dim3(kScanThreads), 0, s, hist, nb, NDIG,
                           totals, n_dev, n, 256 * IPT);
    else
        hipLaunchKernelGGL(k_radix_digit_scan_dm, dim3(NDIG), dim3(256), 0, s, hist, nb, totals, n_dev, n, 256 * IPT);
#define GS_SCATTER(IDV, VM)                                                                                   \
    hipLaunchKernelGGL((k_radix_scatter<BITS, IPT, IDV, VM>), dim3(nb), dim3(256), 0, s, kin, vin, kout, vout,  \
                       gauss_by_slot, n, shift, hist, totals, nb, bm, ro, bias_not, n_dev)
    if (vm == kValPairFirst && !kout)  // the last tile-sort pass: no sorted keys
        hipLaunchKernelGGL((k_radix_scatter<BITS, IPT, true, kValPairFirst, false>), dim3(nb), dim3(256), 0, s, kin,
                           vin, kout, vout, gauss_by_slot, n, shift, hist, totals, nb, bm, ro, bias_not, n_dev);
    else if (vm == kValPairFirst) GS_SCATTER(true, kValPairFirst);
    else if (vm == kValPair) GS_SCATTER(false, kValPair);
    else if (idv) GS_SCATTER(true, kValU32);
    else GS_SCATTER(false, kValU32);
#undef GS_SCATTER
}

static void radix_pass_bits(int bits, int ipt, const uint32_t* kin, const void* vin, uint32_t* kout, void* vout,
                            const uint32_t* gauss_by_slot, uint32_t n, int shift, bool idv, int vm, uint32_t* hist,
                            uint32_t* totals, int nb, RangeOut ro, const uint32_t* bias_not, hipStream_t s,
                            const uint32_t* n_dev) {
#define GS_CASE(B)                                                                                              \
    case B:                                                                                                     \
        if (ipt == kDepthSortIPT)                                                                               \
            radix_pass<B, kDepthSortIPT>(kin, vin, kout, vout, gauss_by_slot, n, shift, idv, vm, hist, totals, nb, ro, bias_not, s, n_dev); \
        else                                                                                                    \
            radix_pass<B, kSortIPT>(kin, vin, kout, vout, gauss_by_slot, n, shift, idv, vm, hist, totals, nb, ro, bias_not, s, n_dev); \
        break;
    switch (bits) {
        GS_CASE(1) GS_CASE(2) GS_CASE(3) GS_CASE(4) GS_CASE(5) GS_CASE(6)
        GS_CASE(7) GS_CASE(8) GS_CASE(9) GS_CASE(10) GS_CASE(11)
        default: break;
    }
#undef GS_CASE
}

// passes over [begin_bit, end_bit) with at most max_pass_bits per pass, bits split evenly
static int pass_bits(int begin_bit, int end_bit, int max_pass_bits, int p, int& shift) {
    const int passes = (end_bit - begin_bit + max_pass_bits - 1) / max_pass_bits;
    const int rem = end_bit - shift;
    (void)begin_bit;
    return (rem + (passes - p) - 1) / (passes - p);
}

int radix_sort_aux(uint32_t* key0, uint32_t* key1, uint2* pair0, uint2* pair1, const uint32_t* aux, uint32_t n,
                   int bits, int max_pass_bits, int ipt, uint32_t* hist, uint32_t* totals, int nblocks, hipStream_t s,
                   uint2* ranges, const uint32_t* key_bias_not, uint32_t* tile_order, int ntiles,
                   const uint32_t* n_dev) {
    uint32_t* k[2] = {key0, key1};
    uint2* v[2] = {pair0, pair1};
    int cur = 0;
    // max_pass_bits < 0: |max_pass_bits|-bit low passes, the remainder (<= 11 bits) in the last
    const int low = max_pass_bits < 0 ? -max_pass_bits : 0;
    const int passes = low ? 1 + (bits - kMaxSinglePassBits + low - 1) / low
                           : (bits + max_pass_bits - 1) / max_pass_bits;
    int shift = 0;
    for (int p = 0; p < passes; ++p) {
        const int b = low ? (p + 1 < passes ? low : bits - shift) : pass_bits(0, bits, max_pass_bits, p, shift);
        if (b < 1 || b > kMaxSinglePassBits) return -1;  // (histograms are sized for <= 11-bit digits)
        // a single pass given `ranges` writes the tile ranges and no sorted keys
        const bool ranges_here = ranges && passes == 1;
        radix_pass_bits(b, ipt, k[cur], v[cur], ranges_here ? nullptr : k[cur ^ 1], v[cur ^ 1], aux, n, shift,
                        p == 0, p == 0 ? kValPairFirst : kValPair, hist, totals, nblocks,
                        RangeOut{ranges_here ? ranges : nullptr, ranges_here ? tile_order : nullptr, ntiles},
                        p == 0 ? key_bias_not : nullptr, s, n_dev);
        cur ^= 1;
        shift += b;
    }
    return cur;
}

int tile_sort(uint32_t* key0, uint32_t* key1, uint2* pair0, uint2* pair1, const uint32_t* gauss_by_slot, uint32_t n,
              int bits, uint32_t* hist, uint32_t* totals, int nblocks, hipStream_t s, uint2* ranges,
              uint32_t* tile_order, int ntiles, const uint32_t* n_dev) {
    return radix_sort_aux(key0, key1, pair0, pair1, gauss_by_slot, n, bits, kMaxSinglePassBits, kSortIPT, hist, totals,
                          nblocks, s, ranges, nullptr, tile_order, ntiles, n_dev);
}

// ---------------------------------------------------------------------
// depth sort: MSD bucketing + per-bucket local sort (round 5)
// ---------------------------------------------------------------------
// The reference orders the instances by (tile, depth bits, Gaussian index) with one 64-bit cub sort
// (rasterizer_impl.cu:253-261); the emission here needs the Gaussians in (depth bits, index) order.  One
// stable 11-bit MSD pass (histogram, digit scan, scatter: the LSD kernels with msd_digit) puts every visible
// Gaussian into its depth bucket in index order; k_depth_bucket_sort then orders each bucket on the key
// bits below the bucket (the s bits of msd_params) in LDS, stable, so the result is the (key, index) order of
// a full stable sort for any key range: 4 launches where the 3-pass LSD sort took 9 (and a 32-bit fallback for
// ranges over 27 bits).  Buckets over kBucketCap keys (a dense depth band, measured max 1.6k at c2 and 3.6k
// at c4) take an in-kernel global-memory LSD over the bucket, one workgroup, correct at any size.
constexpr int kBucketIPT = 16, kBucketCap = 256 * kBucketIPT;
constexpr int kLocalBits = 7, kLocalDig = 1 << kLocalBits;

// Stable digit-major positions of one chunk (<= kBucketCap elements) held in registers: element j of the chunk
// is (wave w, it, lane) with j = w * 64 * ipt + it * 64 + lane, so the waves own consecutive stretches (the
// per-wave counters then rank in input order).  pos[it] <- the element's position in the chunk's digit-major
// order; s_start[d] / s_tot[d] <- digit d's run in the chunk.
template <int IPT>
__device__ __forceinline__ void chunk_rank(const uint32_t (&dig)[IPT], int ipt, uint32_t n, uint32_t (&pos)[IPT],
                                           uint16_t (*cnt)[kLocalDig], uint32_t* s_start, uint32_t* s_tot,
                                           uint32_t* lds4) {
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int i = tid; i < 4 * kLocalDig; i += 256) (&cnt[0][0])[i] = 0;
    __syncthreads();
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
        const uint32_t j = (uint32_t)(w * 64 * ipt + it * 64 + lane);
        const bool valid = it < ipt && j < n;
        const uint64_t vm = __ballot(valid);
        if (vm != 0) {  // (wave-uniform)
            const uint32_t d = valid ? dig[it] : 0u;
            const uint64_t peers = match_digit<kLocalBits>(d, vm);
            const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
            const uint32_t old = cnt[w][d];
            pos[it] = old + rank;
            if (valid && rank == 0) cnt[w][d] = (uint16_t)(old + (uint32_t)__popcll(peers));
        }
    }
    __syncthreads();
    uint32_t c0 = 0, c1 = 0, c2 = 0, tot = 0;
    if (tid < kLocalDig) {
        c0 = cnt[0][tid];
        c1 = cnt[1][tid];
        c2 = cnt[2][tid];
        tot = c0 + c1 + c2 + cnt[3][tid];
    }
    uint32_t all;
    const uint32_t run = block_exclusive_scan(tot, lds4, all);
    if (tid < kLocalDig) {
        cnt[0][tid] = (uint16_t)run;
        cnt[1][tid] = (uint16_t)(run + c0);
        cnt[2][tid] = (uint16_t)(run + c0 + c1);
        cnt[3][tid] = (uint16_t)(run + c0 + c1 + c2);
        s_start[tid] = run;
        s_tot[tid] = tot;
    }
    __syncthreads();
#pragma unroll
    for (int it = 0; it < IPT; ++it) {
        const uint32_t j = (uint32_t)(w * 64 * ipt + it * 64 + lane);
        if (it < ipt && j < n) pos[it] += cnt[w][dig[it]];
    }
}

// One workgroup per MSD bucket: keys_b / vals_b (the MSD pass's output: keys relative to kmin, (rect,
// Gaussian) values) -> vals_a in (key, index) order.  The culled bucket and buckets of one key value are
// copied (already in index order).
__global__ __launch_bounds__(256) void k_depth_bucket_sort(uint32_t* __restrict__ keys_b, uint2* __restrict__ vals_b,
                                                           uint32_t* __restrict__ keys_a, uint2* __restrict__ vals_a,
                                                           const uint2* __restrict__ ranges,
                                                           const uint32_t* __restrict__ bias_not) {
    __shared__ uint32_t s_key[kBucketCap];
    __shared__ uint16_t s_pos[kBucketCap];  // each staged key's position in the bucket (its value: re-read at the end)
    __shared__ uint16_t cnt[4][kLocalDig];
    __shared__ uint32_t s_start[kLocalDig], s_tot[kLocalDig], s_base[kLocalDig];
    __shared__ uint32_t lds4[4];
    const uint2 r = ranges[blockIdx.x];
    const uint32_t n = r.y - r.x;
    if (n == 0) return;
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const MsdParams m = msd_params(bias_not);
    const int passes = ((int)m.s + kLocalBits - 1) / kLocalBits;
    if (blockIdx.x == (uint32_t)kMsdCulled) return;  // (the MSD scatter wrote the culled bucket's values in place)
    if (passes == 0 || n == 1) {
        for (uint32_t i = tid; i < n; i += 256) vals_a[r.x + i] = vals_b[r.x + i];
        return;
    }
    uint32_t key[kBucketIPT], dig[kBucketIPT], pos[kBucketIPT];
    uint2 val[kBucketIPT];
    if (n <= (uint32_t)kBucketCap) {  // in LDS: every pass ranks the bucket held in registers
        const int ipt = (int)div_up_u(n, 256u);
        uint32_t src[kBucketIPT];  // the element's position in the bucket's input
#pragma unroll
        for (int it = 0; it < kBucketIPT; ++it) {
            const uint32_t j = (uint32_t)(w * 64 * ipt + it * 64 + lane);
            src[it] = j;
            if (it < ipt && j < n) key[it] = keys_b[r.x + j];
        }
        for (int p = 0; p < passes; ++p) {
#pragma unroll
            for (int it = 0; it < kBucketIPT; ++it) dig[it] = (key[it] >> (p * kLocalBits)) & (kLocalDig - 1);
            chunk_rank<kBucketIPT>(dig, ipt, n, pos, cnt, s_start, s_tot, lds4);
#pragma unroll
            for (int it = 0; it < kBucketIPT; ++it) {
                const uint32_t j = (uint32_t)(w * 64 * ipt + it * 64 + lane);
                if (it < ipt && j < n) {
                    s_key[pos[it]] = key[it];
                    s_pos[pos[it]] = (uint16_t)src[it];
                }
            }
            __syncthreads();
            if (p + 1 == passes) break;
#pragma unroll
            for (int it = 0; it < kBucketIPT; ++it) {
                const uint32_t j = (uint32_t)(w * 64 * ipt + it * 64 + lane);
                if (it < ipt && j < n) {
                    key[it] = s_key[j];
                    src[it] = s_pos[j];
                }
            }
            __syncthreads();  // (the next pass's counters and staging)
        }
        for (uint32_t i = tid; i < n; i += 256) vals_a[r.x + i] = vals_b[r.x + s_pos[i]];
        return;
    }
    // a bucket over kBucketCap keys: LSD passes over it in global memory, chunk after chunk in input order
    // (stable), ping-pong between the B and A copies of its range
    uint32_t* ks = keys_b;
    uint32_t* kd = keys_a;
    uint2* vs = vals_b;
    uint2* vd = vals_a;
    for (int p = 0; p < passes; ++p) {
        const int shift = p * kLocalBits;
        if (tid < kLocalDig) s_base[tid] = 0u;
        __syncthreads();
        for (uint32_t i = tid; i < n; i += 256) atomicAdd(&s_base[(ks[r.x + i] >> shift) & (kLocalDig - 1)], 1u);
        __syncthreads();
        {
            const uint32_t c = tid < kLocalDig ? s_base[tid] : 0u;
            uint32_t all;
            const uint32_t run = block_exclusive_scan(c, lds4, all);
            if (tid < kLocalDig) s_base[tid] = run;
        }
        __syncthreads();
        for (uint32_t c0 = 0; c0 < n; c0 += (uint32_t)kBucketCap) {
            const uint32_t cn = n - c0 < (uint32_t)kBucketCap ? n - c0 : (uint32_t)kBucketCap;
            const int ipt = (int)div_up_u(cn, 256u);
#pragma unroll
            for (int it = 0; it < kBucketIPT; ++it) {
                const uint32_t j = (uint32_t)(w * 64 * ipt + it * 64 + lane);
                if (it < ipt && j < cn) {
                    key[it] = ks[r.x + c0 + j];
                    val[it] = vs[r.x + c0 + j];
                }
                dig[it] = (key[it] >> shift) & (kLocalDig - 1);
            }
            chunk_rank<kBucketIPT>(dig, ipt, cn, pos, cnt, s_start, s_tot, lds4);
#pragma unroll
            for (int it = 0; it < kBucketIPT; ++it) {
                const uint32_t j = (uint32_t)(w * 64 * ipt + it * 64 + lane);
                if (it < ipt && j < cn) {
                    const uint32_t g = s_base[dig[it]] + pos[it] - s_start[dig[it]];
                    kd[r.x + g] = key[it];
                    vd[r.x + g] = val[it];
                }
            }
            __syncthreads();
            if (tid < kLocalDig) s_base[tid] += s_tot[tid];
            __syncthreads();
        }
        uint32_t* kt = ks; ks = kd; kd = kt;
        uint2* vt = vs; vs = vd; vd = vt;
    }
    if (vs != vals_a)  // (an even number of passes ends in the B copy)
        for (uint32_t i = tid; i < n; i += 256) vals_a[r.x + i] = vals_b[r.x + i];
}

int depth_sort_msd(uint32_t* key0, uint32_t* key1, uint2* pair0, uint2* pair1, const uint32_t* rect, uint32_t n,
                   uint32_t* hist, uint32_t* totals, int nblocks, uint2* bucket_ranges, const uint32_t* bias_not,
                   hipStream_t s, CountPublish pub) {
    if (n == 0) return 0;
    constexpr int IPT = kMsdIPT, NDIG = kMsdBuckets;
    nblocks = (int)div_up_u(n, 256u * IPT);  // (<= the table's rows: sized for kDepthSortTile-key blocks)
    const int bm = nblocks <= kScanBmRows ? 1 : 0;
    hipLaunchKernelGGL((k_radix_hist<kMsdBits, IPT, uint32_t, true>), dim3(nblocks), dim3(256), 0, s, key0, n, 0, hist,
                       nblocks, bm, bias_not, (const uint32_t*)nullptr, pub);
    if (bm)
        hipLaunchKernelGGL(k_radix_digit_scan, dim3(div_up(NDIG, kScanDigits)), dim3(kScanThreads), 0, s, hist, nblocks, NDIG,
                           totals, (const uint32_t*)nullptr, n, 256 * IPT);
    else
        hipLaunchKernelGGL(k_radix_digit_scan_dm, dim3(NDIG), dim3(256), 0, s, hist, nblocks, totals,
                           (const uint32_t*)nullptr, n, 256 * IPT);
    // (block 0 writes every bucket's range, as a single-pass tile sort writes the tile ranges)
    hipLaunchKernelGGL((k_radix_scatter<kMsdBits, IPT, true, kValPairFirst, true, false, uint32_t, true>), dim3(nblocks),
                       dim3(256), 0, s, key0, nullptr, key1, pair1, rect, n, 0, hist, totals, nblocks, bm,
                       RangeOut{bucket_ranges, nullptr, NDIG, nullptr, 0, pair0}, bias_not, (const uint32_t*)nullptr);
    hipLaunchKernelGGL(k_depth_bucket_sort, dim3(NDIG), dim3(256), 0, s, key1, pair1, key0, pair0, bucket_ranges,
                       bias_not);
    return 0;  // (the (rect, Gaussian) values in depth order are in pair0)
}

// ---------------------------------------------------------------------
// instance scan in depth order + emission
// ---------------------------------------------------------------------
// instances of a Gaussian from its depth-sort payload
__device__ __forceinline__ uint32_t rect_count(uint32_t v, int packed) {
    if (!packed) return v;
    return ((v >> 16 & 0xFFu) - (v & 0xFFu)) * ((v >> 24) - (v >> 8 & 0xFFu));
}

// Block sums of the instance counts in depth order (k_scan_emit derives each
// block's first slot from them).
__global__ __launch_bounds__(256) void k_scan_reduce(EmitArgs a) {
    __shared__ uint32_t lds4[4];
    uint32_t s = 0;
    const uint32_t base = blockIdx.x * (uint32_t)kScanTile;
    // (clamped loads, all issued before the first use: a guarded load per iteration was waited
    // for one at a time)
    uint32_t v[kScanIPT];
#pragma unroll
    for (int it = 0; it < kScanIPT; ++it) {
        const uint32_t r = base + it * 256 + threadIdx.x;
        v[it] = a.order[r < (uint32_t)a.P ? r : (uint32_t)a.P - 1u].x;
    }
#pragma unroll
    for (int it = 0; it < kScanIPT; ++it) {
        const uint32_t r = base + it * 256 + threadIdx.x;
        s += r < (uint32_t)a.P ? rect_count(v[it], a.rect_packed) : 0u;
    }
    uint32_t total;
    block_exclusive_scan(s, lds4, total);
    if (threadIdx.x == 0) a.scan_sums[blockIdx.x] = total;
    if (a.xhist) {  // two-level binning: the block's instances per tile column (rect height per column)
        __shared__ uint32_t h[kXDigits];
        if (threadIdx.x < kXDigits) h[threadIdx.x] = 0u;
        __syncthreads();
#pragma unroll
        for (int it = 0; it < kScanIPT; ++it) {
            const uint32_t r = base + it * 256 + threadIdx.x;
            const uint32_t q = v[it];
            const uint32_t x0 = q & 0xFFu, y0 = (q >> 8) & 0xFFu, x1 = (q >> 16) & 0xFFu, y1 = q >> 24;
            if (r < (uint32_t)a.P && y1 > y0)
                for (uint32_t x = x0; x < x1; ++x) atomicAdd(&h[x], y1 - y0);
        }
        __syncthreads();
        if (threadIdx.x < kXDigits) a.xhist[(size_t)blockIdx.x * kXDigits + threadIdx.x] = h[threadIdx.x];
    }
    if (a.thist) {
        // direct emission: the block's instances per tile.  A rect adds +1 at (x0, y0), -1 at (x1, y0) and
        // (x0, y1), +1 at (x1, y1) (corners past the grid dropped); prefix sums along x, then along y, give
        // every tile's count: four LDS atomics per Gaussian whatever its size.  Rows are gx + 1 apart (odd:
        // the row pass's lanes, one row each, hit distinct banks); each prefix runs in registers, 16 cells
        // loaded at a time, one thread per row (gy <= 255), then one per column (gx <= 255).
        constexpr int kCells = (1 << kMaxSinglePassBits) + kRectPackMax;  // gx * gy + gy cells at most
        __shared__ int s_d[kCells];
        const int gx = a.gx, gy = a.gy, nt = a.ntiles, gp = gx + 1;
        for (int t = threadIdx.x; t < gy * gp; t += 256) s_d[t] = 0;
        __syncthreads();
#pragma unroll
        for (int it = 0; it < kScanIPT; ++it) {
            const uint32_t r = base + it * 256 + threadIdx.x;
            const uint32_t q = v[it];
            const int x0 = (int)(q & 0xFFu), y0 = (int)((q >> 8) & 0xFFu), x1 = (int)((q >> 16) & 0xFFu),
                      y1 = (int)(q >> 24);
            if (r < (uint32_t)a.P && x1 > x0 && y1 > y0) {
                atomicAdd(&s_d[y0 * gp + x0], 1);
                if (x1 < gx) atomicAdd(&s_d[y0 * gp + x1], -1);
                if (y1 < gy) {
                    atomicAdd(&s_d[y1 * gp + x0], -1);
                    if (x1 < gx) atomicAdd(&s_d[y1 * gp + x1], 1);
                }
            }
        }
        __syncthreads();
        auto prefix = [&](int first, int n, int stride) {  // inclusive prefix of s_d[first + i * stride], i < n
            int run = 0;
            for (int i0 = 0; i0 < n; i0 += 16) {
                int c[16];
#pragma unroll
                for (int i = 0; i < 16; ++i) c[i] = i0 + i < n ? s_d[first + (i0 + i) * stride] : 0;
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    run += c[i];
                    if (i0 + i < n) s_d[first + (i0 + i) * stride] = run;
                }
            }
        };
        if ((int)threadIdx.x < gy) prefix((int)threadIdx.x * gp, gx, 1);
        __syncthreads();
        if ((int)threadIdx.x < gx) prefix((int)threadIdx.x, gy, gp);
        __syncthreads();
        const int bm = a.scan_blocks <= kScanBmRows ? 1 : 0;
        for (int t = threadIdx.x; t < nt; t += 256)
            a.thist[hist_at(bm, blockIdx.x, (uint32_t)t, a.scan_blocks, nt)] = (uint32_t)s_d[(t / gx) * gp + t % gx];
    }
}

// Emission in depth order: rounds of 256 Gaussians; a block scan of their
// instance counts gives each its first slot, then the round's instances are
// expanded cooperatively — thread j writes slot base+j, finding its Gaussian
// by binary search over the round's start offsets in LDS — so every store of
// a wave is coalesced (duplicateWithKeys, rasterizer_impl.cu:67-100, writes
// per Gaussian instead).
__global__ __launch_bounds__(256) void k_scan_emit(EmitArgs a) {
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t s_start[256];
    __shared__ uint32_t s_gauss[256];
    __shared__ int4 s_rect[256];  // x0, y0, width, -
    // the block's first slot: the sum of the block sums before it (k_scan_reduce's, read from L2:
    // at most scan_blocks words; this replaced a one-workgroup top-level scan launch)
    uint32_t base;
    {
        uint32_t part = 0;
        part = strided_part(a.scan_sums, blockIdx.x);
        block_exclusive_scan(part, lds4, base);
    }
    const uint32_t r_block = blockIdx.x * (uint32_t)kScanTile;
    // every round's inputs loaded up front (one memory round trip instead of dependent ones per round):
    // (rect, Gaussian), and where the rect is not packed the Splat's 2D mean and the radius it comes from
    uint2 grs[kScanIPT];
    float2 xys[kScanIPT];
    int rads[kScanIPT];
#pragma unroll
    for (int it = 0; it < kScanIPT; ++it) {
        const uint32_t r = r_block + it * 256 + threadIdx.x;
        grs[it] = r < (uint32_t)a.P ? a.order[r] : make_uint2(0u, 0u);
    }
#pragma unroll
    for (int it = 0; it < kScanIPT; ++it) {
        const uint32_t c = rect_count(grs[it].x, a.rect_packed), g = grs[it].y;
        xys[it] = c && !a.rect_packed ? a.splat[g].xy : make_float2(0.f, 0.f);
        rads[it] = c && !a.rect_packed ? a.radii[g] : 0;
    }
#pragma unroll  // (the prefetched arrays stay in registers)
    for (int it = 0; it < kScanIPT; ++it) {
        const uint2 gr = grs[it];
        const uint32_t g = gr.y;
        const uint32_t c = rect_count(gr.x, a.rect_packed);
        uint32_t total;
        const uint32_t off = block_exclusive_scan(c, lds4, total);
        if (c) {
            a.first_slot[g] = base + off;
            Rect q;
            if (a.rect_packed) {
                q.x0 = (int)(gr.x & 0xFFu); q.y0 = (int)((gr.x >> 8) & 0xFFu);
                q.x1 = (int)((gr.x >> 16) & 0xFFu); q.y1 = (int)(gr.x >> 24);
            } else {
                q = tile_rect(xys[it].x, xys[it].y, rads[it], a.gx, a.gy);
            }
            s_rect[threadIdx.x] = make_int4(q.x0, q.y0, q.x1 - q.x0, 0);
        }
        s_start[threadIdx.x] = off;
        s_gauss[threadIdx.x] = g;
        __syncthreads();
        for (uint32_t j = threadIdx.x; j < total; j += 256) {
            // owner: the last entry with start <= j.  Starts are an exclusive scan (non-decreasing); an
            // empty entry shares its start with the later entry that owns that slot, so it is never last.
            int lo = 0, hi = 255;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (s_start[mid] <= j) lo = mid;
                else hi = mid - 1;
            }
            const int4 q = s_rect[lo];
            const uint32_t k = j - s_start[lo];
            const uint32_t ky = (uint32_t)(((float)k + 0.5f) / (float)q.z);  // exact: k < 2^20, margin 0.5/width
            const uint32_t kx = k - ky * (uint32_t)q.z;
            if (base + j >= a.cap) break;  // speculative capacity exceeded (gs_views_check reports it)
            a.tile_key[base + j] = (uint32_t)((q.y + (int)ky) * a.gx + q.x + (int)kx);
            a.slot_gauss[base + j] = s_gauss[lo];
            if (a.rec_flags32) a.rec_flags32[base + j] = 0u;  // slot's four quadrant flags (no memset launch)
        }
        base += total;
        __syncthreads();
    }
}

// Direct emission (round 5; single-pass grids with packed rects, direct_emission_grid): the emission writes
// every instance straight to its place in its tile's list, so the tile sort (histogram, digit scan, scatter
// over the K emitted keys) is gone.  k_scan_reduce counted each block's instances per tile and
// launch_scan_reduce scanned those counts over the blocks, so block b's instances of tile t start at
// (instances of tiles < t) + (tile t's instances in blocks < b).  Inside the block, instances are taken in
// slot order (= depth order: the block's Gaussians by rank, each one's tiles row-major) in batches of
// kEtBatch: the owner of every instance is a prefix max over marks at the Gaussians' first slots, each
// instance is ranked among the batch's instances of its tile with 64-lane ballots and per-wave counters
// (waves own consecutive stretches of the batch, so ranks follow slot order: stable), staged in LDS in
// tile-major order and stored with consecutive lanes on consecutive positions of each tile's run.  The lists
// are therefore the single-pass tile sort's (Gaussian, slot) pairs, bit for bit.  Block 0 also writes the
// tile ranges and the forward's dispatch order.  IDS: the Gaussian id alone (EmitArgs::ids_only).
#ifndef GS_EMIT_TILE_EPT
#define GS_EMIT_TILE_EPT 16  // instances per thread of a batch (A/B)
#endif
constexpr int kEtEPT = GS_EMIT_TILE_EPT, kEtBatch = 256 * kEtEPT;
static_assert(kEtBatch <= 65536 && kScanTile < 65535, "u16 staged positions and owners");
template <int BITS, bool IDS>
__global__ __launch_bounds__(256) void k_emit_tiles(EmitArgs a) {
    constexpr int NDIG = 1 << BITS, PER = NDIG >= 256 ? NDIG / 256 : 1;
    constexpr int GPT = kScanTile / 256;  // consecutive Gaussians (depth ranks) per thread
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t s_start[kScanTile];  // each Gaussian's first instance, relative to the block's first slot
    __shared__ uint32_t s_rect[kScanTile];   // its packed tile rect
    __shared__ uint16_t s_own[kEtBatch];     // the batch's owners (+1): marks at the Gaussians' starts, prefix max
    __shared__ uint16_t cnt[4][NDIG];        // per-wave tile counters, then the staged runs' starts
    // per tile: the global position of the block's next instance; while a batch is stored, its run's global
    // position minus its staged position
    __shared__ uint32_t s_pos[NDIG];
    __shared__ uint16_t s_idx[kEtBatch];     // staged, tile-major: the instance's position in the batch
    __shared__ uint32_t s_carry;
    __shared__ uint32_t s_magic[256];
    fill_div_magic(s_magic);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int nt = a.ntiles;
    const uint32_t r_block = blockIdx.x * (uint32_t)kScanTile;
    for (int i = tid; i < 4 * NDIG; i += 256) (&cnt[0][0])[i] = 0;
    uint32_t base;  // the block's first slot (as k_scan_emit)
    {
        uint32_t part = 0;
        part = strided_part(a.scan_sums, blockIdx.x);
        block_exclusive_scan(part, lds4, base);
    }
    {   // each tile's first position for this block; block 0: the ranges and the dispatch order
        const int bm = a.scan_blocks <= kScanBmRows ? 1 : 0;
        uint32_t c[PER], h[PER];
        uint32_t s = 0;
        // (totals and this block's row loaded together, clamped: no load waits alone)
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int d = min(tid * PER + i, nt - 1);
            c[i] = a.ttotals[d];
            h[i] = a.thist[hist_at(bm, blockIdx.x, (uint32_t)d, a.scan_blocks, nt)];
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            if (tid * PER + i >= nt) c[i] = 0u;
            s += c[i];
        }
        uint32_t all;
        const uint32_t run0 = block_exclusive_scan(s, lds4, all);
        uint32_t run = run0;
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int d = tid * PER + i;
            s_pos[d] = d < nt ? run + h[i] : 0u;
            run += c[i];
        }
        if (blockIdx.x == 0) write_tile_ranges<PER>(c, run0, nt, a.ranges, a.tile_order, a.cap);
    }
    // the block's Gaussians, GPT consecutive ranks per thread: first slots, rects
    const uint32_t r0 = r_block + (uint32_t)(tid * GPT);
    uint32_t gst[GPT], gc[GPT];
    uint32_t total;
    {
        uint2 gr[GPT];
#pragma unroll
        for (int i = 0; i < GPT; ++i) gr[i] = a.order[min(r0 + i, (uint32_t)a.P - 1)];  // (clamped: loads together)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < GPT; ++i)
            if (r0 + i >= (uint32_t)a.P) gr[i] = make_uint2(0u, 0u);
        uint32_t s = 0;
#pragma unroll
        for (int i = 0; i < GPT; ++i) {
            gc[i] = rect_count(gr[i].x, 1);
            s += gc[i];
        }
        uint32_t off = block_exclusive_scan(s, lds4, total);
#pragma unroll
        for (int i = 0; i < GPT; ++i) {
            gst[i] = off;
            s_start[tid * GPT + i] = off;
            s_rect[tid * GPT + i] = gr[i].x;
            if (gc[i]) a.first_slot[gr[i].y] = base + off;
            off += gc[i];
        }
    }
    if (tid == 0) s_carry = 0u;
    // instance j of the block (relative to its first slot) owned by block Gaussian o: its tile
    auto tile_of = [&](uint32_t j, int o) {
        const uint32_t q = s_rect[o];
        const uint32_t x0 = q & 0xFFu, y0 = (q >> 8) & 0xFFu, wd = ((q >> 16) & 0xFFu) - x0;
        const uint32_t k = j - s_start[o];
        const uint32_t ky = div_small(k, wd, s_magic);
        return (y0 + ky) * (uint32_t)a.gx + x0 + (k - ky * wd);
    };
    for (uint32_t j0 = 0; j0 < total; j0 += (uint32_t)kEtBatch) {
        const uint32_t nb = total - j0 < (uint32_t)kEtBatch ? total - j0 : (uint32_t)kEtBatch;
        // owner of every instance of the batch: marks at the starts of the Gaussians starting in it (starts of
        // Gaussians with instances are distinct), prefix max, carried in from the previous batch
#pragma unroll
        for (int i = 0; i < kEtEPT; ++i) s_own[tid * kEtEPT + i] = 0;
        __syncthreads();
#pragma unroll
        for (int i = 0; i < GPT; ++i)
            if (gc[i] && gst[i] >= j0 && gst[i] < j0 + nb) s_own[gst[i] - j0] = (uint16_t)(tid * GPT + i + 1);
        const uint32_t carry = s_carry;
        __syncthreads();
        {
            uint32_t run = 0;
#pragma unroll
            for (int i = 0; i < kEtEPT; ++i) run = max(run, (uint32_t)s_own[tid * kEtEPT + i]);
            run = max(carry, block_exclusive_max(run, lds4));
#pragma unroll
            for (int i = 0; i < kEtEPT; ++i) {
                run = max(run, (uint32_t)s_own[tid * kEtEPT + i]);
                s_own[tid * kEtEPT + i] = (uint16_t)run;
            }
        }
        __syncthreads();
        uint32_t dg[kEtEPT], loc[kEtEPT];
#pragma unroll
        for (int e = 0; e < kEtEPT; ++e) {
            const uint32_t jj = (uint32_t)(w * 64 * kEtEPT + e * 64 + lane);
            const bool valid = jj < nb;
            const uint64_t vm = __ballot(valid);
            dg[e] = 0u;
            loc[e] = 0u;
            if (vm != 0) {  // (wave-uniform; no break: the loop stays unrolled)
                const uint32_t d = valid ? tile_of(j0 + jj, (int)s_own[jj] - 1) : 0u;
                const uint32_t slot = base + j0 + jj;
                if (valid && a.rec_flags32 && slot < a.cap) a.rec_flags32[slot] = 0u;  // (slot order: coalesced)
                const uint64_t peers = match_digit<BITS>(d, vm);
                const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
                const uint32_t old = cnt[w][d];
                dg[e] = d;
                loc[e] = old + rank;
                if (valid && rank == 0) cnt[w][d] = (uint16_t)(old + (uint32_t)__popcll(peers));
            }
        }
        __syncthreads();
        {   // the batch's tile runs (wave-major inside a tile) and their global bases
            uint32_t t4[PER][4];
            uint32_t s = 0;
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int d = tid * PER + i;
#pragma unroll
                for (int v = 0; v < 4; ++v) t4[i][v] = cnt[v][d];
                s += t4[i][0] + t4[i][1] + t4[i][2] + t4[i][3];
            }
            uint32_t all;
            uint32_t run = block_exclusive_scan(s, lds4, all);
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int d = tid * PER + i;
                cnt[0][d] = (uint16_t)run;
                cnt[1][d] = (uint16_t)(run + t4[i][0]);
                cnt[2][d] = (uint16_t)(run + t4[i][0] + t4[i][1]);
                cnt[3][d] = (uint16_t)(run + t4[i][0] + t4[i][1] + t4[i][2]);
                s_pos[d] -= run;
                run += t4[i][0] + t4[i][1] + t4[i][2] + t4[i][3];
            }
        }
        __syncthreads();
#pragma unroll
        for (int e = 0; e < kEtEPT; ++e) {
            const uint32_t jj = (uint32_t)(w * 64 * kEtEPT + e * 64 + lane);
            if (jj < nb) s_idx[cnt[w][dg[e]] + loc[e]] = (uint16_t)jj;
        }
        __syncthreads();
        // every staged instance's loads issued before the stores (fixed trip count, unrolled; the scheduling
        // barrier keeps the ids-only build from storing each id as its load returns: 16 round trips a batch)
        if constexpr (IDS) {  // (the pairs build batches its loads by itself, and this form measured slower there)
        uint32_t st_pos[kEtEPT], st_g[kEtEPT], st_j[kEtEPT];
#pragma unroll
        for (int e = 0; e < kEtEPT; ++e) {
            const uint32_t i = (uint32_t)(e * 256 + tid);
            const uint32_t jj = i < nb ? s_idx[i] : 0u;
            const int o = i < nb ? (int)s_own[jj] - 1 : 0;
            st_pos[e] = i < nb ? s_pos[tile_of(j0 + jj, o)] + i : 0xFFFFFFFFu;
            st_g[e] = a.order[r_block + (uint32_t)o].y;  // (the block's own entries: L2; o valid either way)
            st_j[e] = jj;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int e = 0; e < kEtEPT; ++e) {
            // (speculative capacity: gs_views_check reports an overflow; an overflowed binning is redone,
            // but until then its lists must stay inside the buffer: the ranges are clamped to the
            // capacity, and so is every slot — the backward's record address)
            const uint32_t pos = st_pos[e];
            if (pos < a.cap) reinterpret_cast<uint32_t*>(a.pairs_out)[pos] = st_g[e];
        }
        (void)st_j;
        } else {
#pragma unroll
        for (int e = 0; e < kEtEPT; ++e) {
            const uint32_t i = (uint32_t)(e * 256 + tid);
            if (i < nb) {
                const uint32_t jj = s_idx[i];
                const int o = (int)s_own[jj] - 1;
                const uint32_t pos = s_pos[tile_of(j0 + jj, o)] + i;
                const uint32_t g = a.order[r_block + (uint32_t)o].y;  // (the block's own entries: L2)
                // (speculative capacity: gs_views_check reports an overflow; an overflowed binning is redone,
                // but until then its lists must stay inside the buffer: the ranges are clamped to the
                // capacity, and so is every slot — the backward's record address)
                if (pos < a.cap) a.pairs_out[pos] = make_uint2(g, min(base + j0 + jj, a.cap - 1u));
            }
        }
        }
        __syncthreads();
        // the next batch's positions: each tile's run ends where the next tile's begins (the batch's end
        // for the last digit)
#pragma unroll
        for (int i = 0; i < PER; ++i) {
            const int d = tid * PER + i;
            s_pos[d] += d + 1 < NDIG ? (uint32_t)cnt[0][d + 1] : nb;
        }
        if (tid == 0) s_carry = s_own[nb - 1];
        __syncthreads();
        for (int i = tid; i < 4 * NDIG; i += 256) (&cnt[0][0])[i] = 0;
    }
}

// Two-level binning, first level: the emission writes every instance straight
// into its tile column's run (the first LSD pass of the tile sort, digit = x),
// stable — instances of one column in emission (depth) order.  Each block's
// column runs start at the scanned k_scan_reduce counts; the round's instances
// are expanded in batches of kEmitBatch, ranked per column with 64-lane ballots
// and per-wave counters (waves own consecutive stretches of the batch, as in
// k_radix_scatter), staged in LDS in column-major order and stored with
// consecutive lanes on consecutive positions of each column run.  The key
// written is y << 7 | x (the row pass's digit and the tile's column).
// IDS: the (Gaussian, slot) pair's Gaussian alone (EmitArgs::ids_only)
#ifndef GS_EMIT_EPT
#define GS_EMIT_EPT 8  // instances per thread of an emission batch (A/B: -DGS_EMIT_EPT=...)
#endif
constexpr int kEmitEPT = GS_EMIT_EPT, kEmitBatch = 256 * kEmitEPT;
template <bool IDS>
__global__ __launch_bounds__(256) void k_scan_emit_x(EmitArgs a) {
    using PV = typename std::conditional<IDS, uint32_t, uint2>::type;
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t s_start[256];
    __shared__ uint32_t s_gauss[256];
    __shared__ int4 s_rect[256];
    __shared__ uint32_t s_dpos[kXDigits];   // global position of the block's next instance per column
    __shared__ uint32_t s_gbase[kXDigits];  // the batch's column run: global position - staged position
    __shared__ uint16_t cnt[4][kXDigits];   // per-wave column counters, then the staged run starts
    __shared__ uint16_t s_key[kEmitBatch];
    __shared__ PV s_pair[kEmitBatch];
    __shared__ uint16_t s_own[kEmitBatch];  // the batch's owners (+1): marks at the entries' starts, prefix max
    __shared__ uint32_t s_carry;
    __shared__ uint32_t s_magic[256];
    fill_div_magic(s_magic);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    if (blockIdx.x == 0)
        for (int t = tid; t < a.ntiles; t += 256) a.tile_count[t] = 0u;  // (the row pass counts into it)
    uint32_t base;
    {
        uint32_t part = 0;
        part = strided_part(a.scan_sums, blockIdx.x);
        block_exclusive_scan(part, lds4, base);
    }
    {
        const uint32_t tv = tid < kXDigits ? a.xtotals[tid] : 0u;
        uint32_t all;
        const uint32_t run = block_exclusive_scan(tv, lds4, all);
        if (tid < kXDigits) s_dpos[tid] = run + a.xhist[(size_t)blockIdx.x * kXDigits + tid];
    }
    for (int i = tid; i < 4 * kXDigits; i += 256) (&cnt[0][0])[i] = 0;
    __syncthreads();
    const uint32_t r_block = blockIdx.x * (uint32_t)kScanTile;
    uint2 grs[kScanIPT];  // every round's (rect, Gaussian) up front (as k_scan_emit)
#pragma unroll
    for (int it = 0; it < kScanIPT; ++it) {
        const uint32_t r = r_block + it * 256 + tid;
        grs[it] = r < (uint32_t)a.P ? a.order[r] : make_uint2(0u, 0u);
    }
#pragma unroll  // (the prefetched arrays stay in registers)
    for (int it = 0; it < kScanIPT; ++it) {
        const uint2 gr = grs[it];
        const uint32_t g = gr.y;
        const uint32_t c = rect_count(gr.x, 1);
        uint32_t total;
        const uint32_t off = block_exclusive_scan(c, lds4, total);
        if (c) {
            a.first_slot[g] = base + off;
            s_rect[tid] = make_int4((int)(gr.x & 0xFFu), (int)((gr.x >> 8) & 0xFFu),
                                    (int)((gr.x >> 16) & 0xFFu) - (int)(gr.x & 0xFFu), 0);
        }
        s_start[tid] = off;
        s_gauss[tid] = g;
        __syncthreads();
        for (uint32_t j0 = 0; j0 < total; j0 += kEmitBatch) {
            const uint32_t nb = total - j0 < (uint32_t)kEmitBatch ? total - j0 : (uint32_t)kEmitBatch;
            uint32_t kk[kEmitEPT], loc[kEmitEPT];
            PV pv[kEmitEPT];
            // owner of every instance of the batch (the last entry with start <= j, see k_scan_emit) as a
            // prefix max over the batch of the entries' marks at their starts: one LDS read per instance
            // instead of a binary search of eight dependent reads
            {
                uint32_t carry = 0;  // owner of j0 (+1), from a search over the round's starts
                if (tid == 0) {
                    int lo = 0, hi = 255;
                    while (lo < hi) {
                        const int mid = (lo + hi + 1) >> 1;
                        if (s_start[mid] <= j0) lo = mid;
                        else hi = mid - 1;
                    }
                    s_carry = (uint32_t)lo + 1u;
                }
#pragma unroll
                for (int i = 0; i < kEmitEPT; ++i) s_own[tid * kEmitEPT + i] = 0;
                __syncthreads();
                const uint32_t st = s_start[tid];
                if (c && st >= j0 && st < j0 + nb) s_own[st - j0] = (uint16_t)(tid + 1);  // (starts of c > 0: distinct)
                carry = s_carry;
                __syncthreads();
                uint32_t run = 0;
#pragma unroll
                for (int i = 0; i < kEmitEPT; ++i) run = max(run, (uint32_t)s_own[tid * kEmitEPT + i]);
                run = max(carry, block_exclusive_max(run, lds4));
#pragma unroll
                for (int i = 0; i < kEmitEPT; ++i) {
                    run = max(run, (uint32_t)s_own[tid * kEmitEPT + i]);
                    s_own[tid * kEmitEPT + i] = (uint16_t)run;
                }
                __syncthreads();
            }
#pragma unroll
            for (int e = 0; e < kEmitEPT; ++e) {
                const uint32_t jj = (uint32_t)(w * 64 * kEmitEPT + e * 64 + lane);
                const bool valid = jj < nb;
                const uint64_t vm = __ballot(valid);
                if (vm == 0) break;
                const uint32_t j = j0 + (valid ? jj : 0u);
                const int lo = (int)s_own[valid ? jj : 0u] - 1;
                const int4 q = s_rect[lo];
                const uint32_t k = j - s_start[lo];
                const uint32_t ky = div_small(k, (uint32_t)q.z, s_magic);
                const uint32_t kx = k - ky * (uint32_t)q.z;
                const uint32_t x = (uint32_t)q.x + kx, y = (uint32_t)q.y + ky;
                kk[e] = y << kXBits | x;
                if constexpr (IDS) pv[e] = s_gauss[lo];
                else pv[e] = make_uint2(s_gauss[lo], base + j);
                if (valid && a.rec_flags32 && base + j < a.cap) a.rec_flags32[base + j] = 0u;  // (slot order: coalesced)
                const uint32_t d = valid ? x : 0u;
                const uint64_t peers = match_digit<kXBits>(d, vm);
                const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
                const uint32_t old = cnt[w][d];
                loc[e] = old + rank;
                if (valid && rank == 0) cnt[w][d] = (uint16_t)(old + (uint32_t)__popcll(peers));
            }
            __syncthreads();
            {   // staged column runs of the batch (wave-major inside a column), their global bases
                uint32_t c0 = 0, c1 = 0, c2 = 0, tot = 0;
                if (tid < kXDigits) {
                    c0 = cnt[0][tid];
                    c1 = cnt[1][tid];
                    c2 = cnt[2][tid];
                    tot = c0 + c1 + c2 + cnt[3][tid];
                }
                uint32_t all;
                const uint32_t run = block_exclusive_scan(tot, lds4, all);
                if (tid < kXDigits) {
                    cnt[0][tid] = (uint16_t)run;
                    cnt[1][tid] = (uint16_t)(run + c0);
                    cnt[2][tid] = (uint16_t)(run + c0 + c1);
                    cnt[3][tid] = (uint16_t)(run + c0 + c1 + c2);
                    s_gbase[tid] = s_dpos[tid] - run;
                    s_dpos[tid] += tot;
                }
            }
            __syncthreads();
#pragma unroll
            for (int e = 0; e < kEmitEPT; ++e) {
                const uint32_t jj = (uint32_t)(w * 64 * kEmitEPT + e * 64 + lane);
                if (jj < nb) {
                    const uint32_t lp = cnt[w][kk[e] & (kXDigits - 1)] + loc[e];
                    s_key[lp] = (uint16_t)kk[e];
                    s_pair[lp] = pv[e];
                }
            }
            __syncthreads();
            for (uint32_t i = tid; i < nb; i += 256) {
                const uint32_t kv = s_key[i];
                const uint32_t pos = s_gbase[kv & (kXDigits - 1)] + i;
                if (pos < a.cap) {  // (speculative capacity: gs_views_check reports an overflow)
                    reinterpret_cast<uint16_t*>(a.tile_key)[pos] = (uint16_t)kv;  // (the row pass reads u16 keys)
                    if constexpr (IDS) reinterpret_cast<uint32_t*>(a.pairs_out)[pos] = s_pair[i];
                    else a.pairs_out[pos] = s_pair[i];
                }
            }
            for (int i = tid; i < 4 * kXDigits; i += 256) (&cnt[0][0])[i] = 0;
            __syncthreads();
        }
        base += total;
        __syncthreads();
    }
}

// Tile ranges from the per-tile instance counts (one workgroup): an exclusive
// scan in tile order — the ranges identifyTileRanges (rasterizer_impl.cu:105-125)
// finds in the sorted keys; empty tiles keep (0, 0).
// Each thread's run of counts is loaded at once into registers (one memory round trip instead of one
// per count).  Two-level grids have at most 128 x 128 tiles.  Also the forward's dispatch order
// (k_tile_order's: tiles by list length, longest first) from the same counts, when tile_order is set.
constexpr int kRangesPer = kXDigits * kXDigits / 256;
// cap: a speculative forward's binning capacity (the band emission's counts are the full instance counts:
// ranges clamped to it, as write_tile_ranges does); starts: every tile's first position, unclamped (the band
// emission's bases), when set
__global__ __launch_bounds__(256) void k_ranges_counts(const uint32_t* __restrict__ count, int tiles,
                                                       uint2* __restrict__ ranges, uint32_t* __restrict__ tile_order,
                                                       uint32_t cap, uint32_t* __restrict__ starts) {
    __shared__ uint32_t lds4[4];
    constexpr int kClasses = 64;
    __shared__ uint32_t s_cls[kClasses];
    auto cls = [](uint32_t len) { return min(kClasses - 1, (int)(__log2f((float)len + 1.0f) * 3.0f)); };
    if (threadIdx.x < kClasses) s_cls[threadIdx.x] = 0u;
    const int per = (tiles + 255) / 256, t0 = threadIdx.x * per;
    uint32_t c[kRangesPer];
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < kRangesPer; ++i) c[i] = i < per && t0 + i < tiles ? count[t0 + i] : 0u;
#pragma unroll
    for (int i = 0; i < kRangesPer; ++i) s += c[i];
    uint32_t all;
    uint32_t run = block_exclusive_scan(s, lds4, all);
#pragma unroll
    for (int i = 0; i < kRangesPer; ++i) {
        const int t = t0 + i;
        if (i < per && t < tiles) {
            ranges[t] = c[i] ? make_uint2(min(run, cap), min(run + c[i], cap)) : make_uint2(0u, 0u);
            if (starts) starts[t] = run;
            run += c[i];
            if (tile_order) atomicAdd(&s_cls[cls(c[i])], 1u);
        }
    }
    if (!tile_order) return;
    __syncthreads();
    if (threadIdx.x == 0) {  // start of each class, longest class first
        uint32_t acc = 0;
        for (int k = kClasses - 1; k >= 0; --k) {
            const uint32_t m = s_cls[k];
            s_cls[k] = acc;
            acc += m;
        }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < kRangesPer; ++i) {
        const int t = t0 + i;
        if (i < per && t < tiles) tile_order[atomicAdd(&s_cls[cls(c[i])], 1u)] = (uint32_t)t;
    }
}

// ---------------------------------------------------------------------
// region emission (round 6; region_emission_grid: 2049..kRegionMaxTiles tiles, packed rects — c4's 120 x 68)
// ---------------------------------------------------------------------
// The direct emission's idea (every instance written once, straight to its place in its tile's list) for grids
// too large for its per-(1024-Gaussian block, tile) tables.  The depth order is cut into chunks of kChunkG
// Gaussians, the grid into regions of region_rows tile rows (~1024 tiles):
//   k_chunk_count  the chunk's instances per tile (a rect adds +-1 at its four corners in LDS, then prefix sums
//                  along x and y), one table row per chunk; also every Gaussian's first slot (emission order) and,
//                  for a training binning, the zeroed record flags of the chunk's slots;
//   digit scan     over the chunks per tile (in place: each chunk's first position relative to its tile's
//                  start) and the tile totals; k_ranges_counts: ranges, dispatch order, the tiles' starts;
//   k_region_emit  one workgroup per (chunk, region): the chunk's Gaussians that reach the region are appended
//                  in depth order to an LDS list (one block scan per 1024 ranks), and the list's instances inside
//                  the region are expanded in batches as in k_emit_tiles — owner = prefix max over marks at the
//                  entries' first instances, rank among the batch's instances of the tile by 64-lane ballots and
//                  per-wave counters (stable), staged tile-major in LDS — and stored as per-tile runs (~32 ids
//                  at c4: coalesced, where one store per instance at its final place measured 5x slower).
// Per tile the instances come chunk by chunk, Gaussian by Gaussian in depth order: the lists are the tile sort's,
// bit for bit (and the (Gaussian, slot) pairs carry the emission-order slot, first slot + the instance's
// row-major index in its rect).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ uint32_t dpp_u32(uint32_t v) {
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, CTRL, ROW_MASK, 0xF, false);
}
// 64-lane inclusive scan with DPP row shifts and row broadcasts (no LDS crossbar trip per step)
__device__ __forceinline__ uint32_t wave_incl_scan_u32(uint32_t v) {
    v += dpp_u32<0x111, 0xF>(v);  // row_shr:1
    v += dpp_u32<0x112, 0xF>(v);  // row_shr:2
    v += dpp_u32<0x114, 0xF>(v);  // row_shr:4
    v += dpp_u32<0x118, 0xF>(v);  // row_shr:8
    v += dpp_u32<0x142, 0xA>(v);  // row_bcast:15 into rows 1, 3
    v += dpp_u32<0x143, 0xC>(v);  // row_bcast:31 into rows 2, 3
    return v;
}
// NT-thread exclusive scan; `total` receives the workgroup sum
template <int NT>
__device__ __forceinline__ uint32_t block_excl_scan_n(uint32_t v, uint32_t* lds, uint32_t& total) {
    constexpr int NW = NT / 64;
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint32_t x = wave_incl_scan_u32(v);
    if (lane == 63) lds[w] = x;
    __syncthreads();
    uint32_t base = 0, t = 0;
#pragma unroll
    for (int i = 0; i < NW; ++i) {
        const uint32_t c = lds[i];
        base += i < w ? c : 0u;
        t += c;
    }
    __syncthreads();
    total = t;
    return base + x - v;
}

constexpr int kCcThreads = 1024;
__global__ __launch_bounds__(kCcThreads) void k_chunk_count(EmitArgs a) {
    extern __shared__ int s_d[];  // gy rows of gx + 1 cells
    __shared__ uint32_t lds16[kCcThreads / 64];
    const int gx = a.gx, gy = a.gy, nt = a.ntiles, gp = gx + 1, tid = threadIdx.x;
    const uint32_t d = blockIdx.x, P = (uint32_t)a.P;
    constexpr uint32_t SBC = kChunkG / kScanTile;  // scan blocks per chunk
    constexpr int IT = kChunkG / kCcThreads, HI = IT < 8 ? IT : 8;  // rounds of kCcThreads ranks, HI at a time
    static_assert(IT % HI == 0, "whole halves");
    const uint32_t r0 = d * (uint32_t)kChunkG;
    __shared__ uint32_t s_tot[HI][kCcThreads / 64];  // per (round, wave): its instances
    uint32_t cbase;  // the chunk's first slot: the scan's block sums before it
    {
        uint32_t part = 0;
        for (uint32_t i = (uint32_t)tid; i < d * SBC; i += kCcThreads) part += a.scan_sums[i];
        block_excl_scan_n<kCcThreads>(part, lds16, cbase);
    }
    for (int t = tid; t < gy * gp; t += kCcThreads) s_d[t] = 0;
    __syncthreads();
    const int lane = tid & 63, w = tid >> 6;
    uint32_t run = cbase;
    for (int h0 = 0; h0 < IT; h0 += HI) {
        uint2 gr[HI];  // (every load of the part in flight at once)
#pragma unroll
        for (int it = 0; it < HI; ++it) {
            const uint32_t r = r0 + (uint32_t)((h0 + it) * kCcThreads + tid);
            gr[it] = r < P ? a.order[r] : make_uint2(0u, 0u);
        }
        uint32_t c[HI], incl[HI];
#pragma unroll
        for (int it = 0; it < HI; ++it) {
            const uint32_t q = gr[it].x;
            const int x0 = (int)(q & 0xFFu), y0 = (int)((q >> 8) & 0xFFu), x1 = (int)((q >> 16) & 0xFFu),
                      y1 = (int)(q >> 24);
            const bool any = x1 > x0 && y1 > y0;
            if (any) {
                atomicAdd(&s_d[y0 * gp + x0], 1);
                if (x1 < gx) atomicAdd(&s_d[y0 * gp + x1], -1);
                if (y1 < gy) {
                    atomicAdd(&s_d[y1 * gp + x0], -1);
                    if (x1 < gx) atomicAdd(&s_d[y1 * gp + x1], 1);
                }
            }
            c[it] = any ? (uint32_t)((x1 - x0) * (y1 - y0)) : 0u;
            incl[it] = wave_incl_scan_u32(c[it]);
            if (lane == 63) s_tot[it][w] = incl[it];
        }
        __syncthreads();
        // first slots in depth order (rank r0 + round * kCcThreads + tid): the rounds before, the waves before
#pragma unroll
        for (int it = 0; it < HI; ++it) {
            uint32_t wb = 0, rt = 0;
            for (int v = 0; v < kCcThreads / 64; ++v) {
                const uint32_t t = s_tot[it][v];
                wb += v < w ? t : 0u;
                rt += t;
            }
            if (c[it]) a.first_slot[gr[it].y] = run + wb + incl[it] - c[it];
            run += rt;
        }
        __syncthreads();
    }
    if (a.rec_flags32)  // the chunk's slots' four quadrant flags (slot order: coalesced; no memset launch)
        for (uint32_t sl = cbase + (uint32_t)tid; sl < run; sl += kCcThreads)
            if (sl < a.cap) a.rec_flags32[sl] = 0u;
    __syncthreads();
    auto prefix = [&](int first, int n, int stride) {  // inclusive prefix of s_d[first + i * stride], i < n
        int acc = 0;
        for (int i0 = 0; i0 < n; i0 += 16) {
            int c[16];
#pragma unroll
            for (int i = 0; i < 16; ++i) c[i] = i0 + i < n ? s_d[first + (i0 + i) * stride] : 0;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                acc += c[i];
                if (i0 + i < n) s_d[first + (i0 + i) * stride] = acc;
            }
        }
    };
    if (tid < gy) prefix(tid * gp, gx, 1);
    __syncthreads();
    if (tid < gx) prefix(tid, gy, gp);
    __syncthreads();
    uint32_t* __restrict__ row = a.chunk_hist + (size_t)d * nt;  // (block-major: one coalesced row)
    for (int t = tid; t < nt; t += kCcThreads) row[t] = (uint32_t)s_d[(t / gx) * gp + t % gx];
}

constexpr int kReEPT = 16, kReBatch = 256 * kReEPT, kReList = 2048, kReSub = 1024;
static_assert(kReList < 65535 && kReBatch <= 65536, "u16 owners and staged positions");
// BITS: bits of a tile's index inside its region (region_rows x gx <= 1024 tiles)
template <int BITS, bool IDS>
__global__ __launch_bounds__(256) void k_region_emit(EmitArgs a) {
    constexpr int NDIG = 1 << BITS, PER = NDIG >= 256 ? NDIG / 256 : 1;
    __shared__ uint32_t lds4[4];
    __shared__ uint32_t s_magic[256];
    __shared__ uint32_t s_pos[NDIG];      // per region tile: global position of the next instance (see k_emit_tiles)
    __shared__ uint16_t cnt[4][NDIG];     // per-wave tile counters, then the staged runs' starts
    __shared__ uint16_t s_own[kReBatch];  // the batch's owners (+1): marks at the entries' first instances, prefix max
    __shared__ uint16_t s_idx[kReBatch];  // staged, tile-major: the instance's position in the batch
    __shared__ uint32_t s_lrect[kReList], s_lstart[kReList], s_lid[kReList];  // the list: rect, first instance, id
    __shared__ uint32_t s_lsf[IDS ? 1 : kReList];                             // first slot (pairs)
    __shared__ uint32_t s_carry;
    fill_div_magic(s_magic);
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int gx = a.gx, gy = a.gy, nt = a.ntiles, RH = a.region_rows;
    const uint32_t P = (uint32_t)a.P;
    // (chunk, region): consecutive (chunk-major) on one XCD (workgroups go to the XCDs round-robin), so a chunk's
    // depth-order entries, read by each of its regions, stay in that XCD's L2
    const uint32_t nreg = (uint32_t)div_up_u((uint32_t)gy, (uint32_t)RH), N = (uint32_t)a.chunks * nreg;
    const uint32_t per_x = div_up_u(N, 8u);
    const uint32_t logical = (blockIdx.x & 7u) * per_x + (blockIdx.x >> 3);
    if (logical >= N) return;  // (workgroup-uniform, before any barrier)
    const uint32_t d = logical / nreg, reg = logical - d * nreg;
    const uint32_t ry0 = reg * (uint32_t)RH, ry1 = min((uint32_t)gy, ry0 + (uint32_t)RH);
    const uint32_t t0 = ry0 * (uint32_t)gx, RT = (ry1 - ry0) * (uint32_t)gx;
    for (int i = tid; i < NDIG; i += 256)
        s_pos[i] = (uint32_t)i < RT ? a.tile_start[t0 + i] + a.chunk_hist[(size_t)d * nt + t0 + i] : 0u;
    for (int i = tid; i < 4 * NDIG; i += 256) (&cnt[0][0])[i] = 0;
    // region-local tile of instance j (relative to the list's first) owned by list entry o; y, x and the
    // instance's row-major index in its whole rect on the side
    auto place = [&](uint32_t j, uint32_t o, uint32_t& y, uint32_t& x, uint32_t& kr) {
        const uint32_t q = s_lrect[o];
        const uint32_t x0 = q & 0xFFu, y0 = (q >> 8) & 0xFFu, wd = ((q >> 16) & 0xFFu) - x0;
        const uint32_t ya = max(y0, ry0);
        const uint32_t k = j - s_lstart[o];
        const uint32_t ky = div_small(k, wd, s_magic), kx = k - ky * wd;
        y = ya + ky;
        x = x0 + kx;
        kr = (y - y0) * wd + kx;
        return (y - ry0) * (uint32_t)gx + x;
    };
    // expand the list's n_inst instances (n_list entries): batches of kReBatch, ranked, staged, stored
    auto expand = [&](uint32_t n_list, uint32_t n_inst) {
        for (uint32_t j0 = 0; j0 < n_inst; j0 += (uint32_t)kReBatch) {
            const uint32_t nb = n_inst - j0 < (uint32_t)kReBatch ? n_inst - j0 : (uint32_t)kReBatch;
#pragma unroll
            for (int i = 0; i < kReEPT; ++i) s_own[tid * kReEPT + i] = 0;
            __syncthreads();
            for (uint32_t i = (uint32_t)tid; i < n_list; i += 256) {
                const uint32_t st = s_lstart[i];
                if (st >= j0 && st < j0 + nb) s_own[st - j0] = (uint16_t)(i + 1u);  // (list entries: distinct starts)
            }
            const uint32_t carry = j0 ? s_carry : 0u;
            __syncthreads();
            {
                uint32_t run = 0;
#pragma unroll
                for (int i = 0; i < kReEPT; ++i) run = max(run, (uint32_t)s_own[tid * kReEPT + i]);
                run = max(carry, block_exclusive_max(run, lds4));
#pragma unroll
                for (int i = 0; i < kReEPT; ++i) {
                    run = max(run, (uint32_t)s_own[tid * kReEPT + i]);
                    s_own[tid * kReEPT + i] = (uint16_t)run;
                }
            }
            __syncthreads();
            uint32_t dg[kReEPT], loc[kReEPT];
#pragma unroll
            for (int e = 0; e < kReEPT; ++e) {
                const uint32_t jj = (uint32_t)(w * 64 * kReEPT + e * 64 + lane);
                const bool valid = jj < nb;
                const uint64_t vm = __ballot(valid);
                dg[e] = 0u;
                loc[e] = 0u;
                if (vm != 0) {  // (wave-uniform; no break: the loop stays unrolled)
                    uint32_t y, x, kr;
                    const uint32_t t = valid ? place(j0 + jj, (uint32_t)s_own[jj] - 1u, y, x, kr) : 0u;
                    const uint64_t peers = match_digit<BITS>(t, vm);
                    const uint32_t rank = (uint32_t)__popcll(peers & lanemask_lt());
                    const uint32_t old = cnt[w][t];
                    dg[e] = t;
                    loc[e] = old + rank;
                    if (valid && rank == 0) cnt[w][t] = (uint16_t)(old + (uint32_t)__popcll(peers));
                }
            }
            __syncthreads();
            {   // the batch's tile runs (wave-major inside a tile) and their global bases
                uint32_t t4[PER][4];
                uint32_t sum = 0;
#pragma unroll
                for (int i = 0; i < PER; ++i) {
                    const int t = tid * PER + i;
#pragma unroll
                    for (int v = 0; v < 4; ++v) t4[i][v] = t < NDIG ? cnt[v][t] : 0u;
                    sum += t4[i][0] + t4[i][1] + t4[i][2] + t4[i][3];
                }
                uint32_t all;
                uint32_t run = block_exclusive_scan(sum, lds4, all);
#pragma unroll
                for (int i = 0; i < PER; ++i) {
                    const int t = tid * PER + i;
                    if (t < NDIG) {
                        cnt[0][t] = (uint16_t)run;
                        cnt[1][t] = (uint16_t)(run + t4[i][0]);
                        cnt[2][t] = (uint16_t)(run + t4[i][0] + t4[i][1]);
                        cnt[3][t] = (uint16_t)(run + t4[i][0] + t4[i][1] + t4[i][2]);
                        s_pos[t] -= run;
                    }
                    run += t4[i][0] + t4[i][1] + t4[i][2] + t4[i][3];
                }
            }
            __syncthreads();
#pragma unroll
            for (int e = 0; e < kReEPT; ++e) {
                const uint32_t jj = (uint32_t)(w * 64 * kReEPT + e * 64 + lane);
                if (jj < nb) s_idx[cnt[w][dg[e]] + loc[e]] = (uint16_t)jj;
            }
            __syncthreads();
#pragma unroll
            for (int e = 0; e < kReEPT; ++e) {
                const uint32_t i = (uint32_t)(e * 256 + tid);
                if (i < nb) {
                    const uint32_t jj = s_idx[i];
                    const uint32_t o = (uint32_t)s_own[jj] - 1u;
                    uint32_t y, x, kr;
                    const uint32_t t = place(j0 + jj, o, y, x, kr);
                    const uint32_t pos = s_pos[t] + i;
                    if (pos < a.cap) {  // (bounded by the layout: see bin_emit)
                        if constexpr (IDS) reinterpret_cast<uint32_t*>(a.pairs_out)[pos] = s_lid[o];
                        else a.pairs_out[pos] = make_uint2(s_lid[o], min(s_lsf[o] + kr, a.cap - 1u));
                    }
                }
            }
            __syncthreads();
            // the next batch's positions: each tile's run ends where the next tile's begins (the batch's end for
            // the last)
#pragma unroll
            for (int i = 0; i < PER; ++i) {
                const int t = tid * PER + i;
                if (t < NDIG) s_pos[t] += t + 1 < NDIG ? (uint32_t)cnt[0][t + 1] : nb;
            }
            if (tid == 0) s_carry = s_own[nb - 1];
            __syncthreads();
            for (int i = tid; i < 4 * NDIG; i += 256) (&cnt[0][0])[i] = 0;
        }
    };
    const uint32_t r0 = d * (uint32_t)kChunkG;
    uint32_t n_list = 0, n_inst = 0;
    for (uint32_t sb = 0; sb < (uint32_t)kChunkG && r0 + sb < P; sb += (uint32_t)kReSub) {
        // four consecutive depth ranks per thread; an entry of the list if its rect reaches the region's rows
        uint2 gr[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t r = r0 + sb + (uint32_t)(tid * 4 + i);
            gr[i] = r < P ? a.order[r] : make_uint2(0u, 0u);
        }
        uint32_t cr[4], nsel = 0, ninst = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const uint32_t q = gr[i].x;
            const uint32_t x0 = q & 0xFFu, y0 = (q >> 8) & 0xFFu, x1 = (q >> 16) & 0xFFu, y1 = q >> 24;
            const uint32_t ya = max(y0, ry0), yb = min(y1, ry1);
            cr[i] = x1 > x0 && yb > ya ? (yb - ya) * (x1 - x0) : 0u;  // (<= 1024: the region's tiles)
            nsel += cr[i] ? 1u : 0u;
            ninst += cr[i];
        }
        // one scan for both: entries (< 2^11) above instances (<= 1024 x 1024 = 2^20 per 1024 ranks)
        uint32_t tot;
        const uint32_t ex = block_exclusive_scan(nsel << 21 | ninst, lds4, tot);
        uint32_t lp = n_list + (ex >> 21), io = n_inst + (ex & 0x1FFFFFu);
#pragma unroll
        for (int i = 0; i < 4; ++i)
            if (cr[i]) {
                s_lrect[lp] = gr[i].x;
                s_lstart[lp] = io;
                s_lid[lp] = gr[i].y;
                if constexpr (!IDS) s_lsf[lp] = a.first_slot[gr[i].y];
                ++lp;
                io += cr[i];
            }
        n_list += tot >> 21;
        n_inst += tot & 0x1FFFFFu;
        const bool last = sb + (uint32_t)kReSub >= (uint32_t)kChunkG || r0 + sb + (uint32_t)kReSub >= P;
        if (n_list > (uint32_t)(kReList - kReSub) || (last && n_list)) {
            __syncthreads();
            expand(n_list, n_inst);
            __syncthreads();
            n_list = 0;
            n_inst = 0;
        }
    }
}

void launch_region_emit(const EmitArgs& a, hipStream_t s) {
    if (a.P <= 0) return;
    const int nt = a.ntiles, nc = a.chunks;
    hipLaunchKernelGGL(k_chunk_count, dim3(nc), dim3(kCcThreads), (size_t)4 * a.gy * (a.gx + 1), s, a);
    hipLaunchKernelGGL(k_radix_digit_scan, dim3(div_up(nt, kScanDigits)), dim3(kScanThreads), 0, s, a.chunk_hist, nc, nt,
                       a.ttotals, (const uint32_t*)nullptr, 0u, 1);
    hipLaunchKernelGGL(k_ranges_counts, dim3(1), dim3(256), 0, s, a.ttotals, nt, a.ranges, a.tile_order, a.cap,
                       a.tile_start);
    const int nreg = div_up(a.gy, a.region_rows), grid = 8 * div_up((long long)nc * nreg, 8);
    const int bits = ceil_log2((uint32_t)(a.region_rows * a.gx));
#define GS_RE(B)                                                                                   \
    if (a.ids_only) hipLaunchKernelGGL((k_region_emit<B, true>), dim3(grid), dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((k_region_emit<B, false>), dim3(grid), dim3(256), 0, s, a)
    if (bits <= 8) { GS_RE(8); }
    else if (bits <= 9) { GS_RE(9); }
    else { GS_RE(10); }
#undef GS_RE
}

void launch_emit_fused(const EmitArgs& a, hipStream_t s) {
    if (a.P <= 0) return;
    // first level: column totals and each block's column offsets, then the column-ordered emission
    hipLaunchKernelGGL(k_radix_digit_scan, dim3(kXDigits / kScanDigits), dim3(kScanThreads), 0, s, a.xhist, a.scan_blocks,
                       kXDigits, a.xtotals, (const uint32_t*)nullptr, 0u, 1);
    if (a.ids_only)
        hipLaunchKernelGGL(k_scan_emit_x<true>, dim3(a.scan_blocks), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_scan_emit_x<false>, dim3(a.scan_blocks), dim3(256), 0, s, a);
}

#ifndef GS_ROW_IPT
#define GS_ROW_IPT 16  // elements per thread of the row pass (A/B: -DGS_ROW_IPT=32)
#endif
constexpr int kRowIPT = GS_ROW_IPT;
void launch_row_pass(const EmitArgs& a, uint32_t K, uint2* point_pairs, uint32_t* hist, int sort_blocks,
                     uint2* ranges, uint32_t* tile_order, hipStream_t s, const uint32_t* n_dev) {
    if (a.P <= 0 || K == 0) return;
    // second level: the stable row pass (digit y), counting instances per tile on the way
    // (u16 keys: y << 7 | x fits; half the key bytes of the emission's writes and of the pass's reads)
    RangeOut ro{nullptr, nullptr, a.ntiles, a.tile_count, a.gx};
    const uint16_t* keys = reinterpret_cast<const uint16_t*>(a.tile_key);
    constexpr int NDIG = kXDigits, IPT = kRowIPT, TILE = 256 * kRowIPT;
    static_assert(TILE >= kSortTile, "the histogram table is sized for kSortTile-row blocks");
    const int nb = (int)div_up_u(K, (uint32_t)TILE), bm = nb <= kScanBmRows ? 1 : 0;
    (void)sort_blocks;
    hipLaunchKernelGGL((k_radix_hist<kXBits, IPT, uint16_t>), dim3(nb), dim3(256), 0, s, keys, K, kXBits, hist, nb,
                       bm, (const uint32_t*)nullptr, n_dev, CountPublish{});
    if (bm)
        hipLaunchKernelGGL(k_radix_digit_scan, dim3(div_up(NDIG, kScanDigits)), dim3(kScanThreads), 0, s, hist, nb, NDIG,
                           a.xtotals, n_dev, K, TILE);
    else
        hipLaunchKernelGGL(k_radix_digit_scan_dm, dim3(NDIG), dim3(256), 0, s, hist, nb, a.xtotals, n_dev, K, TILE);
    if (a.ids_only)
        hipLaunchKernelGGL((k_radix_scatter<kXBits, IPT, false, kValU32, false, true, uint16_t>), dim3(nb), dim3(256),
                           0, s, keys, a.pairs_out, nullptr, point_pairs, nullptr, K, kXBits, hist, a.xtotals, nb, bm, ro,
                           (const uint32_t*)nullptr, n_dev);
    else
        hipLaunchKernelGGL((k_radix_scatter<kXBits, IPT, false, kValPair, false, true, uint16_t>), dim3(nb), dim3(256),
                           0, s, keys, a.pairs_out, nullptr, point_pairs, nullptr, K, kXBits, hist, a.xtotals, nb, bm, ro,
                           (const uint32_t*)nullptr, n_dev);
    hipLaunchKernelGGL(k_ranges_counts, dim3(1), dim3(256), 0, s, a.tile_count, a.ntiles, ranges, tile_order,
                       0xFFFFFFFFu, (uint32_t*)nullptr);
}

void launch_scan_reduce(const EmitArgs& a, hipStream_t s) {
    if (a.P <= 0) return;
    hipLaunchKernelGGL(k_scan_reduce, dim3(a.scan_blocks), dim3(256), 0, s, a);
    if (a.thist) {  // direct emission: each block's first position per tile, the tile totals
        if (a.scan_blocks <= kScanBmRows)
            hipLaunchKernelGGL(k_radix_digit_scan, dim3(div_up(a.ntiles, kScanDigits)), dim3(kScanThreads), 0, s, a.thist,
                               a.scan_blocks, a.ntiles, a.ttotals, (const uint32_t*)nullptr, 0u, 1);
        else
            hipLaunchKernelGGL(k_radix_digit_scan_dm, dim3(a.ntiles), dim3(256), 0, s, a.thist, a.scan_blocks, a.ttotals,
                               (const uint32_t*)nullptr, 0u, 1);
    }
}

void launch_emit_tiles(const EmitArgs& a, hipStream_t s) {
    if (a.P <= 0) return;
    const int bits = ceil_log2((uint32_t)(a.ntiles > 1 ? a.ntiles : 2));
#define GS_ET(B)                                                                                       \
    if (a.ids_only) hipLaunchKernelGGL((k_emit_tiles<B, true>), dim3(a.scan_blocks), dim3(256), 0, s, a); \
    else hipLaunchKernelGGL((k_emit_tiles<B, false>), dim3(a.scan_blocks), dim3(256), 0, s, a)
    if (bits <= 8) { GS_ET(8); }
    else if (bits <= 10) { GS_ET(10); }
    else { GS_ET(11); }
#undef GS_ET
}

void launch_scan_emit(const EmitArgs& a, hipStream_t s) {
    if (a.P <= 0) return;
    hipLaunchKernelGGL(k_scan_emit, dim3(a.scan_blocks), dim3(256), 0, s, a);
}

// ---------------------------------------------------------------------
// identifyTileRanges (rasterizer_impl.cu:105-125) + instance maps
// ---------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ranges(const uint32_t* __restrict__ tile, int K, uint2* __restrict__ ranges,
                                                uint32_t* __restrict__ rec_flags32) {
    const int pos = blockIdx.x * 256 + threadIdx.x;
    if (pos >= K) return;
    if (rec_flags32) rec_flags32[pos] = 0u;  // (slot `pos`: the four quadrant flags; no memset launch)
    const uint32_t t = tile[pos];
    if (pos == 0) {
        ranges[t].x = 0;
    } else {
        const uint32_t prev = tile[pos - 1];
        if (prev != t) {
            ranges[prev].y = (uint32_t)pos;
            ranges[t].x = (uint32_t)pos;
        }
    }
    if (pos == K - 1) ranges[t].y = (uint32_t)K;
}

void launch_ranges(const uint32_t* sorted_tile, int K, uint2* ranges, uint32_t* rec_flags32, hipStream_t s) {
    if (K <= 0) return;
    hipLaunchKernelGGL(k_ranges, dim3(div_up(K, 256)), dim3(256), 0, s, sorted_tile, K, ranges, rec_flags32);
}

// The speculated views' overflow decision on the device (the same test as gs_views_check's on the
// host copy of the counters): one wave, lane v < n reads view v's counter slots.
__global__ __launch_bounds__(64) void k_views_overflow(OverflowArgs a, uint8_t* __restrict__ flag) {
    const int v = threadIdx.x;
    // a speculated view's (cap != 0; exact views and views of no Gaussians have no counters) slot counts,
    // loaded together under the lane's condition and summed after it: the summing loop inside the condition
    // waited for each load in turn
    const bool act = v < a.n && a.cap[v] != 0u && a.counters[v] != nullptr;
    uint32_t cs[kCounterSlots];
#pragma unroll
    for (int i = 0; i < kCounterSlots; ++i) cs[i] = 0u;
    if (act) {
        const uint32_t* __restrict__ c = a.counters[v];
#pragma unroll
        for (int i = 0; i < kCounterSlots; ++i) cs[i] = c[i * kCounterStride];
    }
    __builtin_amdgcn_sched_barrier(0);
    uint64_t k = 0;
#pragma unroll
    for (int i = 0; i < kCounterSlots; ++i) k += cs[i];
    const bool bad = act && k > a.cap[v];  // (any depth-key range sorts: depth_sort_msd)
    const uint64_t any = __ballot(bad);
    if (v == 0) flag[0] = any ? 1 : 0;
}

void launch_views_overflow(const OverflowArgs& a, uint8_t* flag, hipStream_t s) {
    hipLaunchKernelGGL(k_views_overflow, dim3(1), dim3(64), 0, s, a, flag);
}

}  // namespace gs
