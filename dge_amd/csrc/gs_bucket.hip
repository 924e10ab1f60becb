// gs_bucket.hip — the sparse-row gradient exchange of the multi-view step, for gfx950.
//
// DGE sums the parameter gradients of a batch of views before the optimizer
// step (threestudio/systems/DGE.py:170-296).  Sharded over ranks, that sum is an
// all-reduce of the GaussianModel's six .grad tensors (59 floats per Gaussian,
// 236 MB at 1M).  A Gaussian no view of a rank blends has exactly zero gradient
// there, so dge_amd/multiview.py GradBucket moves only the rows that are
// nonzero on some rank.  These kernels are its bookkeeping, each one pass at the
// HBM roofline instead of torch's per-tensor compare / any / index_select / cat /
// index_copy chain (~680 us at c3 on one MI355X, tools/probes/bucket_cost.py):
//   k_rows_live    live[r] = row r of some region has an element != 0   (reads 4·pitch·n B)
//   k_rows_gather  packed[i, :] = row rows[i] of every region           (4·W·m B each way)
//   k_rows_scatter row rows[i] of every region = packed[i, :]
#include "gs_internal.h"
#include "gs_raster.h"

namespace gs {

struct RowsLaunch {
    int nreg, width;                               // regions, total floats per row
    float* base[GS_ROWS_MAX_REGIONS];
    int w[GS_ROWS_MAX_REGIONS];                    // used columns of each region
    int p[GS_ROWS_MAX_REGIONS];                    // its row stride (>= w)
    int col0[GS_ROWS_MAX_REGIONS + 1];             // first packed column of each region
};

constexpr int kRowsBlock = 256;  // rows per workgroup of k_rows_live

// One workgroup per 256 rows: each region's rows [r0, r0 + nr) are one contiguous span of pitch-wide
// rows, read coalesced (float4 when the span is 16-B aligned, four in flight per thread); a nonzero
// element of the first w columns marks its row in LDS (benign same-value stores).
__device__ __forceinline__ int row_of(int j, int w, float inv_w) {
    int r = (int)((float)j * inv_w);  // exact after the correction: j < 2^24
    r -= (r * w > j);
    r += ((r + 1) * w <= j);
    return r;
}

// element j of the span: mark its row when it is nonzero (NaN counts, as torch's `!= 0`) and a used column
__device__ __forceinline__ void mark_elem(uint32_t* flag, float v, int j, int p, float inv_p, int w) {
    if (v != 0.f) {
        const int r = row_of(j, p, inv_p);
        if (p == w || j - r * p < w) flag[r] = 1u;
    }
}

__global__ __launch_bounds__(kRowsBlock) void k_rows_live(RowsLaunch a, long long n, uint8_t* __restrict__ live) {
    __shared__ uint32_t flag[kRowsBlock];
    const long long r0 = (long long)blockIdx.x * kRowsBlock;
    const int nr = n - r0 < kRowsBlock ? (int)(n - r0) : kRowsBlock;
    flag[threadIdx.x] = 0u;
    __syncthreads();
    for (int k = 0; k < a.nreg; ++k) {
        const int w = a.w[k], p = a.p[k];
        const float* __restrict__ src = a.base[k] + r0 * p;
        const int span = (nr - 1) * p + w;  // (the last row's padding may lie past the allocation)
        const float inv_p = 1.f / (float)p;
        int e = 0;  // elements below e are done
        if ((reinterpret_cast<uintptr_t>(src) & 15) == 0) {
            const float4* __restrict__ s4 = reinterpret_cast<const float4*>(src);
            const int n4 = span >> 2;
            int q = threadIdx.x;
            for (; q + 3 * kRowsBlock < n4; q += 4 * kRowsBlock) {
                float4 v[4];
#pragma unroll
                for (int u = 0; u < 4; ++u) v[u] = s4[q + u * kRowsBlock];
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const int j = 4 * (q + u * kRowsBlock);
                    mark_elem(flag, v[u].x, j, p, inv_p, w);
                    mark_elem(flag, v[u].y, j + 1, p, inv_p, w);
                    mark_elem(flag, v[u].z, j + 2, p, inv_p, w);
                    mark_elem(flag, v[u].w, j + 3, p, inv_p, w);
                }
            }
            for (; q < n4; q += kRowsBlock) {
                const float4 v = s4[q];
                const int j = 4 * q;
                mark_elem(flag, v.x, j, p, inv_p, w);
                mark_elem(flag, v.y, j + 1, p, inv_p, w);
                mark_elem(flag, v.z, j + 2, p, inv_p, w);
                mark_elem(flag, v.w, j + 3, p, inv_p, w);
            }
            e = n4 << 2;
        }
        for (int j = e + threadIdx.x; j < span; j += kRowsBlock) mark_elem(flag, src[j], j, p, inv_p, w);
    }
    __syncthreads();
    if ((int)threadIdx.x < nr) live[r0 + threadIdx.x] = (uint8_t)flag[threadIdx.x];
}

// A 64-lane wave moves kRowsPerWave packed rows, lane = column (rows wider than 64 loop): all of a
// wave's loads are issued before its stores; no index division.
constexpr int kRowsPerWave = 8;

// m_dev (the _dev entry points): the packed buffer has m rows (the capacity), the row list only
// min(m, *m_dev) — a gather zero-fills the packed rows past it, a scatter leaves them
template <bool GATHER>
__global__ __launch_bounds__(256) void k_rows_move(RowsLaunch a, const long long* __restrict__ rows, long long m,
                                                   float* __restrict__ packed, const long long* __restrict__ m_dev) {
    const long long i0 = ((long long)blockIdx.x * 4 + (threadIdx.x >> 6)) * kRowsPerWave;
    if (i0 >= m) return;
    const long long mv = m_dev ? (*m_dev < m ? *m_dev : m) : m;  // rows with a list entry
    if (!GATHER && i0 >= mv) return;
    const int ncap = m - i0 < kRowsPerWave ? (int)(m - i0) : kRowsPerWave;  // packed rows of this wave
    const int nrow = mv - i0 <= 0 ? 0 : mv - i0 < kRowsPerWave ? (int)(mv - i0) : kRowsPerWave;
    long long row[kRowsPerWave];
#pragma unroll
    for (int u = 0; u < kRowsPerWave; ++u) row[u] = nrow ? rows[i0 + (u < nrow ? u : 0)] : 0;
    for (int c = threadIdx.x & 63; c < a.width; c += 64) {
        int k = 0;
#pragma unroll
        for (int q = 1; q < GS_ROWS_MAX_REGIONS; ++q) k += (c >= a.col0[q]);
        float* __restrict__ col = a.base[k] + (c - a.col0[k]);
        const int w = a.p[k];  // (row stride)
        float* __restrict__ out = packed + i0 * a.width + c;
        float v[kRowsPerWave];
        if (GATHER) {
#pragma unroll
            for (int u = 0; u < kRowsPerWave; ++u) v[u] = col[row[u] * w];  // (row[u] is a valid row)
#pragma unroll
            for (int u = 0; u < kRowsPerWave; ++u)
                if (u < ncap) out[(long long)u * a.width] = u < nrow ? v[u] : 0.f;
        } else {
#pragma unroll
            for (int u = 0; u < kRowsPerWave; ++u) v[u] = out[(long long)(u < nrow ? u : 0) * a.width];
#pragma unroll
            for (int u = 0; u < kRowsPerWave; ++u)
                if (u < nrow) col[row[u] * w] = v[u];
        }
    }
}

// rows = ascending indices r with live[r] != 0, count = their number, without a host round trip
// (torch.nonzero reads the count back): per-block counts, then each block adds up the counts before
// it and writes its rows in order.  At most kCompactMaxBlocks blocks (each takes `chunks` runs of 1024
// rows), so that prefix stays at most ~1k words from L2 per block whatever n is.
constexpr int kCompactRows = 1024;        // rows per chunk (4 per thread)
constexpr int kCompactMaxBlocks = 1024;

__global__ __launch_bounds__(256) void k_compact_count(const uint8_t* __restrict__ live, long long n, int chunks,
                                                       long long* __restrict__ sums) {
    __shared__ uint32_t part[4];
    uint32_t c = 0;
    for (int k = 0; k < chunks; ++k) {
        const long long r0 = ((long long)blockIdx.x * chunks + k) * kCompactRows + 4 * threadIdx.x;
#pragma unroll
        for (int u = 0; u < 4; ++u) c += (r0 + u < n && live[r0 + u]) ? 1u : 0u;
    }
    c = __reduce_add_sync(~0ull, c);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) sums[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

__global__ __launch_bounds__(256) void k_compact_write(const uint8_t* __restrict__ live, long long n, int chunks,
                                                       const long long* __restrict__ sums, long long* __restrict__ rows,
                                                       long long* __restrict__ count) {
    __shared__ long long s_part[4];
    __shared__ uint32_t s_wave[2][4];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    long long before = 0;  // rows of the blocks before this one
    for (int b = tid; b < (int)blockIdx.x; b += 256) before += sums[b];
    for (int o = 32; o >= 1; o >>= 1) before += __shfl_xor(before, o);
    if (lane == 0) s_part[w] = before;
    __syncthreads();
    long long base = s_part[0] + s_part[1] + s_part[2] + s_part[3];
    for (int k = 0; k < chunks; ++k) {
        const long long r0 = ((long long)blockIdx.x * chunks + k) * kCompactRows + 4 * tid;
        bool l[4];
        uint32_t c = 0;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            l[u] = r0 + u < n && live[r0 + u];
            c += l[u] ? 1u : 0u;
        }
        // exclusive prefix of c over the chunk (thread order = row order)
        uint32_t x = c;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = (uint32_t)__shfl_up((int)x, o);
            if (lane >= o) x += y;
        }
        uint32_t* sw = s_wave[k & 1];  // (double-buffered: one barrier per chunk)
        if (lane == 63) sw[w] = x;
        __syncthreads();
        uint32_t off = x - c;
        for (int q = 0; q < w; ++q) off += sw[q];
        long long at = base + off;
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (l[u]) rows[at++] = r0 + u;
        base += sw[0] + sw[1] + sw[2] + sw[3];
    }
    if (blockIdx.x == gridDim.x - 1 && tid == 0) *count = base;
}

// One thread per row reads its flag (coalesced) and clears it; each wave then zeroes its dirty rows one after
// another, all 64 lanes on one row (one 256-B store per 64 floats) — a grid of n / 256 workgroups, not one
// thread per float: the clean rows cost a byte read.
__global__ __launch_bounds__(256) void k_rows_zero_dirty(float* __restrict__ rows, long long pitch, int width,
                                                         uint8_t* __restrict__ dirty, long long n) {
    const long long r = (long long)blockIdx.x * 256 + threadIdx.x;
    const int lane = threadIdx.x & 63;
    const bool d = r < n && dirty[r];
    if (d) dirty[r] = 0;
    uint64_t m = __ballot(d);
    const long long wbase = r - lane;  // the wave's first row
    while (m) {  // (wave-uniform)
        const int k = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        float* row = rows + (wbase + k) * pitch;
        for (int c = lane; c < width; c += 64) row[c] = 0.f;
    }
}

__global__ __launch_bounds__(256) void k_rows_mark_dirty(uint8_t* __restrict__ dirty, const long long* __restrict__ rows,
                                                         long long m, const long long* __restrict__ m_dev) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    const long long mv = m_dev ? (*m_dev < m ? *m_dev : m) : m;
    if (i < mv) dirty[rows[i]] = 1;
}

static int rows_launch(const gs_rows_region* regions, int nreg, RowsLaunch& a, const char* fn) {
    if (nreg < 1 || nreg > GS_ROWS_MAX_REGIONS || !regions)
        return report_error(GS_ERR_INVALID_ARG, fn);
    a.nreg = nreg;
    a.col0[0] = 0;
    for (int k = 0; k < nreg; ++k) {
        if (!regions[k].base || regions[k].width < 1 || (regions[k].pitch && regions[k].pitch < regions[k].width))
            return report_error(GS_ERR_INVALID_ARG, fn);
        a.base[k] = regions[k].base;
        a.w[k] = regions[k].width;
        a.p[k] = regions[k].pitch ? regions[k].pitch : regions[k].width;
        a.col0[k + 1] = a.col0[k] + regions[k].width;
    }
    for (int k = nreg; k < GS_ROWS_MAX_REGIONS; ++k) {
        a.base[k] = nullptr;
        a.w[k] = 1;
        a.p[k] = 1;
        a.col0[k + 1] = a.col0[k];
    }
    a.width = a.col0[nreg];
    return GS_OK;
}

static int launched() {
    const hipError_t e = hipGetLastError();
    return e == hipSuccess ? GS_OK : report_error(GS_ERR_HIP, hipGetErrorString(e));
}

}  // namespace gs

extern "C" int gs_rows_live(const gs_rows_region* regions, int nreg, long long n, uint8_t* live, gs_stream_t stream) {
    using namespace gs;
    RowsLaunch a;
    if (int rc = rows_launch(regions, nreg, a, "gs_rows_live: bad region list")) return rc;
    if (n < 0 || (n > 0 && !live)) return report_error(GS_ERR_INVALID_ARG, "gs_rows_live: bad row count / mask");
    for (int k = 0; k < nreg; ++k)
        if ((long long)kRowsBlock * a.p[k] >= (1ll << 24))
            return report_error(GS_ERR_INVALID_ARG, "gs_rows_live: region too wide");
    if (n == 0) return GS_OK;
    hipLaunchKernelGGL(k_rows_live, dim3((unsigned)((n + kRowsBlock - 1) / kRowsBlock)), dim3(kRowsBlock), 0,
                       (hipStream_t)stream, a, n, live);
    return launched();
}

static int rows_move(const gs_rows_region* regions, int nreg, const long long* rows, long long m, float* packed,
                     gs_stream_t stream, bool gather, const char* fn, const long long* m_dev = nullptr) {
    using namespace gs;
    RowsLaunch a;
    if (int rc = rows_launch(regions, nreg, a, fn)) return rc;
    if (m < 0 || (m > 0 && (!rows || !packed))) return report_error(GS_ERR_INVALID_ARG, fn);
    if (m == 0) return GS_OK;
    const long long blocks = (m + 4 * kRowsPerWave - 1) / (4 * kRowsPerWave);
    if (blocks > 0x7FFFFFFF) return report_error(GS_ERR_INVALID_ARG, fn);
    if (gather)
        hipLaunchKernelGGL(k_rows_move<true>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a, rows, m,
                           packed, m_dev);
    else
        hipLaunchKernelGGL(k_rows_move<false>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a, rows, m,
                           packed, m_dev);
    return launched();
}

extern "C" int gs_rows_gather(const gs_rows_region* regions, int nreg, const long long* rows, long long m,
                              float* packed, gs_stream_t stream) {
    return rows_move(regions, nreg, rows, m, packed, stream, true, "gs_rows_gather: bad arguments");
}

extern "C" int gs_rows_scatter(const gs_rows_region* regions, int nreg, const long long* rows, long long m,
                               const float* packed, gs_stream_t stream) {
    return rows_move(regions, nreg, rows, m, const_cast<float*>(packed), stream, false,
                     "gs_rows_scatter: bad arguments");
}

extern "C" int gs_rows_gather_dev(const gs_rows_region* regions, int nreg, const long long* rows, long long cap,
                                  const long long* count, float* packed, gs_stream_t stream) {
    if (!count) return gs::report_error(GS_ERR_INVALID_ARG, "gs_rows_gather_dev: count is required");
    return rows_move(regions, nreg, rows, cap, packed, stream, true, "gs_rows_gather_dev: bad arguments", count);
}

extern "C" int gs_rows_scatter_dev(const gs_rows_region* regions, int nreg, const long long* rows, long long cap,
                                   const long long* count, const float* packed, gs_stream_t stream) {
    if (!count) return gs::report_error(GS_ERR_INVALID_ARG, "gs_rows_scatter_dev: count is required");
    return rows_move(regions, nreg, rows, cap, const_cast<float*>(packed), stream, false,
                     "gs_rows_scatter_dev: bad arguments", count);
}

extern "C" int gs_rows_compact(const uint8_t* live, long long n, long long* rows, long long* count_scratch,
                               gs_stream_t stream) {
    using namespace gs;
    if (n < 0 || (n > 0 && (!live || !rows)) || !count_scratch)
        return report_error(GS_ERR_INVALID_ARG, "gs_rows_compact: bad arguments");
    if (n == 0) return hipMemsetAsync(count_scratch, 0, sizeof(long long), (hipStream_t)stream) == hipSuccess
                           ? GS_OK : report_error(GS_ERR_HIP, "gs_rows_compact: memset failed");
    const long long runs = (n + kCompactRows - 1) / kCompactRows;  // (<= the scratch's ceil(n / 1024))
    if (runs > 0x7FFFFFFF) return report_error(GS_ERR_INVALID_ARG, "gs_rows_compact: n too large");
    const long long per = (runs + kCompactMaxBlocks - 1) / kCompactMaxBlocks;  // chunks per block
    const long long blocks = (runs + per - 1) / per;
    hipLaunchKernelGGL(k_compact_count, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, live, n, (int)per,
                       count_scratch + 1);
    hipLaunchKernelGGL(k_compact_write, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, live, n, (int)per,
                       count_scratch + 1, rows, count_scratch);
    return launched();
}

extern "C" int gs_rows_zero_dirty(float* rows, long long pitch, int width, uint8_t* dirty, long long n,
                                  gs_stream_t stream) {
    using namespace gs;
    if (n < 0 || (n > 0 && (!rows || !dirty)) || width < 0 || width > pitch || (pitch & 3) || (width & 3) ||
        (reinterpret_cast<uintptr_t>(rows) & 15))
        return report_error(GS_ERR_INVALID_ARG, "gs_rows_zero_dirty: bad arguments (16-B rows, 4-float pitch/width)");
    if (n == 0 || width == 0) return GS_OK;
    const long long blocks = (n + 255) / 256;
    if (blocks > 0x7FFFFFFF) return report_error(GS_ERR_INVALID_ARG, "gs_rows_zero_dirty: n too large");
    hipLaunchKernelGGL(k_rows_zero_dirty, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, rows, pitch, width,
                       dirty, n);
    return launched();
}

extern "C" int gs_rows_mark_dirty(uint8_t* dirty, const long long* rows, long long m, const long long* count,
                                  gs_stream_t stream) {
    using namespace gs;
    if (m < 0 || (m > 0 && (!dirty || !rows))) return report_error(GS_ERR_INVALID_ARG, "gs_rows_mark_dirty: bad arguments");
    if (m == 0) return GS_OK;
    const long long blocks = (m + 255) / 256;
    if (blocks > 0x7FFFFFFF) return report_error(GS_ERR_INVALID_ARG, "gs_rows_mark_dirty: m too large");
    hipLaunchKernelGGL(k_rows_mark_dirty, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, dirty, rows, m,
                       count);
    return launched();
}
