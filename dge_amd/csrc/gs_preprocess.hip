// gs_preprocess.hip — per-Gaussian forward preprocessing for gfx950.
//
// Restates preprocessCUDA (forward.cu:155-256) with computeCov3D (:118-152),
// computeCov2D (:74-113), computeColorFromSH (:20-71) and in_frustum
// (auxiliary.h:139-164), and fuses three steps the reference runs separately:
//   * the depth sort key (bits of the view-space depth, or 0xFFFFFFFF when the
//     Gaussian is culled) that replaces the reference's (tile|depth) 64-bit key;
//   * the instance total num_rendered (one atomic per workgroup), so the host
//     read-back overlaps the depth sort instead of draining the stream;
//   * colour and depth packed into one float4 (rgbd) for the blend loop.
// One thread per Gaussian; 256-thread workgroups (4 waves).
// Exact IEEE single-precision operations in the order written (no FMA
// contraction): the per-Gaussian geometry, depth keys, radii and tile rects
// then match the CPU restatement bit for bit, so the discrete outputs
// (num_rendered, radii, sorted tile lists) are identical, not just close.
// These kernels are HBM-bound; the extra multiplies cost nothing measurable.
#pragma clang fp contract(off)
#include "gs_common.h"
#include "gs_internal.h"

namespace gs {

// forward.cu:20-71, in two parts so the coefficient rows can be staged in two
// halves: sh_rgb_head = bands 0-2 (c0 = coefficient 0, rA = coefficients 1..8),
// sh_rgb_tail = band 3 (rB = coefficients 9..15) + the offset and clamp.  The
// sum is accumulated in the reference's order either way.
__device__ __forceinline__ f3 sh_dir(f3 pos, f3 campos) {
    f3 dir = pos - campos;
    const float len = sqrtf(dot3(dir, dir));
    return mk3(dir.x / len, dir.y / len, dir.z / len);
}

__device__ __forceinline__ f3 sh_rgb_head(int deg, f3 dir, f3 c0, const float* __restrict__ r) {
    f3 res = c0 * kSH_C0;
    if (deg > 0) {
        const float x = dir.x, y = dir.y, z = dir.z;
        res = res - ld3(r) * (kSH_C1 * y) + ld3(r + 3) * (kSH_C1 * z) - ld3(r + 6) * (kSH_C1 * x);
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            res = res + ld3(r + 9) * (kSH_C2_0 * xy) + ld3(r + 12) * (kSH_C2_1 * yz) +
                  ld3(r + 15) * (kSH_C2_2 * (2.0f * zz - xx - yy)) + ld3(r + 18) * (kSH_C2_3 * xz) +
                  ld3(r + 21) * (kSH_C2_4 * (xx - yy));
        }
    }
    return res;
}

__device__ __forceinline__ f3 sh_rgb_tail(int deg, f3 dir, f3 res, const float* __restrict__ r, uint8_t& clamp_bits) {
    if (deg > 2) {
        const float x = dir.x, y = dir.y, z = dir.z;
        const float xx = x * x, yy = y * y, zz = z * z, xy = x * y;
        res = res + ld3(r) * (kSH_C3_0 * y * (3.0f * xx - yy)) + ld3(r + 3) * (kSH_C3_1 * xy * z) +
              ld3(r + 6) * (kSH_C3_2 * y * (4.0f * zz - xx - yy)) +
              ld3(r + 9) * (kSH_C3_3 * z * (2.0f * zz - 3.0f * xx - 3.0f * yy)) +
              ld3(r + 12) * (kSH_C3_4 * x * (4.0f * zz - xx - yy)) + ld3(r + 15) * (kSH_C3_5 * z * (xx - yy)) +
              ld3(r + 18) * (kSH_C3_6 * x * (xx - 3.0f * yy));
    }
    res = mk3(res.x + 0.5f, res.y + 0.5f, res.z + 0.5f);
    clamp_bits = (res.x < 0 ? 1 : 0) | (res.y < 0 ? 2 : 0) | (res.z < 0 ? 4 : 0);
    return mk3(fmaxf(res.x, 0.0f), fmaxf(res.y, 0.0f), fmaxf(res.z, 0.0f));
}

// fp16 SH rows (kSplit): coefficient rows 1..15 of the block's Gaussians are
// staged through LDS in two halves (coefficients 1..8 = 24 values, then 9..15
// = 21) in one 25-float-pitch buffer: 25.6 KB instead of 46 KB per block, 6
// waves per SIMD instead of 3 (c5: 48 -> 34 us).  Both halves are loaded at
// kernel start — the second into registers, written to LDS once the first
// half is consumed.  Element f of a half: row f / n, column f % n.  fp32 rows
// keep the one-pass float4 staging (measured faster there: 93 vs 95 us at c2).
constexpr int kShA = 24, kShB = 21, kShPitchAB = 25;
constexpr int kShBPer = (256 * kShB + 255) / 256;  // = 21 register values per thread



template <bool kSplit>
__global__ __launch_bounds__(256) void k_preprocess(PreprocessArgs a) {
    constexpr int kPitch = kSplit ? kShPitchAB : kShPitch;
    __shared__ float s_sh[256 * kPitch];
    const int idx0 = blockIdx.x * 256;
    const int idx = idx0 + threadIdx.x;
    uint32_t touched = 0;
    uint32_t rect = 0;  // packed tile rect (or the count), 0 for a culled Gaussian
    int radius_out = 0;
    uint32_t key = 0xFFFFFFFFu;
    uint8_t clamp_bits = 0;
    f3 p = mk3(0, 0, 0), rgb = mk3(0, 0, 0);
    float2 pix = make_float2(0.f, 0.f);
    float4 conic = make_float4(0.f, 0.f, 0.f, 0.f);
    float depth = 0.f;
    uint32_t auxv = 0;  // gs_params.aux_mask byte, compared at the Splat store (a compare beside the load,
                        // in a branch of its own, waited for every load in flight)
    // SH rows of the whole block staged first, in flight together with the per-Gaussian loads below
    // (one memory phase instead of geometry -> compute -> SH rows); rows of Gaussians that turn out
    // culled are read needlessly (180 B each), which object-centric views hardly have
    const int ncol = (a.M - 1) * 3 < kShPitch ? (a.M - 1) * 3 : kShPitch;
    const bool stage_sh = a.copy_colors && !a.colors_precomp && a.sh.dc && ncol > 0;
    const int nrow = a.P - idx0 < 256 ? a.P - idx0 : 256;
    const int ncolA = ncol < kShA ? ncol : kShA, ncolB = ncol - ncolA;
    float shB[kShBPer];
    // parameter rows of the block's Gaussians (gs_params.index: the localize subset, gathered here)
    __shared__ int s_src[256];
    if (a.index) {
        s_src[threadIdx.x] = (int)threadIdx.x < nrow ? a.index[idx0 + threadIdx.x] : 0;
        __syncthreads();
    }
    const int src = a.index ? s_src[threadIdx.x] : idx;
    if (stage_sh && !kSplit) {
        sh_rows_load<256>(a.sh.rest + (size_t)idx0 * a.sh.rest_stride, a.sh.rest_stride, s_sh, nrow, ncol);
    } else if (stage_sh) {
        // both halves' loads issued together (32-bit offsets from the block's uniform base): the first
        // half is stored to LDS as it arrives, the second stays in registers
        const int stride = a.sh.rest_stride;
        const float invA = 1.0f / (float)ncolA, invB = ncolB > 0 ? 1.0f / (float)ncolB : 0.f;
        const int rbase = a.index ? 0 : idx0;  // rows: s_src[row] (gathered) or idx0 + row
        const float* baseF = a.sh.rest + (size_t)rbase * stride;
        const uint16_t* baseH = reinterpret_cast<const uint16_t*>(a.sh.rest) + (size_t)rbase * stride;
        // raw bits first, converted once every load is issued (a conversion next to its load made each
        // fp16 load wait in turn: c5's 45 rows of round trips)
        const bool half = a.sh.half != 0;
        auto ld = [&](uint32_t off) { return half ? (uint32_t)baseH[off] : __float_as_uint(baseF[off]); };
        auto cvt = [&](uint32_t r) {
            return half ? __half2float(__ushort_as_half((unsigned short)r)) : __uint_as_float(r);
        };
        auto srow = [&](int row) { return a.index ? s_src[row] : row; };
        uint32_t rawA[kShA], rawB[kShBPer];
#pragma unroll
        for (int i = 0; i < kShA; ++i) {
            const int f = threadIdx.x + 256 * i;
            const int row = (int)(((float)f + 0.5f) * invA), col = f - row * ncolA;
            rawA[i] = row < nrow ? ld((uint32_t)(srow(row) * stride + col)) : 0u;
        }
#pragma unroll
        for (int i = 0; i < kShBPer; ++i) {
            const int f = threadIdx.x + 256 * i;
            const int row = (int)(((float)f + 0.5f) * invB), col = f - row * ncolB;
            rawB[i] = ncolB > 0 && row < nrow ? ld((uint32_t)(srow(row) * stride + kShA + col)) : 0u;
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < kShBPer; ++i) shB[i] = cvt(rawB[i]);
#pragma unroll
        for (int i = 0; i < kShA; ++i) {
            const int f = threadIdx.x + 256 * i;
            const int row = (int)(((float)f + 0.5f) * invA), col = f - row * ncolA;
            if (row < nrow) s_sh[row * kShPitchAB + col] = cvt(rawA[i]);
        }
    }
    if (idx < a.P) {
        const float* v = a.view;
        const float* pm = a.proj;
        // every per-Gaussian input is loaded up front, culled or not (one memory round trip
        // instead of xyz -> frustum test -> scale/rotation -> opacity)
        p = ld3(a.means3D + 3 * (size_t)src);
        float cov3[6];
        float4 q = make_float4(0.f, 0.f, 0.f, 0.f);
        f3 sc = mk3(0.f, 0.f, 0.f);
        if (a.cov3D_precomp) {
#pragma unroll
            for (int k = 0; k < 6; ++k) cov3[k] = a.cov3D_precomp[6 * (size_t)src + k];
        } else {
            q = *reinterpret_cast<const float4*>(a.rotations + 4 * (size_t)src);
            sc = ld3(a.scales + 3 * (size_t)src);
        }
        const float op_in = a.opacities[src];
        // (no branch: without a mask the load reads the opacities' bytes, a valid address, and is ignored)
        auxv = (a.aux_mask ? a.aux_mask : reinterpret_cast<const uint8_t*>(a.opacities))[src];
        // in_frustum (auxiliary.h:139-164): only the near test is live
        const float4 ph = proj_point(pm, p);
        const float pw = 1.0f / (ph.w + 0.0000001f);
        const f3 pv = view_point(v, p);
        bool visible = pv.z > 0.2f;
        if (!visible && a.prefiltered) atomicOr(&a.counters[3], 1u);  // (slot 0, word 3)
        if (visible) {
            if (!a.cov3D_precomp) {
                if (a.activation) {  // get_rotation / get_scaling (gaussian_model.py:228-240)
                    float len;
                    q = act_normalize(q, len);
                    sc = mk3(expf(sc.x), expf(sc.y), expf(sc.z));
                }
                cov3d_from_scale_rot(sc, a.scale_modifier, q, cov3);
            }
            Ewa e;
            ewa_setup(p, a.fx, a.fy, a.tanfovx, a.tanfovy, cov3, v, e);
            float ca, cb, cc;
            ewa_cov2d(e, ca, cb, cc);
            const float det = ca * cc - cb * cb;
            if (det != 0.0f) {
                const float det_inv = 1.f / det;
                const float op = a.activation ? act_sigmoid(op_in) : op_in;
                conic = make_float4(cc * det_inv, -cb * det_inv, ca * det_inv, op);
                const float mid = 0.5f * (ca + cc);
                const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
                const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
                const float rad = ceilf(3.f * sqrtf(fmaxf(l1, l2)));
                pix = make_float2(ndc_to_pixel(ph.x * pw, a.W), ndc_to_pixel(ph.y * pw, a.H));
                const Rect r = tile_rect(pix.x, pix.y, (int)rad, a.gx, a.gy);
                const uint32_t area = (uint32_t)((r.y1 - r.y0) * (r.x1 - r.x0));
                if (area != 0) {
                    rect = a.rect_packed ? pack_rect(r.x0, r.y0, r.x1, r.y1) : area;
                    radius_out = (int)rad;
                    touched = area;
                    depth = pv.z;
                    key = __float_as_uint(pv.z);  // depth > 0.2: the bits sort as the value
                }
            }
        }
    }
    // colours: precomputed, or SH evaluated from rows staged through LDS (coalesced)
    const bool need_sh = touched && a.copy_colors && !a.colors_precomp && a.sh.dc;
    (void)need_sh;
    if (stage_sh) __syncthreads();  // first half staged
    f3 dir = mk3(0.f, 0.f, 0.f), head = mk3(0.f, 0.f, 0.f);
    const bool sh_color = touched && a.copy_colors && !a.colors_precomp;
    if (touched && a.copy_colors && a.colors_precomp) rgb = ld3(a.colors_precomp + 3 * (size_t)idx);
    if (sh_color) {
        dir = sh_dir(p, ld3(a.campos));
        head = sh_rgb_head(a.D, dir, sh_dc3(a.sh.dc, a.sh.half, (size_t)src * a.sh.dc_stride),
                           s_sh + threadIdx.x * kPitch);
    }
    if (kSplit && stage_sh && ncolB > 0) {
        __syncthreads();  // every row's first half read
        const float invB = 1.0f / (float)ncolB;
#pragma unroll
        for (int i = 0; i < kShBPer; ++i) {
            const int f = threadIdx.x + 256 * i;
            const int row = (int)(((float)f + 0.5f) * invB), col = f - row * ncolB;
            if (row < nrow) s_sh[row * kShPitchAB + col] = shB[i];
        }
        __syncthreads();  // second half staged
    }
    if (sh_color) rgb = sh_rgb_tail(a.D, dir, head, s_sh + threadIdx.x * kPitch + (kSplit ? 0 : kShA), clamp_bits);
    if (idx < a.P) {
        if (touched) {  // (whole 64-B records: writing only the used 40 B measured slower — partial lines)
            Splat sp;
            sp.xy = pix;
            sp.pad0 = make_float2(0.f, 0.f);
            sp.co = conic;
            sp.rgbd = make_float4(rgb.x, rgb.y, rgb.z, a.aux_mask && auxv != 0u ? -depth : depth);  // (Splat: the aux bit)
            sp.pad1 = make_float4(0.f, 0.f, 0.f, 0.f);
            a.splat[idx] = sp;
        }
        // the geometry buffer's radii feed only the emission of grids too large to pack a rect
        // (and layout queries); the caller's radii serve everything else
        if (!a.rect_packed || !a.radii_out) a.radii[idx] = radius_out;
        if (a.radii_out) a.radii_out[idx] = radius_out;
        if (a.visible_out) a.visible_out[idx] = radius_out > 0;
        a.tiles_touched[idx] = touched;
        a.clamped[idx] = clamp_bits;
        a.depth_key[idx] = key;
        a.rect[idx] = rect;
        if (a.touched) a.touched[idx] = 0;
    }
    // workgroup total of instances and the range of the visible depth keys -> three atomics
    // (per slot: [0] instances, [1] max key, [2] ~min key: all start at 0).  The depth sort's MSD buckets
    // split [min, max] (depth_sort_msd).
    __shared__ uint32_t part[4][3];
    uint32_t s = touched, kmax = touched ? key : 0u, kmin_n = touched ? ~key : 0u;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        s += (uint32_t)__shfl_xor((int)s, o);
        kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
        kmin_n = max(kmin_n, (uint32_t)__shfl_xor((int)kmin_n, o));
    }
    if ((threadIdx.x & 63) == 0) {
        part[threadIdx.x >> 6][0] = s;
        part[threadIdx.x >> 6][1] = kmax;
        part[threadIdx.x >> 6][2] = kmin_n;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const uint32_t t = part[0][0] + part[1][0] + part[2][0] + part[3][0];
        if (t) {
            // kCounterSlots copies in separate 64-B lines: same-address device atomics from every
            // workgroup serialise (one slot: +35 us per counter at 1M Gaussians); the host sums them
            uint32_t* c = a.counters + kCounterStride * (blockIdx.x % kCounterSlots);
            atomicAdd(&c[0], t);
            atomicMax(&c[1], max(max(part[0][1], part[1][1]), max(part[2][1], part[3][1])));
            atomicMax(&c[2], max(max(part[0][2], part[1][2]), max(part[2][2], part[3][2])));
        }
    }
}

// The image buffer's per-forward state (counters, ranges, tile windows, work-list counts: ~30 KB at 512^2)
// zeroed before the preprocess: 16-B stores, one per thread.  (hipMemsetAsync's fill kernel took 7-8 us for it
// at the head of every view's chain, against ~2 us.)
__global__ __launch_bounds__(256) void k_zero16(uint4* __restrict__ p, uint32_t n16) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i < n16) p[i] = make_uint4(0u, 0u, 0u, 0u);
}

void launch_zero16(void* p, size_t bytes, hipStream_t s) {
    const uint32_t n16 = (uint32_t)(bytes / 16);
    if (n16) hipLaunchKernelGGL(k_zero16, dim3(div_up(n16, 256)), dim3(256), 0, s, static_cast<uint4*>(p), n16);
}

void launch_preprocess(const PreprocessArgs& a, hipStream_t s) {
    if (a.P <= 0) return;
    if (a.sh.half || a.index)  // (the one-pass staging needs the block's rows contiguous)
        hipLaunchKernelGGL(k_preprocess<true>, dim3(div_up(a.P, 256)), dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL(k_preprocess<false>, dim3(div_up(a.P, 256)), dim3(256), 0, s, a);
}

// Full 32-bit depth keys (the reference's key, rasterizer_impl.cu:86-92) from what preprocess left:
// the 32-bit LSD redo of the depth order that DGE_AMD_DEPTH_KEYS32=1 forces (a test of the MSD sort;
// the MSD pass has overwritten the original keys with relative ones by then).
__global__ __launch_bounds__(256) void k_depth_keys32(int P, const uint32_t* __restrict__ rect,
                                                      const Splat* __restrict__ splat, uint32_t* __restrict__ key) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    key[i] = rect[i] ? __float_as_uint(fabsf(splat[i].rgbd.w)) : 0xFFFFFFFFu;
}

void launch_depth_keys32(int P, const uint32_t* rect, const Splat* splat, uint32_t* key, hipStream_t s) {
    if (P <= 0) return;
    hipLaunchKernelGGL(k_depth_keys32, dim3(div_up(P, 256)), dim3(256), 0, s, P, rect, splat, key);
}

// test hook: the activations k_preprocess applies to raw parameters (gs_params.activation), same device
// functions, so the oracle can be handed exactly the values the fused path used
__global__ __launch_bounds__(256) void k_activate_params(int P, const float* __restrict__ raw_opacity,
                                                         const float* __restrict__ raw_scaling,
                                                         const float* __restrict__ raw_rotation,
                                                         float* __restrict__ opacity, float* __restrict__ scaling,
                                                         float* __restrict__ rotation) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    if (opacity) opacity[i] = act_sigmoid(raw_opacity[i]);
    if (scaling) {
        const f3 sc = ld3(raw_scaling + 3 * (size_t)i);
        scaling[3 * (size_t)i] = expf(sc.x);
        scaling[3 * (size_t)i + 1] = expf(sc.y);
        scaling[3 * (size_t)i + 2] = expf(sc.z);
    }
    if (rotation) {
        float len;
        const float4 q = act_normalize(*reinterpret_cast<const float4*>(raw_rotation + 4 * (size_t)i), len);
        *reinterpret_cast<float4*>(rotation + 4 * (size_t)i) = q;
    }
}

void launch_activate_params(int P, const float* raw_opacity, const float* raw_scaling, const float* raw_rotation,
                            float* opacity, float* scaling, float* rotation, hipStream_t s) {
    if (P <= 0) return;
    hipLaunchKernelGGL(k_activate_params, dim3(div_up(P, 256)), dim3(256), 0, s, P, raw_opacity, raw_scaling,
                       raw_rotation, opacity, scaling, rotation);
}

// checkFrustum (rasterizer_impl.cu:53-63)
__global__ __launch_bounds__(256) void k_mark_visible(int P, const float* __restrict__ means3D,
                                                      const float* __restrict__ view, uint8_t* __restrict__ present) {
    const int idx = blockIdx.x * 256 + threadIdx.x;
    if (idx >= P) return;
    const f3 pv = view_point(view, ld3(means3D + 3 * (size_t)idx));
    present[idx] = pv.z > 0.2f ? 1 : 0;
}

void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t s) {
    if (P <= 0) return;
    hipLaunchKernelGGL(k_mark_visible, dim3(div_up(P, 256)), dim3(256), 0, s, P, means3D, view, present);
}

}  // namespace gs
