// gs_optim.hip — the optimizer step after the backward, for gfx950.
//
// The reference trains the Gaussians with torch.optim.Adam(eps=1e-15) over six
// parameter groups (gaussian_model.py:336-380: xyz, f_dc, f_rest, opacity,
// scaling, rotation; 59 floats per Gaussian).  torch runs that as a chain of
// elementwise kernels per tensor (lerp, mul, addcmul, sqrt, div, add,
// addcdiv), each a full pass over HBM.  Here ONE launch updates every group:
// per element read p, g, m, v and write p, m, v (28 B) — the HBM roofline of
// the step (~1.65 GB per step at 1M Gaussians).
//
// Arithmetic follows the Adam DGE runs — torch.optim.Adam on CUDA/ROCm tensors,
// i.e. the foreach implementation (torch/optim/adam.py, _multi_tensor_adam) —
// in the float32 operation order its kernels compile to on ROCm (ATen's
// elementwise kernels are built with fp contraction on; the order was
// measured bitwise against torch on an MI355X, tools/probes/adam_order.py):
//   m = fma(1 - b1, g - m, m)          _foreach_lerp_(exp_avgs, grads, 1 - b1)  (weight < 0.5 branch)
//   v = fma(1 - b2, g * g, v * b2)     _foreach_mul_(exp_avg_sqs, b2); _foreach_addcmul_(.., g, g, 1 - b2)
//   d = sqrt(v) / bc2_sqrt + eps       _foreach_sqrt; _foreach_div_(.., bc2_sqrt); _foreach_add_(.., eps)
//   p = fma(-step_size, m / d, p)      _foreach_addcdiv_(params, exp_avgs, denom, -step_size)
// with step_size = lr / (1 - b1^t) and bc2_sqrt = sqrt(1 - b2^t) computed on
// the host in double, as torch does with Python floats.
#pragma clang fp contract(off)
#include "gs_internal.h"
#include "gs_raster.h"

namespace gs {

struct AdamLaunch {
    int nseg;
    gs_adam_segment seg[GS_ADAM_MAX_SEGMENTS];
    long long block0[GS_ADAM_MAX_SEGMENTS + 1];  // first block of each segment
    float b1, b2, one_minus_b1, one_minus_b2, eps;
};

constexpr int kAdamThreads = 256;
constexpr int kAdamVec = 4;                          // float4 per thread per iteration
constexpr long long kAdamBlockElems = (long long)kAdamThreads * kAdamVec * 4;  // 4 float4 per thread

__device__ __forceinline__ void adam_one(float& p, float g, float& m, float& v, const AdamLaunch& a, float nstep,
                                         float bc2s) {
    m = __builtin_fmaf(a.one_minus_b1, g - m, m);
    v = __builtin_fmaf(a.one_minus_b2, g * g, v * a.b2);
    const float d = sqrtf(v) / bc2s + a.eps;
    p = __builtin_fmaf(nstep, m / d, p);
}

__global__ __launch_bounds__(kAdamThreads) void k_adam(AdamLaunch a) {
    int s = 0;
#pragma unroll
    for (int i = 1; i < GS_ADAM_MAX_SEGMENTS; ++i) s += (i < a.nseg && (long long)blockIdx.x >= a.block0[i]) ? 1 : 0;
    const gs_adam_segment& sg = a.seg[s];
    const long long e0 = ((long long)blockIdx.x - a.block0[s]) * kAdamBlockElems;
    const long long n = sg.n;
    const float nstep = -sg.step_size;
    const float bc2s = sg.bias_correction2_sqrt;
    if (sg.grad_pitch > 0) {
        // grad rows at a pitch (a row-major gradient bucket's column block): p, m, v packed as float4, each
        // thread's four gradients gathered (element e of row e / w, column e % w)
        const uint32_t w = (uint32_t)sg.grad_width, pitch = (uint32_t)sg.grad_pitch;
        auto gat = [&](long long e) { return sg.grad[(size_t)((uint64_t)e / w) * pitch + (uint64_t)e % w]; };
        const bool vec4 = ((reinterpret_cast<uintptr_t>(sg.param) | reinterpret_cast<uintptr_t>(sg.exp_avg) |
                            reinterpret_cast<uintptr_t>(sg.exp_avg_sq)) & 15) == 0;
        for (int u = 0; u < 4; ++u) {
            const long long e4 = e0 + 4 * ((long long)u * kAdamThreads + threadIdx.x);
            if (vec4 && e4 + 3 < n) {
                float4 p = reinterpret_cast<float4*>(sg.param)[e4 >> 2];
                float4 m = reinterpret_cast<float4*>(sg.exp_avg)[e4 >> 2];
                float4 v = reinterpret_cast<float4*>(sg.exp_avg_sq)[e4 >> 2];
                adam_one(p.x, gat(e4), m.x, v.x, a, nstep, bc2s);
                adam_one(p.y, gat(e4 + 1), m.y, v.y, a, nstep, bc2s);
                adam_one(p.z, gat(e4 + 2), m.z, v.z, a, nstep, bc2s);
                adam_one(p.w, gat(e4 + 3), m.w, v.w, a, nstep, bc2s);
                reinterpret_cast<float4*>(sg.param)[e4 >> 2] = p;
                reinterpret_cast<float4*>(sg.exp_avg)[e4 >> 2] = m;
                reinterpret_cast<float4*>(sg.exp_avg_sq)[e4 >> 2] = v;
            } else {
                for (long long e = e4; e < n && e < e4 + 4; ++e) {
                    float pe = sg.param[e], me = sg.exp_avg[e], ve = sg.exp_avg_sq[e];
                    adam_one(pe, gat(e), me, ve, a, nstep, bc2s);
                    sg.param[e] = pe;
                    sg.exp_avg[e] = me;
                    sg.exp_avg_sq[e] = ve;
                }
            }
        }
        return;
    }
    const bool vec = ((reinterpret_cast<uintptr_t>(sg.param) | reinterpret_cast<uintptr_t>(sg.grad) |
                       reinterpret_cast<uintptr_t>(sg.exp_avg) | reinterpret_cast<uintptr_t>(sg.exp_avg_sq)) & 15) == 0;
    if (vec) {
        float4* P = reinterpret_cast<float4*>(sg.param);
        const float4* G = reinterpret_cast<const float4*>(sg.grad);
        float4* Mv = reinterpret_cast<float4*>(sg.exp_avg);
        float4* V = reinterpret_cast<float4*>(sg.exp_avg_sq);
        float4 p[4], g[4], m[4], v[4];
        long long i4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {  // all loads of the thread first
            i4[u] = (e0 >> 2) + (long long)u * kAdamThreads + threadIdx.x;
            if (4 * i4[u] + 3 < n) {
                p[u] = P[i4[u]];
                g[u] = G[i4[u]];
                m[u] = Mv[i4[u]];
                v[u] = V[i4[u]];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (4 * i4[u] + 3 < n) {
                adam_one(p[u].x, g[u].x, m[u].x, v[u].x, a, nstep, bc2s);
                adam_one(p[u].y, g[u].y, m[u].y, v[u].y, a, nstep, bc2s);
                adam_one(p[u].z, g[u].z, m[u].z, v[u].z, a, nstep, bc2s);
                adam_one(p[u].w, g[u].w, m[u].w, v[u].w, a, nstep, bc2s);
                P[i4[u]] = p[u];
                Mv[i4[u]] = m[u];
                V[i4[u]] = v[u];
            } else {
                for (long long e = 4 * i4[u]; e < n && e < 4 * i4[u] + 4; ++e) {  // ragged tail
                    float pe = sg.param[e], me = sg.exp_avg[e], ve = sg.exp_avg_sq[e];
                    adam_one(pe, sg.grad[e], me, ve, a, nstep, bc2s);
                    sg.param[e] = pe;
                    sg.exp_avg[e] = me;
                    sg.exp_avg_sq[e] = ve;
                }
            }
        }
    } else {
        for (long long e = e0 + threadIdx.x; e < e0 + kAdamBlockElems && e < n; e += kAdamThreads) {
            float pe = sg.param[e], me = sg.exp_avg[e], ve = sg.exp_avg_sq[e];
            adam_one(pe, sg.grad[e], me, ve, a, nstep, bc2s);
            sg.param[e] = pe;
            sg.exp_avg[e] = me;
            sg.exp_avg_sq[e] = ve;
        }
    }
}

}  // namespace gs

extern "C" int gs_adam_step(const gs_adam_segment* segs, int nseg, double beta1, double beta2, float eps,
                            gs_stream_t stream) {
    using namespace gs;
    if (nseg < 0 || (nseg > 0 && !segs)) return report_error(GS_ERR_INVALID_ARG, "gs_adam_step: bad segment list");
    hipStream_t s = (hipStream_t)stream;
    int i = 0;
    while (i < nseg) {  // launches of up to GS_ADAM_MAX_SEGMENTS non-empty segments
        AdamLaunch a{};
        a.b1 = (float)beta1;
        a.b2 = (float)beta2;
        a.one_minus_b1 = (float)(1.0 - beta1);  // (torch: the Python float 1 - beta, rounded once)
        a.one_minus_b2 = (float)(1.0 - beta2);
        a.eps = eps;
        long long blocks = 0;
        int k = 0;
        for (; i < nseg && k < GS_ADAM_MAX_SEGMENTS; ++i) {
            const gs_adam_segment& sg = segs[i];
            if (sg.n < 0 || (sg.n > 0 && (!sg.param || !sg.grad || !sg.exp_avg || !sg.exp_avg_sq)))
                return report_error(GS_ERR_INVALID_ARG, "gs_adam_step: segment with NULL tensors");
            if (sg.grad_pitch < 0 || (sg.grad_pitch > 0 && (sg.grad_width <= 0 || sg.grad_pitch < sg.grad_width ||
                                                            sg.n % sg.grad_width)))
                return report_error(GS_ERR_INVALID_ARG, "gs_adam_step: grad rows need 0 < width <= pitch, n % width == 0");
            if (sg.n == 0) continue;
            a.seg[k] = sg;
            a.block0[k] = blocks;
            blocks += (sg.n + kAdamBlockElems - 1) / kAdamBlockElems;
            ++k;
        }
        a.nseg = k;
        a.block0[k] = blocks;
        if (blocks == 0) continue;
        if (blocks > 0x7FFFFFFF) return report_error(GS_ERR_INVALID_ARG, "gs_adam_step: segments too large");
        hipLaunchKernelGGL(k_adam, dim3((unsigned)blocks), dim3(kAdamThreads), 0, s, a);
        const hipError_t e = hipGetLastError();
        if (e != hipSuccess) return report_error(GS_ERR_HIP, hipGetErrorString(e));
    }
    return GS_OK;
}
