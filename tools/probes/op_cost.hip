// Probe (GPU box): cycles per call of the blend building blocks for one lone
// wave (s_memtime): cull_keep, pixel_alpha4 (4 entries), the signed-T chain.
//   hipcc -O3 --offload-arch=gfx950 -I../../dge_amd/csrc op_cost.hip -o op_cost
#include <hip/hip_runtime.h>
#include <cstdio>
#include "gs_common.h"
using namespace gs;

constexpr int N = 2048;

__device__ __forceinline__ void pixel_alpha4(f4v x, f4v y, f4v cx, f4v ncy, f4v cz, f4v op, float npx, float npy,
                                             f4v& dx, f4v& dy, f4v& G, f4v& alpha, bool (&ok)[4]) {
#pragma clang fp contract(off)
    dx = x + npx;
    dy = y + npy;
    const f4v power = -0.5f * (cx * dx * dx + cz * dy * dy) + ncy * dx * dy;
    G = gs_exp4(power);
    const f4v oG = op * G;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        alpha[u] = fminf(0.99f, oG[u]);
        ok[u] = !(power[u] > 0.0f) && !(alpha[u] < 1.0f / 255.0f);
    }
}

__global__ void k_probe(const float* in, float* out, unsigned long long* cyc, int nwaves_busy) {
    const int lane = threadIdx.x & 63;
    const float a = in[lane], b = in[64 + lane];
    unsigned long long t0, t1;
    // 1: cull_keep, two independent entries per step
    float2 xy0 = make_float2(a * 10.f, b * 10.f), xy1 = make_float2(b * 11.f, a * 9.f);
    float4 co = make_float4(0.3f, 0.01f * a, 0.25f, 0.7f);
    int keep = 0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        keep += cull_keep(xy0, co, 8.f, 16.f) ? 1 : 0;
        keep += cull_keep(xy1, co, 8.f, 16.f) ? 1 : 0;
        asm volatile("" : "+v"(xy0.x), "+v"(xy1.x));
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[0] = (t1 - t0);
    out[lane] = (float)keep;
    // 2: pixel_alpha4 (4 entries), results folded
    f4v x = {a, b, a + 1, b + 1}, y = {b, a, b + 2, a + 2}, cx = {0.3f, 0.2f, 0.1f, 0.4f}, ncy = {-0.01f, 0.f, 0.02f, 0.f},
        cz = {0.2f, 0.3f, 0.2f, 0.1f}, op = {0.5f, 0.6f, 0.7f, 0.8f};
    f4v acc = {0.f, 0.f, 0.f, 0.f};
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        f4v dx, dy, G, al;
        bool ok[4];
        pixel_alpha4(x, y, cx, ncy, cz, op, -3.f, -4.f, dx, dy, G, al, ok);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] += ok[u] ? al[u] : 0.f;
        asm volatile("" : "+v"(x));
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[1] = (t1 - t0);
    out[64 + lane] = acc.x + acc.y + acc.z + acc.w;
    // 3: two pixel_alpha4 per step (8 entries)
    f4v x2 = x + 0.5f, acc2 = acc;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        f4v dx, dy, G, al, dx2, dy2, G2, al2;
        bool ok[4], ok2[4];
        pixel_alpha4(x, y, cx, ncy, cz, op, -3.f, -4.f, dx, dy, G, al, ok);
        pixel_alpha4(x2, y, cx, ncy, cz, op, -3.f, -4.f, dx2, dy2, G2, al2, ok2);
#pragma unroll
        for (int u = 0; u < 4; ++u) { acc[u] += ok[u] ? al[u] : 0.f; acc2[u] += ok2[u] ? al2[u] : 0.f; }
        asm volatile("" : "+v"(x), "+v"(x2));
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[2] = (t1 - t0);
    out[128 + lane] = acc.x + acc2.y;
    // 4: the scalar exp alone (gs_exp), 4 independent
    float e0 = a * -1.f, e1 = b * -1.f, e2 = -a - 1.f, e3 = -b - 1.f;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        e0 = gs_exp(e0) - 1.5f; e1 = gs_exp(e1) - 1.5f; e2 = gs_exp(e2) - 1.5f; e3 = gs_exp(e3) - 1.5f;
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[3] = (t1 - t0);
    out[192 + lane] = e0 + e1 + e2 + e3;
    // 5: 32 independent v_fma per step (issue rate)
    float f[8];
    for (int k = 0; k < 8; ++k) f[k] = a + k;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) f[k] = __builtin_fmaf(f[k], b, 0.25f);
        asm volatile("" : "+v"(f[0]), "+v"(f[1]), "+v"(f[2]), "+v"(f[3]), "+v"(f[4]), "+v"(f[5]), "+v"(f[6]), "+v"(f[7]));
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[4] = (t1 - t0);
    out[256 + lane] = f[0] + f[7];
    // 6: 16 independent v_pk_fma per step
    f2v g[8];
    for (int k = 0; k < 8; ++k) g[k] = f2v{a + k, b + k};
    const f2v bb = {b, a}, cc = {0.25f, 0.5f};
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
#pragma unroll
        for (int r = 0; r < 2; ++r)
#pragma unroll
            for (int k = 0; k < 8; ++k) g[k] = __builtin_elementwise_fma(g[k], bb, cc);
        asm volatile("" : "+v"(g[0]), "+v"(g[1]), "+v"(g[2]), "+v"(g[3]), "+v"(g[4]), "+v"(g[5]), "+v"(g[6]), "+v"(g[7]));
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[5] = (t1 - t0);
    out[320 + lane] = g[0].x + g[7].y;
}

int main() {
    float *in, *out;
    unsigned long long* cyc;
    (void)hipMalloc(&in, 1024 * 4);
    (void)hipMalloc(&out, 4096 * 4);
    (void)hipMalloc(&cyc, 64 * 8);
    float h[1024];
    for (int i = 0; i < 1024; ++i) h[i] = 0.5f + 0.0001f * i;
    (void)hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    unsigned long long c[8];
    const char* names[] = {"cull_keep x2", "pixel_alpha4 (4 entries)", "pixel_alpha4 x2 (8 entries)", "gs_exp x4 (dep chains)",
                           "32 indep v_fma", "16 indep v_pk_fma"};
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, in, out, cyc, 1);
        (void)hipDeviceSynchronize();
    }
    (void)hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    for (int i = 0; i < 6; ++i) printf("%-32s %8.1f cycles/step\n", names[i], (double)c[i] / N);
    return 0;
}
