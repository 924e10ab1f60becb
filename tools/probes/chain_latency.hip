// Probe (GPU box): cycles per step of dependent VALU chains for one lone wave
// (s_memtime), to size the blend's per-entry transmittance chain.
//   hipcc -O3 --offload-arch=gfx950 chain_latency.hip -o chain_latency
#include <hip/hip_runtime.h>
#include <cstdio>
typedef float f2v __attribute__((ext_vector_type(2)));

constexpr int N = 4096;

__global__ void k_probe(const float* in, float* out, unsigned long long* cyc) {
    const int lane = threadIdx.x;
    float a = in[lane], b = in[64 + lane];
    unsigned long long t0, t1;
    // 1: dependent v_mul chain
    float x = a;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) { x = x * b; asm volatile("" : "+v"(x)); }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[0] = t1 - t0; out[lane] = x;
    // 2: the signed-T chain: mul, cmp, cndmask
    float Ts = 1.0f;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        const float tT = Ts * (1.0f - a);
        Ts = tT >= 1e-4f ? tT : -fabsf(Ts);
        asm volatile("" : "+v"(Ts));
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[1] = t1 - t0; out[64 + lane] = Ts;
    // 3: 4 independent mul chains
    float x0 = a, x1 = a + 1, x2 = a + 2, x3 = a + 3;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        x0 = x0 * b; x1 = x1 * b; x2 = x2 * b; x3 = x3 * b;
        asm volatile("" : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3));
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[2] = t1 - t0; out[128 + lane] = x0 + x1 + x2 + x3;
    // 4: dependent v_pk_fma chain
    f2v c = {a, b}, m = {b, a};
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) { c = __builtin_elementwise_fma(m, c, m); asm volatile("" : "+v"(c)); }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[3] = t1 - t0; out[192 + lane] = c.x + c.y;
    // 5: VALU compare -> SALU use -> VALU (the blended vote)
    unsigned long long bits = 0;
    float w = a;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        w = w * b;
        const unsigned long long vm = __builtin_amdgcn_fcmpf(w, 0.0f, 2);
        bits |= vm ? (1ull << (i & 63)) : 0ull;
        asm volatile("" : "+v"(w));
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[4] = t1 - t0; out[256 + lane] = w + (float)(bits & 1);
    // 6: __any(x > 0) branch per step (VALU compare -> scalar branch)
    float y = a;
    int cnt = 0;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        y = y * b;
        if (!__any(y > 0.0f)) { cnt++; }
        asm volatile("" : "+v"(y));
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[5] = t1 - t0; out[320 + lane] = y + cnt;
    // 7: v_readfirstlane -> SALU -> VALU
    unsigned s = 0;
    unsigned v = lane;
    t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < N; ++i) {
        s += __builtin_amdgcn_readfirstlane(v);
        v = v + s;
        asm volatile("" : "+v"(v));
    }
    t1 = __builtin_amdgcn_s_memtime();
    cyc[6] = t1 - t0; out[384 + lane] = (float)v;
}

int main() {
    float *in, *out; unsigned long long* cyc;
    hipMalloc(&in, 1024 * 4); hipMalloc(&out, 1024 * 4); hipMalloc(&cyc, 64 * 8);
    float h[1024]; for (int i = 0; i < 1024; ++i) h[i] = 0.5f + 0.0001f * i;
    hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
    unsigned long long c[8];
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, in, out, cyc);
        hipDeviceSynchronize();
    }
    hipMemcpy(c, cyc, sizeof(c), hipMemcpyDeviceToHost);
    const char* names[] = {"dep v_mul", "signed-T chain (mul,cmp,cndmask)", "4 indep v_mul", "dep v_pk_fma",
                           "mul + fcmp->SALU vote", "mul + __any branch", "readfirstlane->SALU->VALU"};
    for (int i = 0; i < 7; ++i) printf("%-36s %8.2f cycles/step\n", names[i], (double)c[i] / N);
    return 0;
}
