// Probe (GPU box): VALU THROUGHPUT per SIMD of the blend kernels' instruction kinds, with W waves per SIMD
// (every CU holding W 64-thread workgroups per SIMD), each wave running independent chains of one kind.
// cost = a wave's s_memtime cycles / (W x its instructions): the SIMD cycles one wave-instruction occupies
// when the SIMD is never idle.  Answers: does a packed f32 op (v_pk_fma_f32) cost one or two scalar slots?
//   hipcc -O3 --offload-arch=gfx950 valu_tput.hip -o valu_tput && ./valu_tput
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef float f2v __attribute__((ext_vector_type(2)));
constexpr int kIters = 2048;

#define REP8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int KIND>
__global__ __launch_bounds__(64) void k_tput(float* out, unsigned long long* cyc, float seed) {
    const float s = seed + threadIdx.x * 1e-3f;
    f2v p0 = {s, s + 1}, p1 = {s + 2, s + 3}, p2 = {s + 4, s + 5}, p3 = {s + 6, s + 7}, p4 = {s + 8, s + 9},
        p5 = {s + 10, s + 11}, p6 = {s + 12, s + 13}, p7 = {s + 14, s + 15};
    float a0 = s, a1 = s + 1, a2 = s + 2, a3 = s + 3, a4 = s + 4, a5 = s + 5, a6 = s + 6, a7 = s + 7;
    const f2v m = {0.999f, 0.998f};
    const float k = 0.999f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < kIters; ++i) {
        // 4 x 8 independent instructions per iteration
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            if constexpr (KIND == 0) {  // v_fma_f32
#define X(j) asm volatile("v_fma_f32 %0, %0, %1, %1" : "+v"(a##j) : "v"(k));
                REP8(X)
#undef X
            } else if constexpr (KIND == 1) {  // v_pk_fma_f32
#define X(j) asm volatile("v_pk_fma_f32 %0, %0, %1, %1" : "+v"(p##j) : "v"(m));
                REP8(X)
#undef X
            } else if constexpr (KIND == 2) {  // v_pk_mul_f32
#define X(j) asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(p##j) : "v"(m));
                REP8(X)
#undef X
            } else if constexpr (KIND == 3) {  // v_add_f32_dpp (row op)
#define X(j) asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "+v"(a##j));
                asm volatile("s_nop 1");
                REP8(X)
#undef X
            } else if constexpr (KIND == 4) {  // v_permlane32_swap
#define X(j) asm volatile("v_permlane32_swap_b32 %0, %1" : "+v"(a##j), "+v"(p##j.x));
                REP8(X)
#undef X
            } else if constexpr (KIND == 5) {  // v_rcp_f32
#define X(j) asm volatile("v_rcp_f32 %0, %0" : "+v"(a##j));
                REP8(X)
#undef X
            } else if constexpr (KIND == 6) {  // v_cndmask_b32 (VOP3, sgpr mask)
#define X(j) asm volatile("v_cndmask_b32_e64 %0, %0, %1, s[0:1]" : "+v"(a##j) : "v"(k) : "s0", "s1");
                REP8(X)
#undef X
            } else if constexpr (KIND == 7) {  // v_mov_b32_dpp
#define X(j) asm volatile("v_mov_b32_dpp %0, %1 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf bound_ctrl:1" : "=v"(a##j) : "v"(p##j.y));
                asm volatile("s_nop 1");
                REP8(X)
#undef X
            } else if constexpr (KIND == 8) {  // v_exp_f32
#define X(j) asm volatile("v_exp_f32 %0, %0" : "+v"(a##j));
                REP8(X)
#undef X
            } else if constexpr (KIND == 9) {  // v_add_f32 (VOP2)
#define X(j) asm volatile("v_add_f32 %0, %0, %1" : "+v"(a##j) : "v"(k));
                REP8(X)
#undef X
            }
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    float r = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
    const f2v q = p0 + p1 + p2 + p3 + p4 + p5 + p6 + p7;
    out[blockIdx.x * 64 + threadIdx.x] = r + q.x + q.y;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int KIND>
static void run(const char* name, int W, float* out, unsigned long long* cyc) {
    int cus = 0;
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
    const int blocks = cus * 4 * W;
    hipLaunchKernelGGL(k_tput<KIND>, dim3(blocks), dim3(64), 0, 0, out, cyc, 1.0f);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(blocks);
    hipMemcpy(h.data(), cyc, blocks * sizeof(unsigned long long), hipMemcpyDeviceToHost);
    double s = 0;
    for (auto v : h) s += (double)v;
    const double per_wave = s / blocks;
    const double instrs = (double)kIters * 32;
    printf("%-18s W=%d  wave cycles %.0f  cycles/instr/wave %.2f  SIMD cycles per wave-instruction %.2f\n", name, W,
           per_wave, per_wave / instrs, per_wave / instrs / W);
}

int main() {
    float* out;
    unsigned long long* cyc;
    hipMalloc(&out, 256 * 4 * 16 * 64 * sizeof(float));
    hipMalloc(&cyc, 256 * 4 * 16 * sizeof(unsigned long long));
    for (int W : {1, 4, 8}) {
        run<9>("v_add_f32", W, out, cyc);
        run<0>("v_fma_f32", W, out, cyc);
        run<1>("v_pk_fma_f32", W, out, cyc);
        run<2>("v_pk_mul_f32", W, out, cyc);
        run<6>("v_cndmask_b32_e64", W, out, cyc);
        run<3>("v_add_f32_dpp", W, out, cyc);
        run<7>("v_mov_b32_dpp", W, out, cyc);
        run<4>("v_permlane32_swap", W, out, cyc);
        run<5>("v_rcp_f32", W, out, cyc);
        run<8>("v_exp_f32", W, out, cyc);
    }
    hipFree(out);
    hipFree(cyc);
    return 0;
}
