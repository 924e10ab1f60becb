// Probe of the gfx950 lane-swap semantics the backward reduce-scatter relies on
// (dev tool): prints which (operand, lane) lands in each output lane.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int* out) {
    const int l = threadIdx.x;
    const unsigned a = 1000 + l, b = 2000 + l;
    auto r = __builtin_amdgcn_permlane32_swap(a, b, false, false);
    auto s = __builtin_amdgcn_permlane16_swap(a, b, false, false);
    out[l] = r[0]; out[64 + l] = r[1]; out[128 + l] = s[0]; out[192 + l] = s[1];
}
int main() {
    int* d; int h[256];
    if (hipMalloc(&d, 1024) != hipSuccess) return 1;
    k<<<1, 64>>>(d);
    if (hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost) != hipSuccess) return 1;
    const char* names[4] = {"p32.first", "p32.second", "p16.first", "p16.second"};
    for (int t = 0; t < 4; ++t) {
        printf("%s:", names[t]);
        for (int l = 0; l < 64; l += 8) printf(" [%d]=%d", l, h[64 * t + l]);
        printf("\n");
    }
    return 0;
}
