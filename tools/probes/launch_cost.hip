// Host cost of the HIP calls a forward enqueues (dev probe, GPU): empty-kernel launch, 16-B memset,
// 64-B D2H copy into pinned memory, event record — median host us per call over 2000 calls.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <vector>

__global__ void k_empty(int* p, int n) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && n < 0) p[0] = n;
}

template <class F>
static double per_call_us(F f, int n = 2000) {
    std::vector<double> t;
    for (int r = 0; r < 5; ++r) {
        auto a = std::chrono::steady_clock::now();
        for (int i = 0; i < n; ++i) f();
        auto b = std::chrono::steady_clock::now();
        hipDeviceSynchronize();
        t.push_back(std::chrono::duration<double, std::micro>(b - a).count() / n);
    }
    std::sort(t.begin(), t.end());
    return t[2];
}

int main() {
    hipStream_t s;
    hipStreamCreate(&s);
    int* d = nullptr;
    hipMalloc(&d, 1 << 20);
    unsigned* h = nullptr;
    hipHostMalloc((void**)&h, 4096, hipHostMallocDefault);
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    printf("launch 1 block      %.2f us\n", per_call_us([&] { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, s, d, 1); }));
    printf("launch 4096 blocks  %.2f us\n", per_call_us([&] { hipLaunchKernelGGL(k_empty, dim3(4096), dim3(256), 0, s, d, 1); }));
    printf("memset 16 B         %.2f us\n", per_call_us([&] { hipMemsetAsync(d, 0, 16, s); }));
    printf("memset 2 KB         %.2f us\n", per_call_us([&] { hipMemsetAsync(d, 0, 2048, s); }));
    printf("D2H 256 B pinned    %.2f us\n", per_call_us([&] { hipMemcpyAsync(h, d, 256, hipMemcpyDeviceToHost, s); }));
    printf("event record        %.2f us\n", per_call_us([&] { hipEventRecord(ev, s); }));
    printf("getlasterror        %.2f us\n", per_call_us([&] { (void)hipGetLastError(); }));
    return 0;
}
