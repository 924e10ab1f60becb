// Probe (GPU box): the queue time between two kernels for the stream operations a step puts between its
// kernels — nothing, an event record (with / without timing), a wait on an already-complete event of the
// same or another stream, a wait on another stream's running kernel, a small D2H copy + record, a small
// memset.  Kernel A (one wave) spins ~20 us and stores s_memrealtime at its end; kernel B stores it at its
// start; gap = B.start - A.end (100 MHz clock, 10 ns).  Median of 25 repeats per case.
//   hipcc -O3 --offload-arch=gfx950 queue_gap.hip -o queue_gap && ./queue_gap
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

#define CK(x)                                                                      \
    do {                                                                           \
        hipError_t e_ = (x);                                                       \
        if (e_ != hipSuccess) {                                                    \
            printf("HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); \
            return 1;                                                              \
        }                                                                          \
    } while (0)

__global__ void k_a(unsigned long long* t, unsigned long long spin) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin) {
    }
    if (threadIdx.x == 0) t[0] = __builtin_amdgcn_s_memrealtime();
}
__global__ void k_b(unsigned long long* t) {
    if (threadIdx.x == 0) t[1] = __builtin_amdgcn_s_memrealtime();
}

int main() {
    unsigned long long* t;
    CK(hipMalloc(&t, 64));
    unsigned long long* h;
    CK(hipHostMalloc((void**)&h, 4096, hipHostMallocDefault));
    void* small;
    CK(hipMalloc(&small, 4096));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t e_nt, e_t, e_done;
    CK(hipEventCreateWithFlags(&e_nt, hipEventDisableTiming));
    CK(hipEventCreate(&e_t));
    CK(hipEventCreateWithFlags(&e_done, hipEventDisableTiming));
    const unsigned long long spin = 2000;  // 20 us at 100 MHz
    const char* names[] = {"back to back",
                           "event record (no timing)",
                           "event record (timing)",
                           "wait, same stream's complete event",
                           "wait, other stream's complete event",
                           "wait, other stream's running kernel (B on s2)",
                           "2 waits on complete events",
                           "D2H copy 2 KB + event record",
                           "memset 4 KB",
                           "record + wait + record + wait (a fork/join)"};
    const int ncase = sizeof(names) / sizeof(names[0]);
    for (int c = 0; c < ncase; ++c) {
        std::vector<double> gaps;
        for (int r = 0; r < 27; ++r) {
            CK(hipEventRecord(e_done, s2));  // complete long before A ends
            CK(hipStreamSynchronize(s2));
            hipStream_t sb = s1;
            hipLaunchKernelGGL(k_a, dim3(1), dim3(64), 0, s1, t, spin);
            switch (c) {
            case 0: break;
            case 1: CK(hipEventRecord(e_nt, s1)); break;
            case 2: CK(hipEventRecord(e_t, s1)); break;
            case 3:
                CK(hipEventRecord(e_nt, s1));
                CK(hipStreamWaitEvent(s1, e_nt, 0));
                break;
            case 4: CK(hipStreamWaitEvent(s1, e_done, 0)); break;
            case 5:
                CK(hipEventRecord(e_nt, s1));
                CK(hipStreamWaitEvent(s2, e_nt, 0));
                sb = s2;
                break;
            case 6:
                CK(hipStreamWaitEvent(s1, e_done, 0));
                CK(hipStreamWaitEvent(s1, e_done, 0));
                break;
            case 7:
                CK(hipMemcpyAsync(h, small, 2048, hipMemcpyDeviceToHost, s1));
                CK(hipEventRecord(e_nt, s1));
                break;
            case 8: CK(hipMemsetAsync(small, 0, 4096, s1)); break;
            case 9:
                CK(hipEventRecord(e_nt, s1));
                CK(hipStreamWaitEvent(s2, e_nt, 0));
                CK(hipEventRecord(e_t, s2));
                CK(hipStreamWaitEvent(s1, e_t, 0));
                break;
            }
            hipLaunchKernelGGL(k_b, dim3(1), dim3(64), 0, sb, t);
            CK(hipDeviceSynchronize());
            unsigned long long ht[2];
            CK(hipMemcpy(ht, t, 16, hipMemcpyDeviceToHost));
            if (r >= 2) gaps.push_back(((double)ht[1] - (double)ht[0]) * 0.01);  // us
        }
        std::sort(gaps.begin(), gaps.end());
        printf("%-48s gap p50 %7.2f us  min %7.2f  max %7.2f\n", names[c], gaps[gaps.size() / 2], gaps.front(),
               gaps.back());
    }
    return 0;
}
