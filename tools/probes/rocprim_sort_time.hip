// Dev probe (measurement only, not shipped): rocPRIM's radix_sort_pairs on the binning shapes, to know
// what a tuned library sort reaches on MI355X: 1M depth keys on 27 bits with 8-B values (c2's depth
// sort), 3.6M tile keys on 10 bits with 8-B values (c2's tile sort), 42.8M on 13 bits (c4).
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <random>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

static int run(uint32_t n, int bits, const char* name) {
    std::vector<uint32_t> hk(n);
    std::mt19937 rng(1);
    for (auto& k : hk) k = rng() & ((1u << bits) - 1u);
    uint32_t *k0, *k1;
    unsigned long long *v0, *v1;
    CK(hipMalloc(&k0, 4ull * n)); CK(hipMalloc(&k1, 4ull * n));
    CK(hipMalloc(&v0, 8ull * n)); CK(hipMalloc(&v1, 8ull * n));
    CK(hipMemcpy(k0, hk.data(), 4ull * n, hipMemcpyHostToDevice));
    CK(hipMemset(v0, 0, 8ull * n));
    size_t tmp_bytes = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0, k1, v0, v1, n, 0, bits));
    void* tmp; CK(hipMalloc(&tmp, tmp_bytes));
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    float best = 1e9f, sum = 0.f;
    for (int rep = 0; rep < 12; ++rep) {
        CK(hipEventRecord(a));
        CK(rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, k1, v0, v1, n, 0, bits));
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b));
        if (rep >= 2) { sum += ms / 10; best = ms < best ? ms : best; }
    }
    printf("rocprim %s n=%u bits=%d (u32 key, u64 value): mean %.1f us, best %.1f us\n", name, n, bits, sum * 1e3,
           best * 1e3);
    CK(hipFree(tmp)); CK(hipFree(k0)); CK(hipFree(k1)); CK(hipFree(v0)); CK(hipFree(v1));
    return 0;
}

int main() {
    if (run(1000000, 27, "depth")) return 1;
    if (run(3608838, 10, "tile")) return 1;
    if (run(42800000, 13, "tile-1080p")) return 1;
    return 0;
}
