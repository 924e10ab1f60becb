// Dev probe: time this library's radix sort against rocPRIM's on the
// binning workloads (1M depth keys, 32 bits; 3.6M tile keys, 10 bits) and
// check that both produce the same (stable) order.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>
#include <cstdio>
#include <vector>
#include <random>
#include "../../dge_amd/csrc/gs_internal.h"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

static int run(uint32_t n, int bits, const char* name) {
    std::vector<uint32_t> hk(n);
    std::mt19937 rng(1);
    for (auto& k : hk) k = bits == 32 ? (0x3e4ccccdu + (rng() % 50000000u)) : (rng() % (1u << bits));
    uint32_t *k0, *k1, *v0, *v1, *hist, *tot, *rk, *rv;
    const int nb = (int)((n + gs::kSortTile - 1) / gs::kSortTile);
    CK(hipMalloc(&k0, 4ull * n)); CK(hipMalloc(&k1, 4ull * n)); CK(hipMalloc(&v0, 4ull * n)); CK(hipMalloc(&v1, 4ull * n));
    CK(hipMalloc(&rk, 4ull * n)); CK(hipMalloc(&rv, 4ull * n));
    CK(hipMalloc(&hist, 4ull * 2048 * nb)); CK(hipMalloc(&tot, 4 * 2048));
    std::vector<uint32_t> iota(n);
    for (uint32_t i = 0; i < n; ++i) iota[i] = i;
    hipEvent_t a, b;
    CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
    // ours
    float ours = 0.f;
    int cur = 0;
    for (int rep = 0; rep < 6; ++rep) {
        CK(hipMemcpy(k0, hk.data(), 4ull * n, hipMemcpyHostToDevice));
        CK(hipEventRecord(a));
        cur = gs::radix_sort_pairs(k0, k1, v0, v1, n, 0, bits, gs::kMaxSinglePassBits, true, hist, tot, nb, 0);
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); if (rep >= 2) ours += ms / 4;
    }
    // rocprim
    size_t tmp_bytes = 0;
    CK(rocprim::radix_sort_pairs(nullptr, tmp_bytes, k0, rk, v0, rv, n, 0, bits));
    void* tmp; CK(hipMalloc(&tmp, tmp_bytes));
    float rp = 0.f;
    for (int rep = 0; rep < 6; ++rep) {
        CK(hipMemcpy(k0, hk.data(), 4ull * n, hipMemcpyHostToDevice));
        CK(hipMemcpy(v0, iota.data(), 4ull * n, hipMemcpyHostToDevice));
        CK(hipEventRecord(a));
        CK(rocprim::radix_sort_pairs(tmp, tmp_bytes, k0, rk, v0, rv, n, 0, bits));
        CK(hipEventRecord(b)); CK(hipEventSynchronize(b));
        float ms; CK(hipEventElapsedTime(&ms, a, b)); if (rep >= 2) rp += ms / 4;
    }
    // ours once more for the comparison
    CK(hipMemcpy(k0, hk.data(), 4ull * n, hipMemcpyHostToDevice));
    cur = gs::radix_sort_pairs(k0, k1, v0, v1, n, 0, bits, gs::kMaxSinglePassBits, true, hist, tot, nb, 0);
    std::vector<uint32_t> ov(n), pv(n);
    CK(hipMemcpy(ov.data(), cur ? v1 : v0, 4ull * n, hipMemcpyDeviceToHost));
    CK(hipMemcpy(pv.data(), rv, 4ull * n, hipMemcpyDeviceToHost));
    size_t diff = 0;
    for (uint32_t i = 0; i < n; ++i) diff += ov[i] != pv[i];
    printf("%s n=%u bits=%d: ours %.1f us, rocprim %.1f us (tmp %zu B), value mismatches %zu\n", name, n, bits,
           ours * 1e3, rp * 1e3, tmp_bytes, diff);
    return 0;
}

int main() {
    if (run(1000000, 32, "depth")) return 1;
    if (run(3608838, 10, "tile")) return 1;
    if (run(15000000, 13, "tile-1080p")) return 1;
    return 0;
}
