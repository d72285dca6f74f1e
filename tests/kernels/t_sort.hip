// Test program (tests/test_kernels_gpu.py) and timing harness for the device radix sort
// (4dlangsplat_amd/csrc/sort.hip): stable sort of (key, value) pairs checked against
// std::stable_sort on the host, on the binning's two shapes:
//   depth order : n = P keys, 32 bits (float bits of positive depths, culled = 0xFFFFFFFF)
//   tile order  : n = K keys, ceil(log2 tiles) bits
// Usage: t_sort [reps]   (reps > 0 also prints the mean time per sort)
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <random>
#include <vector>
#include "../../4dlangsplat_amd/csrc/sort.hip"

static int run(const char* name, size_t n, int bits, bool depthlike, int reps) {
    std::mt19937 rng(1234);
    std::vector<uint32_t> hk(n), hv(n);
    for (size_t i = 0; i < n; ++i) {
        if (depthlike) {
            const float z = 2.0f + 8.0f * (float)(rng() & 0xFFFFFF) / 16777216.0f;
            uint32_t b; std::memcpy(&b, &z, 4);
            hk[i] = (rng() % 10 == 0) ? 0xFFFFFFFFu : b;
        } else {
            hk[i] = (uint32_t)(rng() % 5440u);
        }
        hv[i] = (uint32_t)i;
    }
    uint32_t *ka, *va, *kb, *vb;
    void* tmp;
    (void)hipMalloc(&ka, n * 4); (void)hipMalloc(&va, n * 4); (void)hipMalloc(&kb, n * 4); (void)hipMalloc(&vb, n * 4);
    (void)hipMalloc(&tmp, lsr::radix_temp_bytes(n));
    (void)hipMemcpy(ka, hk.data(), n * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(va, hv.data(), n * 4, hipMemcpyHostToDevice);
    const bool in_b = lsr::radix_sort_pairs(ka, va, kb, vb, n, 0, bits, tmp, 0);
    std::vector<uint32_t> ok(n), ov(n);
    (void)hipMemcpy(ok.data(), in_b ? kb : ka, n * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(ov.data(), in_b ? vb : va, n * 4, hipMemcpyDeviceToHost);
    std::vector<uint32_t> idx(n);
    std::iota(idx.begin(), idx.end(), 0u);
    const uint32_t mask = bits >= 32 ? 0xFFFFFFFFu : ((1u << bits) - 1u);
    std::stable_sort(idx.begin(), idx.end(), [&](uint32_t a, uint32_t b) { return (hk[a] & mask) < (hk[b] & mask); });
    size_t bad = 0;
    for (size_t i = 0; i < n; ++i)
        if (ov[i] != idx[i] || ok[i] != hk[idx[i]]) { if (bad < 3) printf("  [%zu] got (%u,%u) want (%u,%u)\n", i, ok[i], ov[i], hk[idx[i]], idx[i]); ++bad; }
    printf("%s n=%zu bits=%d: %s\n", name, n, bits, bad ? "FAIL" : "ok");
    if (reps > 0) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
        (void)hipEventRecord(e0, 0);
        for (int r = 0; r < reps; ++r) lsr::radix_sort_pairs(ka, va, kb, vb, n, 0, bits, tmp, 0);
        (void)hipEventRecord(e1, 0);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        printf("  %.1f us per sort (%.0f GB/s of 16 B/key/pass)\n", 1e3 * ms / reps,
               16.0 * n * ((bits + 7) / 8) / (1e6 * ms / reps));
    }
    (void)hipFree(ka); (void)hipFree(va); (void)hipFree(kb); (void)hipFree(vb); (void)hipFree(tmp);
    return bad ? 1 : 0;
}

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 0;
    int rc = 0;
    rc |= run("small", 1000, 32, true, 0);
    rc |= run("odd", 4097, 13, false, 0);
    rc |= run("depth", 2000000, 32, true, reps);
    rc |= run("tile", 7800000, 13, false, reps);
    return rc;
}
