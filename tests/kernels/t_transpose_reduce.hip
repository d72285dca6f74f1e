// Test program (tests/test_kernels_gpu.py): checks lsr::wave_transpose_reduce<Q> on exact integer
// data -- every lane's register k must hold the wave total of the quantity the mapping names.
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../4dlangsplat_amd/csrc/lsr_common.h"

template <int Q>
__global__ void k(float* out) {
    float v[Q];
    const int l = threadIdx.x;
#pragma unroll
    for (int q = 0; q < Q; ++q) v[q] = (float)((q + 1) * 100 + (l % 7));   // per-lane distinct, exact in f32
    lsr::wave_transpose_reduce<Q>(v);
    constexpr int R = Q >= 64 ? Q / 64 : 1;
#pragma unroll
    for (int k2 = 0; k2 < R; ++k2) out[l * R + k2] = v[k2];
}

template <int Q>
int check() {
    constexpr int R = Q >= 64 ? Q / 64 : 1;
    float* d;
    (void)hipMalloc(&d, 64 * R * sizeof(float));
    hipLaunchKernelGGL(k<Q>, dim3(1), dim3(64), 0, 0, d);
    float h[64 * 2];
    (void)hipMemcpy(h, d, 64 * R * sizeof(float), hipMemcpyDeviceToHost);
    (void)hipFree(d);
    double lanesum = 0;
    for (int l = 0; l < 64; ++l) lanesum += l % 7;
    int bad = 0;
    for (int l = 0; l < 64; ++l)
        for (int k2 = 0; k2 < R; ++k2) {
            int q;
            if (Q >= 64) q = k2 + (Q / 64) * l;
            else {
                q = 0; int half = Q / 2;
                for (int s = 0; s < 6 && half >= 1; ++s, half >>= 1) q += ((l >> (5 - s)) & 1) * half;
            }
            const double want = 64.0 * (q + 1) * 100 + lanesum;
            if (h[l * R + k2] != want) { if (bad < 5) printf("Q=%d lane %d reg %d: got %f want %f\n", Q, l, k2, h[l * R + k2], want); ++bad; }
        }
    printf("Q=%d %s\n", Q, bad ? "FAIL" : "ok");
    return bad;
}

int main() { return (check<16>() + check<32>() + check<64>() + check<128>()) ? 1 : 0; }
