// Test program (tests/test_kernels_gpu.py): LDS-DMA row gather (__builtin_amdgcn_global_load_lds,
// 16 B per lane) as the forward compositor stages a group's language rows: one wave-instruction
// writes 64 x 16 B contiguously from base + 16 * lane, each lane's source address its own, so
// 8 lanes per 128-byte row fetch 8 rows per instruction in any row order.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__global__ void k_gather(const float* __restrict__ rows, const unsigned* __restrict__ ids, float* __restrict__ out) {
    __shared__ __attribute__((aligned(16))) float s_rows[32 * 32];
    const int lane = threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int e = 8 * i + (lane >> 3), c = lane & 7;
        const float* src = rows + (size_t)ids[e] * 32 + 4 * c;
        __builtin_amdgcn_global_load_lds(src, s_rows + 256 * i, 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x0F70 & ~0x0F70);   // vmcnt(0) expcnt(0) lgkmcnt(0)
    __builtin_amdgcn_wave_barrier();
    for (int k = lane; k < 32 * 32; k += 64) out[k] = s_rows[k];
}

int main() {
    const int P = 1000;
    std::vector<float> h(P * 32);
    for (int i = 0; i < P * 32; ++i) h[i] = (float)i;
    std::vector<unsigned> ids(32);
    for (int e = 0; e < 32; ++e) ids[e] = (unsigned)((e * 397 + 11) % P);
    float *d_rows, *d_out;
    unsigned* d_ids;
    (void)hipMalloc(&d_rows, h.size() * 4); (void)hipMalloc(&d_out, 32 * 32 * 4); (void)hipMalloc(&d_ids, 32 * 4);
    (void)hipMemcpy(d_rows, h.data(), h.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(d_ids, ids.data(), 32 * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k_gather, dim3(1), dim3(64), 0, 0, d_rows, d_ids, d_out);
    std::vector<float> o(32 * 32);
    (void)hipMemcpy(o.data(), d_out, o.size() * 4, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int e = 0; e < 32; ++e)
        for (int c = 0; c < 32; ++c)
            if (o[e * 32 + c] != h[ids[e] * 32 + c]) { if (bad < 4) printf("row %d ch %d: %g vs %g\n", e, c, o[e * 32 + c], h[ids[e] * 32 + c]); ++bad; }
    printf("glds row gather: %s\n", bad ? "FAIL" : "ok");
    return bad ? 1 : 0;
}
