// Test program (tests/test_kernels_gpu.py): exact-integer checks of the helpers in
// 4dlangsplat_amd/csrc/lsr_mfma.h used by the compositor backward (render_bwd_wave.hip):
//   1. v_mfma_f32_16x16x32_bf16 lane maps (A, B, D as documented in lsr_mfma.h)
//   2. transpose_lane_groups (4 x 4 transpose across 16-lane groups)
//   3. ds_read_tr16 (4 x 16 block, lane i receives column i)
#include <hip/hip_runtime.h>
#include <cstdio>
#include "../../4dlangsplat_amd/csrc/lsr_mfma.h"
using namespace lsr;

__global__ void k_mfma(const float* A, const float* B, float* D) {   // A [16][32], B [32][16], D [16][16]
    const int l = threadIdx.x, r = l & 15, g = l >> 4;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)A[r * 32 + 8 * g + j];
        b[j] = (__bf16)B[(8 * g + j) * 16 + r];
    }
    f32x4 acc = {};
    acc = LSR_MFMA16(a, b, acc);
    for (int i = 0; i < 4; ++i) D[(4 * g + i) * 16 + r] = acc[i];
}

__global__ void k_transpose(float* out) {   // out [64][4]
    const int l = threadIdx.x;
    float x[4];
    for (int p = 0; p < 4; ++p) x[p] = (float)(100 * p + l);
    transpose_lane_groups(x);
    for (int p = 0; p < 4; ++p) out[l * 4 + p] = x[p];
}

__global__ void k_tr(float* out) {          // out [64][4]
    constexpr int PITCH = 20;
    __shared__ __attribute__((aligned(16))) __bf16 w[16 * PITCH];
    const int l = threadIdx.x, g = l >> 4, i = l & 15;
    for (int e = l; e < 16 * PITCH; e += 64) w[e] = (__bf16)(float)((e / PITCH) * 16 + (e % PITCH));
    __syncthreads();
    const bf16x4 v = ds_read_tr16(w + (4 * g + (i >> 2)) * PITCH + 4 * (i & 3));
    for (int j = 0; j < 4; ++j) out[l * 4 + j] = (float)v[j];
}

int main() {
    int bad = 0;
    {
        float hA[16 * 32], hB[32 * 16], hD[16 * 16], ref[16 * 16];
        for (int i = 0; i < 16; ++i) for (int k = 0; k < 32; ++k) hA[i * 32 + k] = (float)((i * 3 + k * 7) % 11 - 5);
        for (int k = 0; k < 32; ++k) for (int j = 0; j < 16; ++j) hB[k * 16 + j] = (float)((k * 5 + j * 2 + k * j) % 13 - 6);
        for (int i = 0; i < 16; ++i) for (int j = 0; j < 16; ++j) { float s = 0; for (int k = 0; k < 32; ++k) s += hA[i * 32 + k] * hB[k * 16 + j]; ref[i * 16 + j] = s; }
        float *dA, *dB, *dD;
        (void)hipMalloc(&dA, sizeof hA); (void)hipMalloc(&dB, sizeof hB); (void)hipMalloc(&dD, sizeof hD);
        (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_mfma, dim3(1), dim3(64), 0, 0, dA, dB, dD);
        (void)hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
        int b = 0;
        for (int i = 0; i < 256; ++i) if (hD[i] != ref[i]) { if (b < 5) printf("D[%d][%d] = %f want %f\n", i / 16, i % 16, hD[i], ref[i]); ++b; }
        printf("mfma 16x16x32 bf16 layout %s\n", b ? "FAIL" : "ok");
        bad += b;
    }
    float* d;
    float h[256];
    (void)hipMalloc(&d, sizeof h);
    {
        hipLaunchKernelGGL(k_transpose, dim3(1), dim3(64), 0, 0, d);
        (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        int b = 0;
        for (int l = 0; l < 64; ++l) for (int p = 0; p < 4; ++p) {
            const float want = (float)(100 * (l >> 4) + 16 * p + (l & 15));
            if (h[l * 4 + p] != want) { if (b < 5) printf("lane %d x[%d] = %f want %f\n", l, p, h[l * 4 + p], want); ++b; }
        }
        printf("transpose_lane_groups %s\n", b ? "FAIL" : "ok");
        bad += b;
    }
    {
        hipLaunchKernelGGL(k_tr, dim3(1), dim3(64), 0, 0, d);
        (void)hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
        int b = 0;
        for (int l = 0; l < 64; ++l) for (int j = 0; j < 4; ++j) {
            const float want = (float)((4 * (l >> 4) + j) * 16 + (l & 15));
            if (h[l * 4 + j] != want) { if (b < 5) printf("lane %d v[%d] = %f want %f\n", l, j, h[l * 4 + j], want); ++b; }
        }
        printf("ds_read_tr16 %s\n", b ? "FAIL" : "ok");
        bad += b;
    }
    return bad ? 1 : 0;
}
