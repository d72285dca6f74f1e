// Test program (tests/test_kernels_gpu.py): exact-integer check of the v_mfma_f32_32x32x16_bf16
// operand/result lane maps used by the compositors (render_fwd_mfma_wave.hip / render_bwd_wave.hip):
//   A: lane l holds A[row l&31][k = 8(l>>5) + j], j = 0..7
//   B: lane l holds B[k = 8(l>>5) + j][col l&31]
//   D: lane l, register r holds D[row (r&3) + 8(r>>2) + 4(l>>5)][col l&31]
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__global__ void k(const float* A, const float* B, float* D) {   // A [32][16], B [16][32], D [32][32]
    const int l = threadIdx.x, r = l & 31, h = l >> 5;
    bf16x8 a, b;
    for (int j = 0; j < 8; ++j) {
        a[j] = (__bf16)A[r * 16 + 8 * h + j];
        b[j] = (__bf16)B[(8 * h + j) * 32 + r];
    }
    f32x16 acc = {};
    acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc, 0, 0, 0);
    for (int q = 0; q < 16; ++q) D[((q & 3) + 8 * (q >> 2) + 4 * h) * 32 + r] = acc[q];
}

int main() {
    float hA[32 * 16], hB[16 * 32], hD[32 * 32], ref[32 * 32];
    for (int i = 0; i < 32; ++i) for (int kk = 0; kk < 16; ++kk) hA[i * 16 + kk] = (float)((i * 3 + kk * 7) % 11 - 5);
    for (int kk = 0; kk < 16; ++kk) for (int j = 0; j < 32; ++j) hB[kk * 32 + j] = (float)((kk * 5 + j * 2 + kk * j) % 13 - 6);
    for (int i = 0; i < 32; ++i) for (int j = 0; j < 32; ++j) { float s = 0; for (int kk = 0; kk < 16; ++kk) s += hA[i * 16 + kk] * hB[kk * 32 + j]; ref[i * 32 + j] = s; }
    float *dA, *dB, *dD;
    (void)hipMalloc(&dA, sizeof hA); (void)hipMalloc(&dB, sizeof hB); (void)hipMalloc(&dD, sizeof hD);
    (void)hipMemcpy(dA, hA, sizeof hA, hipMemcpyHostToDevice); (void)hipMemcpy(dB, hB, sizeof hB, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    (void)hipMemcpy(hD, dD, sizeof hD, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int i = 0; i < 32 * 32; ++i) if (hD[i] != ref[i]) { if (bad < 5) printf("D[%d][%d] = %f want %f\n", i / 32, i % 32, hD[i], ref[i]); ++bad; }
    printf("mfma 32x32x16 bf16 layout %s\n", bad ? "FAIL" : "ok");
    return bad ? 1 : 0;
}
