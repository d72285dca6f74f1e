// deform.hip -- the 4D deformation field forward: HexPlane sampling + MLP heads, fused, one block
// per 64 Gaussians (include/lsr_deform.h; reference scene/hexplane.py, scene/deformation.py).
//
// Stage 1 (features): 4 threads per Gaussian, each owning 4 of the 16 channels of every plane.
//   Planes are packed channel-last ([H][W][16], lsr_deform_prepare), so a bilinear tap is one
//   float4 per thread; the 6 planes of a scale multiply, the scales concatenate (32 features).
// Stage 2 (MLP): Y = X W^T on v_mfma_f32_32x32x16_bf16 with fp32 accuracy from a bf16 hi/lo split
//   of both operands (hi*hi + hi*lo + lo*hi).  A comes from the block's activation rows in LDS,
//   B straight from the packed bf16 weights ([N][K] rows = the torch layout), which stay
//   L2-resident (94K weights).  Bias, ReLU and the residual adds of the heads are fused into the
//   epilogues; nothing but the deformed parameters leaves the block.
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

typedef __bf16 dbf16x8 __attribute__((ext_vector_type(8)));
typedef float df32x16 __attribute__((ext_vector_type(16)));
#define DMFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

constexpr int DN = 64;            // Gaussians per block
constexpr int DFEAT = 32;         // 2 scales x 16 channels
constexpr int DWID = 128;         // MLP width
constexpr int DXP = DFEAT + 8;    // LDS row pitch (bf16) of the feature rows
constexpr int DAP = DWID + 8;     // LDS row pitch (bf16) of the hidden rows
constexpr int DW2ROWS = 64;       // output rows of every head's last layer, zero padded
__constant__ int kHeadOut[5] = {3, 3, 4, 1, 48};

__device__ __forceinline__ void dsplit(float x, __bf16& hi, __bf16& lo) {
    hi = (__bf16)x;
    lo = (__bf16)(x - (float)hi);
}

// Y[64 x 32] (+)= X[64 x K] W^T for N tile `nt`: both M tiles (the block's 64 Gaussians) share
// every weight fragment, so a block reads each weight once per layer.
template <int K>
__device__ __forceinline__ void mlp_ntile(df32x16 (&acc)[2], const __bf16* __restrict__ xh, const __bf16* __restrict__ xl,
                                          int xp, int nt, const __bf16* __restrict__ wh, const __bf16* __restrict__ wl) {
    const int lane = threadIdx.x & 63, r = lane & 31, h = lane >> 5;
    // every weight fragment of the tile in flight at once (L2-resident, one round trip)
    dbf16x8 bh[K / 16], bl[K / 16];
#pragma unroll
    for (int ks = 0; ks < K / 16; ++ks) {
        const size_t wo = (size_t)(32 * nt + r) * K + 16 * ks + 8 * h;
        bh[ks] = *reinterpret_cast<const dbf16x8*>(wh + wo);
        bl[ks] = *reinterpret_cast<const dbf16x8*>(wl + wo);
    }
    __builtin_amdgcn_sched_barrier(0);   // keep the loads issued here, ahead of the MFMAs
#pragma unroll
    for (int ks = 0; ks < K / 16; ++ks) {
        const int k0 = 16 * ks + 8 * h;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt) {
            const dbf16x8 ah = *reinterpret_cast<const dbf16x8*>(xh + (32 * mt + r) * xp + k0);
            const dbf16x8 al = *reinterpret_cast<const dbf16x8*>(xl + (32 * mt + r) * xp + k0);
            acc[mt] = DMFMA(ah, bh[ks], acc[mt]);
            acc[mt] = DMFMA(ah, bl[ks], acc[mt]);
            acc[mt] = DMFMA(al, bh[ks], acc[mt]);
        }
    }
}

// epilogue to LDS rows: relu(acc + bias) as bf16 hi/lo, N tile `nt`, both M tiles
__device__ __forceinline__ void store_hidden(const df32x16 (&acc)[2], int nt, const float* __restrict__ bias,
                                             __bf16* __restrict__ yh, __bf16* __restrict__ yl) {
    const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5;
    const int col = 32 * nt + c;
    const float b = bias[col];
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int row = 32 * mt + (q & 3) + 8 * (q >> 2) + 4 * h;
            const float v = fmaxf(acc[mt][q] + b, 0.0f);
            __bf16 hi, lo;
            dsplit(v, hi, lo);
            yh[row * DAP + col] = hi;
            yl[row * DAP + col] = lo;
        }
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) k_deform_fwd(DeformArgs a) {
    __shared__ __attribute__((aligned(16))) __bf16 s_xh[DN * DXP];
    __shared__ __attribute__((aligned(16))) __bf16 s_xl[DN * DXP];
    __shared__ __attribute__((aligned(16))) __bf16 s_ah[DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_al[DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_bh[DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_bl[DN * DAP];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int g0 = blockIdx.x * DN;

    // ---- stage 1: HexPlane features, 4 threads per Gaussian ------------------------------------
    {
        const int gl = tid >> 2, q = tid & 3;
        const int g = min(g0 + gl, a.P - 1);
        float crd[4];
        // normalize_aabb: (p - aabb[0]) * (2 / (aabb[1] - aabb[0])) - 1, aabb = [xyz_max, xyz_min]
#pragma unroll
        for (int c = 0; c < 3; ++c)
            crd[c] = (__builtin_nontemporal_load(a.means3D + 3 * g + c) - a.aabb[c]) * (2.0f / (a.aabb[3 + c] - a.aabb[c])) - 1.0f;
        crd[3] = __builtin_nontemporal_load(a.time + g);
        const int c0s[6] = {0, 0, 0, 1, 1, 2}, c1s[6] = {1, 2, 3, 2, 3, 3};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            float4 prod = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
#pragma unroll
            for (int ci = 0; ci < 6; ++ci) {
                const int pi = 6 * s + ci;
                const int W = a.pw[pi], H = a.ph[pi];
                const float ix = fminf(fmaxf((crd[c0s[ci]] + 1.0f) * 0.5f * (float)(W - 1), 0.0f), (float)(W - 1));
                const float iy = fminf(fmaxf((crd[c1s[ci]] + 1.0f) * 0.5f * (float)(H - 1), 0.0f), (float)(H - 1));
                const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
                const int x1 = min(x0 + 1, W - 1), y1 = min(y0 + 1, H - 1);
                const float fx = ix - (float)x0, fy = iy - (float)y0;
                const float4* pl = reinterpret_cast<const float4*>(a.planes + a.poff[pi]) + q;
                const float4 v00 = pl[(y0 * W + x0) * 4], v01 = pl[(y0 * W + x1) * 4];
                const float4 v10 = pl[(y1 * W + x0) * 4], v11 = pl[(y1 * W + x1) * 4];
                const float w00 = (1.0f - fx) * (1.0f - fy), w01 = fx * (1.0f - fy), w10 = (1.0f - fx) * fy, w11 = fx * fy;
                prod.x *= v00.x * w00 + v01.x * w01 + v10.x * w10 + v11.x * w11;
                prod.y *= v00.y * w00 + v01.y * w01 + v10.y * w10 + v11.y * w11;
                prod.z *= v00.z * w00 + v01.z * w01 + v10.z * w10 + v11.z * w11;
                prod.w *= v00.w * w00 + v01.w * w01 + v10.w * w10 + v11.w * w11;
            }
            const float f[4] = {prod.x, prod.y, prod.z, prod.w};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                __bf16 hi, lo;
                dsplit(f[i], hi, lo);
                s_xh[gl * DXP + 16 * s + 4 * q + i] = hi;
                s_xl[gl * DXP + 16 * s + 4 * q + i] = lo;
            }
        }
    }
    __syncthreads();

    // ---- stage 2: hidden = relu(feat W_f^T + b_f); wave w owns hidden columns 32 w .. 32 w + 31 ----
    {
        df32x16 acc[2] = {df32x16{}, df32x16{}};
        mlp_ntile<DFEAT>(acc, s_xh, s_xl, DXP, wave, a.wf_h, a.wf_l);
        store_hidden(acc, wave, a.b_feat, s_ah, s_al);
    }
    __syncthreads();

    // ---- heads: out = in + (relu(hidden W1^T + b1) W2^T + b2) -------------------------------------
    for (int hd = 0; hd < 5; ++hd) {
        const int nout = kHeadOut[hd];
        const bool owner = wave < (nout + 31) / 32;     // 1 N tile, or 2 for the 48 SH coefficients
        const int col = 32 * wave + (lane & 31), h = lane >> 5;
        // the residual inputs of this wave's outputs, loaded now so the head's first layer hides
        // their latency (streamed once: non-temporal, the weights and planes keep the L2)
        float resid[2][16];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int g = g0 + 32 * mt + (q & 3) + 8 * (q >> 2) + 4 * h;
                resid[mt][q] = (owner && col < nout && g < a.P)
                                   ? __builtin_nontemporal_load(a.in[hd] + (size_t)g * nout + col) : 0.0f;
            }
        {
            df32x16 acc[2] = {df32x16{}, df32x16{}};
            mlp_ntile<DWID>(acc, s_ah, s_al, DAP, wave, a.w1_h + (size_t)hd * DWID * DWID,
                            a.w1_l + (size_t)hd * DWID * DWID);
            store_hidden(acc, wave, a.b1[hd], s_bh, s_bl);
        }
        __syncthreads();
        if (owner) {
            df32x16 acc[2] = {df32x16{}, df32x16{}};
            mlp_ntile<DWID>(acc, s_bh, s_bl, DAP, wave, a.w2_h + (size_t)hd * DW2ROWS * DWID,
                            a.w2_l + (size_t)hd * DW2ROWS * DWID);
            if (col < nout) {
                const float b = a.b2[hd][col];
                float* out = a.out[hd];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int g = g0 + 32 * mt + (q & 3) + 8 * (q >> 2) + 4 * h;
                        if (g < a.P) __builtin_nontemporal_store(resid[mt][q] + (acc[mt][q] + b), out + (size_t)g * nout + col);
                    }
            }
        }
        __syncthreads();
    }
}

void launch_deform_fwd(const DeformArgs& a, hipStream_t st) {
    if (a.P <= 0) return;
    hipLaunchKernelGGL(k_deform_fwd, dim3((a.P + DN - 1) / DN), dim3(256), 0, st, a);
}

// ---- parameter packing ----------------------------------------------------------------------------
// plane [C=16][H][W] (torch) -> [H][W][16]
__global__ void k_pack_plane(const float* __restrict__ src, float* __restrict__ dst, int H, int W) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;   // over H * W * 16 destination floats
    if (i >= H * W * 16) return;
    const int c = i & 15, hw = i >> 4;
    dst[i] = src[(size_t)c * H * W + hw];
}

// fp32 [rows][cols] -> bf16 hi / lo [rows_pad][cols], zero rows past `rows`
__global__ void k_pack_weight(const float* __restrict__ src, __bf16* __restrict__ hi, __bf16* __restrict__ lo,
                              int rows, int rows_pad, int cols) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows_pad * cols) return;
    const float v = (i / cols) < rows ? src[i] : 0.0f;
    __bf16 h, l;
    dsplit(v, h, l);
    hi[i] = h;
    lo[i] = l;
}

void launch_pack_plane(const float* src, float* dst, int H, int W, hipStream_t st) {
    hipLaunchKernelGGL(k_pack_plane, dim3((H * W * 16 + 255) / 256), dim3(256), 0, st, src, dst, H, W);
}
void launch_pack_weight(const float* src, __bf16* hi, __bf16* lo, int rows, int rows_pad, int cols, hipStream_t st) {
    hipLaunchKernelGGL(k_pack_weight, dim3((rows_pad * cols + 255) / 256), dim3(256), 0, st, src, hi, lo, rows,
                       rows_pad, cols);
}

}  // namespace lsr
