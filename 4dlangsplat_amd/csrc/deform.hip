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

// ==== backward ====================================================================================
// Phase A, one block per 64 Gaussians (the forward's tiling): recompute the features X and the
// hidden rows A0 = relu(X Wf^T + bf); per head, Z1 = A0 W1^T + b1 (A1 = relu(Z1) saved), the
// upstream gradient G of the head's outputs through the last layer, dZ1 = (G W2) * [Z1 > 0] (saved),
// and dA0 += dZ1 W1, all on the bf16 hi/lo MFMA of the forward with transposed weight packs; then
// dH0 = dA0 * [H0 > 0] (saved), dX = dH0 Wf, and per Gaussian the HexPlane backward: each plane's
// sample gets dX times the product of the other five planes of its scale, scattered to the 4 bilinear
// taps (float atomics into a channel-last gradient copy: the 16 channels of a tap are one 64-byte
// segment), and the coordinate gradient (zero where border padding clips) goes to d_means3D.
constexpr int DGP = 64 + 8;   // LDS row pitch (bf16) of the upstream-gradient rows (K padded to 64)

__global__ void __launch_bounds__(256) k_deform_bwd_a(DeformBwdArgs b) {
    __shared__ __attribute__((aligned(16))) __bf16 s_xh[DN * DXP];
    __shared__ __attribute__((aligned(16))) __bf16 s_xl[DN * DXP];
    __shared__ __attribute__((aligned(16))) __bf16 s_ah[DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_al[DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_bh[DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_bl[DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_gh[DN * DGP];
    __shared__ __attribute__((aligned(16))) __bf16 s_gl[DN * DGP];
    __shared__ float s_dx[DN][DFEAT + 1];
    __shared__ float s_sdv[4][16][17];   // plane scatter staging, per wave: dv of 16 Gaussians
    __shared__ int s_soff[4][16][4];     //   their 4 tap offsets
    __shared__ float s_sw[4][16][4];     //   and bilinear weights
    const DeformArgs& a = b.f;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int g0 = blockIdx.x * DN;
    const int c0s[6] = {0, 0, 0, 1, 1, 2}, c1s[6] = {1, 2, 3, 2, 3, 3};

    // ---- features (as the forward), saved as fp32 for the feature_out weight gradient ----------
    {
        const int gl = tid >> 2, q = tid & 3;
        const int g = min(g0 + gl, a.P - 1);
        float crd[4];
#pragma unroll
        for (int c = 0; c < 3; ++c)
            crd[c] = (a.means3D[3 * g + c] - a.aabb[c]) * (2.0f / (a.aabb[3 + c] - a.aabb[c])) - 1.0f;
        crd[3] = a.time[g];
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
            if (g0 + gl < a.P)
                *reinterpret_cast<float4*>(b.sX + (size_t)(g0 + gl) * DFEAT + 16 * s + 4 * q) = prod;
        }
    }
    __syncthreads();

    const int col = 32 * wave + (lane & 31), hh = lane >> 5;
    auto row_of = [&](int mt, int q) { return 32 * mt + (q & 3) + 8 * (q >> 2) + 4 * hh; };
    // ---- A0 = relu(X Wf^T + bf), saved -------------------------------------------------------------
    {
        df32x16 acc[2] = {df32x16{}, df32x16{}};
        mlp_ntile<DFEAT>(acc, s_xh, s_xl, DXP, wave, a.wf_h, a.wf_l);
        store_hidden(acc, wave, a.b_feat, s_ah, s_al);
        const float bias = a.b_feat[col];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int g = g0 + row_of(mt, q);
                if (g < a.P) b.sA0[(size_t)g * DWID + col] = fmaxf(acc[mt][q] + bias, 0.0f);
            }
    }
    __syncthreads();

    df32x16 dA0[2] = {df32x16{}, df32x16{}};
    for (int hd = 0; hd < 5; ++hd) {
        const int nout = kHeadOut[hd];
        // upstream gradient rows of this head, K padded to 64
        for (int i = tid; i < DN * 64; i += 256) {
            const int r = i >> 6, k = i & 63, g = g0 + r;
            const float v = (k < nout && g < a.P) ? b.up[hd][(size_t)g * nout + k] : 0.0f;
            __bf16 hi, lo;
            dsplit(v, hi, lo);
            s_gh[r * DGP + k] = hi;
            s_gl[r * DGP + k] = lo;
        }
        // Z1 for this wave's 32 columns (its rows finish before the sync below)
        df32x16 z[2] = {df32x16{}, df32x16{}};
        mlp_ntile<DWID>(z, s_ah, s_al, DAP, wave, a.w1_h + (size_t)hd * DWID * DWID, a.w1_l + (size_t)hd * DWID * DWID);
        {
            const float bias = a.b1[hd][col];
            float* sA1 = b.sA1 + (size_t)hd * a.P * DWID;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    z[mt][q] += bias;
                    const int g = g0 + row_of(mt, q);
                    if (g < a.P) sA1[(size_t)g * DWID + col] = fmaxf(z[mt][q], 0.0f);
                }
        }
        __syncthreads();   // G rows complete
        df32x16 d[2] = {df32x16{}, df32x16{}};
        mlp_ntile<64>(d, s_gh, s_gl, DGP, wave, b.w2t_h + (size_t)hd * DWID * 64, b.w2t_l + (size_t)hd * DWID * 64);
        {
            float* sdZ1 = b.sdZ1 + (size_t)hd * a.P * DWID;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int r = row_of(mt, q), g = g0 + r;
                    const float v = z[mt][q] > 0.0f ? d[mt][q] : 0.0f;
                    __bf16 hi, lo;
                    dsplit(v, hi, lo);
                    s_bh[r * DAP + col] = hi;
                    s_bl[r * DAP + col] = lo;
                    if (g < a.P) sdZ1[(size_t)g * DWID + col] = v;
                }
        }
        __syncthreads();   // dZ1 rows complete
        mlp_ntile<DWID>(dA0, s_bh, s_bl, DAP, wave, b.w1t_h + (size_t)hd * DWID * DWID,
                        b.w1t_l + (size_t)hd * DWID * DWID);
        __syncthreads();   // dZ1 / G rows consumed before the next head rewrites them
    }

    // ---- dH0 = dA0 * [H0 > 0] (saved), then dX = dH0 Wf --------------------------------------------
#pragma unroll
    for (int mt = 0; mt < 2; ++mt)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int r = row_of(mt, q), g = g0 + r;
            const bool on = (float)s_ah[r * DAP + col] + (float)s_al[r * DAP + col] > 0.0f;
            const float v = on ? dA0[mt][q] : 0.0f;
            __bf16 hi, lo;
            dsplit(v, hi, lo);
            s_bh[r * DAP + col] = hi;
            s_bl[r * DAP + col] = lo;
            if (g < a.P) b.sdH0[(size_t)g * DWID + col] = v;
        }
    __syncthreads();
    if (wave == 0) {
        df32x16 acc[2] = {df32x16{}, df32x16{}};
        mlp_ntile<DWID>(acc, s_bh, s_bl, DAP, 0, b.wft_h, b.wft_l);
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int q = 0; q < 16; ++q) s_dx[row_of(mt, q)][lane & 31] = acc[mt][q];
    }
    __syncthreads();

    // ---- HexPlane backward: 4 threads per Gaussian, 4 channels each ----------------------------------
    {
        const int gl = tid >> 2, q = tid & 3;
        const bool ok = g0 + gl < a.P;
        const int g = min(g0 + gl, a.P - 1);
        float crd[4];
#pragma unroll
        for (int c = 0; c < 3; ++c)
            crd[c] = (a.means3D[3 * g + c] - a.aabb[c]) * (2.0f / (a.aabb[3 + c] - a.aabb[c])) - 1.0f;
        crd[3] = a.time[g];
        float dq[4] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
        for (int s = 0; s < 2; ++s) {
            float4 v[6];
#pragma unroll
            for (int ci = 0; ci < 6; ++ci) {   // the six samples of this scale
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
                v[ci] = make_float4(v00.x * w00 + v01.x * w01 + v10.x * w10 + v11.x * w11,
                                    v00.y * w00 + v01.y * w01 + v10.y * w10 + v11.y * w11,
                                    v00.z * w00 + v01.z * w01 + v10.z * w10 + v11.z * w11,
                                    v00.w * w00 + v01.w * w01 + v10.w * w10 + v11.w * w11);
            }
            const float dxv[4] = {s_dx[gl][16 * s + 4 * q], s_dx[gl][16 * s + 4 * q + 1], s_dx[gl][16 * s + 4 * q + 2],
                                  s_dx[gl][16 * s + 4 * q + 3]};
#pragma unroll
            for (int ci = 0; ci < 6; ++ci) {
                float4 oth = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
#pragma unroll
                for (int cj = 0; cj < 6; ++cj)
                    if (cj != ci) {
                        oth.x *= v[cj].x; oth.y *= v[cj].y; oth.z *= v[cj].z; oth.w *= v[cj].w;
                    }
                const float dv[4] = {dxv[0] * oth.x, dxv[1] * oth.y, dxv[2] * oth.z, dxv[3] * oth.w};
                const int pi = 6 * s + ci;
                const int W = a.pw[pi], H = a.ph[pi];
                const float rx = (crd[c0s[ci]] + 1.0f) * 0.5f * (float)(W - 1);
                const float ry = (crd[c1s[ci]] + 1.0f) * 0.5f * (float)(H - 1);
                const float ix = fminf(fmaxf(rx, 0.0f), (float)(W - 1));
                const float iy = fminf(fmaxf(ry, 0.0f), (float)(H - 1));
                const int x0 = (int)floorf(ix), y0 = (int)floorf(iy);
                const int x1 = min(x0 + 1, W - 1), y1 = min(y0 + 1, H - 1);
                const float fx = ix - (float)x0, fy = iy - (float)y0;
                const float4* pl = reinterpret_cast<const float4*>(a.planes + a.poff[pi]) + q;
                const float4 t00 = pl[(y0 * W + x0) * 4], t01 = pl[(y0 * W + x1) * 4];
                const float4 t10 = pl[(y1 * W + x0) * 4], t11 = pl[(y1 * W + x1) * 4];
                const float w00 = (1.0f - fx) * (1.0f - fy), w01 = fx * (1.0f - fy), w10 = (1.0f - fx) * fy, w11 = fx * fy;
                // scatter: stage the wave's 16 Gaussians (16 channels, 4 taps each) in LDS, then one
                // atomic instruction per Gaussian covers its 4 taps x 16 channels = four full
                // 64-byte segments (lane = 16 tap + channel) instead of 16 partial ones; blocks add
                // into one of b.replicas copies of the gradient planes (summed by the unpack), so
                // the few cells every Gaussian of a frame shares (the time planes) are not one hot spot
                {
                    const int wl = gl & 15;
#pragma unroll
                    for (int i = 0; i < 4; ++i) s_sdv[wave][wl][4 * q + i] = ok ? dv[i] : 0.0f;
                    if (q == 0) {
                        s_soff[wave][wl][0] = (y0 * W + x0) * 16; s_soff[wave][wl][1] = (y0 * W + x1) * 16;
                        s_soff[wave][wl][2] = (y1 * W + x0) * 16; s_soff[wave][wl][3] = (y1 * W + x1) * 16;
                        s_sw[wave][wl][0] = w00; s_sw[wave][wl][1] = w01; s_sw[wave][wl][2] = w10; s_sw[wave][wl][3] = w11;
                    }
                    wave_lds_sync();
                    float* gp = b.dplanes + (size_t)(blockIdx.x % b.replicas) * b.plane_stride + a.poff[pi];
                    const int tap = lane >> 4, ch = lane & 15;
#pragma unroll 4
                    for (int j = 0; j < 16; ++j) {
                        const float v = s_sdv[wave][j][ch] * s_sw[wave][j][tap];
#ifndef LSR_ABL_NOSCATTER
                        if (v != 0.0f) atomicAdd(gp + s_soff[wave][j][tap] + ch, v);
#else
                        if (v == 12345.0f) gp[0] = v;   // timing ablation only
#endif
                    }
                    wave_lds_sync();   // staging read before the next plane rewrites it
                }
                const float a00[4] = {t00.x, t00.y, t00.z, t00.w}, a01[4] = {t01.x, t01.y, t01.z, t01.w};
                const float a10[4] = {t10.x, t10.y, t10.z, t10.w}, a11[4] = {t11.x, t11.y, t11.z, t11.w};
                float dix = 0.0f, diy = 0.0f;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    dix += dv[i] * ((a01[i] - a00[i]) * (1.0f - fy) + (a11[i] - a10[i]) * fy);
                    diy += dv[i] * ((a10[i] - a00[i]) * (1.0f - fx) + (a11[i] - a01[i]) * fx);
                }
                if (rx > 0.0f && rx < (float)(W - 1)) dq[c0s[ci]] += dix * 0.5f * (float)(W - 1);
                if (ry > 0.0f && ry < (float)(H - 1)) dq[c1s[ci]] += diy * 0.5f * (float)(H - 1);
            }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            dq[c] += __shfl_xor(dq[c], 1);
            dq[c] += __shfl_xor(dq[c], 2);
        }
        if (ok && q == 0) {
            const size_t gg = (size_t)(g0 + gl);
#pragma unroll
            for (int c = 0; c < 3; ++c)
                b.d_means3D[3 * gg + c] = b.up[0][3 * gg + c] + dq[c] * (2.0f / (a.aabb[3 + c] - a.aabb[c]));
        }
    }
}

void launch_deform_bwd_a(const DeformBwdArgs& a, hipStream_t st) {
    if (a.f.P <= 0) return;
    hipLaunchKernelGGL(k_deform_bwd_a, dim3((a.f.P + DN - 1) / DN), dim3(256), 0, st, a);
}

// Phase B: C[M][N] += sum_g L[g][m] R[g][n] (M, N <= 128), bias[m] += sum_g L[g][m]; split-K over
// blocks of rows_per_block rows (blockIdx.x), one job per blockIdx.y.  The reduction index g is the
// MFMA's K, so both fragments come straight from the row-major operands: lane (r, h) loads
// L[g0 + 8h + j][32 mt + r] for j < 8 (each load instruction reads 2 x 128 contiguous bytes) and
// splits it into bf16 hi / lo in registers; no LDS.  A wave owns a strip of 32x32 output tiles (one
// M tile and every N tile when M = 128, else one N tile and every M tile), accumulates it over the
// block's rows and adds it to C with one atomic per element.
__device__ __forceinline__ void atb_frag(const float* __restrict__ src, int ld, int col, int64_t g, int64_t row1,
                                         dbf16x8& h8, dbf16x8& l8, float& sum) {
    float v[8];
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) v[jj] = (g + jj < row1 && col < ld) ? src[(g + jj) * ld + col] : 0.0f;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) {
        __bf16 hi, lo;
        dsplit(v[jj], hi, lo);
        h8[jj] = hi;
        l8[jj] = lo;
        sum += v[jj];
    }
}

template <bool STRIP_M>   // STRIP_M: wave w owns M tile w and all N tiles (M = 128)
__device__ __forceinline__ void atb_body(const AtbJob& j, int64_t row0, int64_t row1) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
    const int M = j.M, N = j.N, Mt = (M + 31) / 32, Nt = (N + 31) / 32;
    const int ntile = STRIP_M ? Nt : (wave < Nt ? Mt : 0);
    if (ntile == 0) return;
    df32x16 acc[4] = {df32x16{}, df32x16{}, df32x16{}, df32x16{}};
    float bsum = 0.0f, dummy = 0.0f;
    for (int64_t k0 = row0; k0 < row1; k0 += 16) {
        const int64_t g = k0 + 8 * hh;
        dbf16x8 ah[4], al[4], bh[4], bl[4];
        if (STRIP_M) {
            atb_frag(j.L, M, 32 * wave + r, g, row1, ah[0], al[0], bsum);
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (t < ntile) atb_frag(j.R, N, 32 * t + r, g, row1, bh[t], bl[t], dummy);
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t)
                if (t < ntile) atb_frag(j.L, M, 32 * t + r, g, row1, ah[t], al[t], t == wave ? bsum : dummy);
            atb_frag(j.R, N, 32 * wave + r, g, row1, bh[0], bl[0], dummy);
        }
#pragma unroll
        for (int t = 0; t < 4; ++t) {
            if (t >= ntile) break;
            const dbf16x8& xh = STRIP_M ? ah[0] : ah[t];
            const dbf16x8& xl = STRIP_M ? al[0] : al[t];
            const dbf16x8& yh = STRIP_M ? bh[t] : bh[0];
            const dbf16x8& yl = STRIP_M ? bl[t] : bl[0];
            acc[t] = DMFMA(xh, yh, acc[t]);
            acc[t] = DMFMA(xh, yl, acc[t]);
            acc[t] = DMFMA(xl, yh, acc[t]);
        }
    }
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        if (t >= ntile) break;
        const int mt = STRIP_M ? wave : t, nt = STRIP_M ? t : wave;
        const int n = 32 * nt + r;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int m = 32 * mt + (q & 3) + 8 * (q >> 2) + 4 * hh;
            if (m < M && n < N) atomicAdd(j.C + (size_t)m * N + n, acc[t][q]);
        }
    }
    // bias: lanes r and r + 32 hold the two row halves of column 32 mt + r (mt = this wave's M tile)
    if (j.bias) {
        const float tot = bsum + __shfl_xor(bsum, 32);
        const int m = 32 * wave + r;
        if (hh == 0 && m < M && (STRIP_M || wave < Mt)) atomicAdd(j.bias + m, tot);
    }
    (void)dummy;
}

__global__ void __launch_bounds__(256) k_atb(AtbArgs ga) {
    const AtbJob& j = ga.job[blockIdx.y];
    const int64_t row0 = (int64_t)blockIdx.x * ga.rows_per_block;
    const int64_t row1 = min((int64_t)ga.P, row0 + ga.rows_per_block);
    if (row0 >= row1) return;
    if (j.M > 96) atb_body<true>(j, row0, row1);
    else atb_body<false>(j, row0, row1);
}

void launch_atb(const AtbArgs& a, int njobs, hipStream_t st) {
    if (a.P <= 0 || njobs <= 0) return;
    const int nb = (a.P + a.rows_per_block - 1) / a.rows_per_block;
    hipLaunchKernelGGL(k_atb, dim3(nb, njobs), dim3(256), 0, st, a);
}

// packed channel-last gradient [H][W][16] -> torch [16][H][W], added
__global__ void k_unpack_plane_grad(const float* __restrict__ src, float* __restrict__ dst, int H, int W, int replicas,
                                    int64_t stride) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;   // over 16 * H * W destination floats
    if (i >= H * W * 16) return;
    const int hw = i % (H * W), c = i / (H * W);
    float s = 0.0f;
    for (int r = 0; r < replicas; ++r) s += src[(size_t)r * stride + (size_t)hw * 16 + c];
    dst[i] += s;
}

void launch_unpack_plane_grad(const float* src, float* dst, int H, int W, int replicas, int64_t stride,
                              hipStream_t st) {
    hipLaunchKernelGGL(k_unpack_plane_grad, dim3((H * W * 16 + 255) / 256), dim3(256), 0, st, src, dst, H, W,
                       replicas, stride);
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

// fp32 [rows][cols] -> bf16 hi / lo [cols][k_pad], dst[c][r] = src[r][c], zero for r >= rows
__global__ void k_pack_weight_t(const float* __restrict__ src, __bf16* __restrict__ hi, __bf16* __restrict__ lo,
                                int rows, int cols, int k_pad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cols * k_pad) return;
    const int c = i / k_pad, r = i - c * k_pad;
    const float v = r < rows ? src[(size_t)r * cols + c] : 0.0f;
    __bf16 h, l;
    dsplit(v, h, l);
    hi[i] = h;
    lo[i] = l;
}

void launch_pack_weight_t(const float* src, __bf16* hi, __bf16* lo, int rows, int cols, int k_pad, hipStream_t st) {
    hipLaunchKernelGGL(k_pack_weight_t, dim3((cols * k_pad + 255) / 256), dim3(256), 0, st, src, hi, lo, rows, cols,
                       k_pad);
}

void launch_pack_plane(const float* src, float* dst, int H, int W, hipStream_t st) {
    hipLaunchKernelGGL(k_pack_plane, dim3((H * W * 16 + 255) / 256), dim3(256), 0, st, src, dst, H, W);
}
void launch_pack_weight(const float* src, __bf16* hi, __bf16* lo, int rows, int rows_pad, int cols, hipStream_t st) {
    hipLaunchKernelGGL(k_pack_weight, dim3((rows_pad * cols + 255) / 256), dim3(256), 0, st, src, hi, lo, rows,
                       rows_pad, cols);
}

}  // namespace lsr
