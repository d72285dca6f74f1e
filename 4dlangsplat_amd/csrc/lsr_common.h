// lsr_common.h -- shared device helpers for the gfx950 rasterizer kernels.
//
// The whole library is compiled with -ffp-contract=off and correctly rounded f32 divide/sqrt, so
// the preprocess arithmetic and the compositing decisions (alpha >= 1/255, T >= 1e-4, radius =
// ceil(3 sqrt(lambda))) are reproducible bit for bit on the host; FMAs are written explicitly only
// where a value is accumulated (channel sums), never where it feeds a comparison.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LSR_TILE_X 16
#define LSR_TILE_Y 16
#define LSR_TILE_PIX 256
#define LSR_WAVE 64

namespace lsr {

// Falloff exp for x <= 0: Cody-Waite reduction + degree-7 Horner, exponent assembled by bits.
// <= 2 ulp, like CUDA expf; written with IEEE +,-,*, rint only so that it is reproducible.
__device__ __forceinline__ float expf_repro(float x) {
    if (!(x >= -87.0f)) return 0.0f;
    const float kf = __builtin_rintf(x * 1.44269504088896341f);
    float r = x - kf * 0.693145751953125f;
    r = r - kf * 1.428606765330187045e-06f;
    float p = 1.98412698412698413e-04f;
    p = p * r + 1.38888888888888889e-03f;
    p = p * r + 8.33333333333333333e-03f;
    p = p * r + 4.16666666666666667e-02f;
    p = p * r + 1.66666666666666667e-01f;
    p = p * r + 0.5f;
    p = p * r + 1.0f;
    p = p * r + 1.0f;
    const int k = (int)kf;
    return p * __uint_as_float((uint32_t)(k + 127) << 23);
}

__device__ __forceinline__ float3 xform4x3(const float* __restrict__ m, float3 p) {
    return make_float3(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                       m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14]);
}
__device__ __forceinline__ float4 xform4x4(const float* __restrict__ m, float3 p) {
    return make_float4(m[0] * p.x + m[4] * p.y + m[8] * p.z + m[12],
                       m[1] * p.x + m[5] * p.y + m[9] * p.z + m[13],
                       m[2] * p.x + m[6] * p.y + m[10] * p.z + m[14],
                       m[3] * p.x + m[7] * p.y + m[11] * p.z + m[15]);
}

__device__ __forceinline__ float ndc2pix(float v, int S) { return ((v + 1.0f) * (float)S - 1.0f) * 0.5f; }

// Tile rectangle [rmin, rmax) touched by a splat of integer radius r centred at p (16x16 tiles).
__device__ __forceinline__ void tile_rect(float2 p, int r, int gx, int gy, int2& rmin, int2& rmax) {
    rmin.x = min(gx, max(0, (int)((p.x - (float)r) / (float)LSR_TILE_X)));
    rmin.y = min(gy, max(0, (int)((p.y - (float)r) / (float)LSR_TILE_Y)));
    rmax.x = min(gx, max(0, (int)((p.x + (float)r + (float)(LSR_TILE_X - 1)) / (float)LSR_TILE_X)));
    rmax.y = min(gy, max(0, (int)((p.y + (float)r + (float)(LSR_TILE_Y - 1)) / (float)LSR_TILE_Y)));
}

// Wave-wide sum, result valid in every lane (DPP rows, then the four row sums via readlane).
__device__ __forceinline__ float wave_sum(float v) {
    v += __shfl_xor(v, 1);
    v += __shfl_xor(v, 2);
    v += __shfl_xor(v, 4);
    v += __shfl_xor(v, 8);
    v += __shfl_xor(v, 16);
    v += __shfl_xor(v, 32);
    return v;
}

__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = __lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

}  // namespace lsr
