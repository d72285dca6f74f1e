// lsr_common.h -- shared device helpers for the gfx950 rasterizer kernels.
//
// The whole library is compiled with -ffp-contract=off and correctly rounded f32 divide/sqrt, so
// the preprocess arithmetic and the compositing decisions (alpha >= 1/255, T >= 1e-4, radius =
// ceil(3 sqrt(lambda))) are reproducible bit for bit on the host; FMAs are written explicitly,
// either where the host does the same fmaf (exp) or where a value is only accumulated.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LSR_TILE_X 16
#define LSR_TILE_Y 16
#define LSR_TILE_PIX 256
#define LSR_WAVE 64

namespace lsr {

// Falloff exp for x <= 0: Cody-Waite reduction + degree-7 Horner in fma, exponent assembled by
// bits.  <= 2 ulp, like CUDA expf; made of correctly rounded operations only (mul, fma, rint) so
// the host oracle reproduces it bit for bit.
__device__ __forceinline__ float expf_repro(float x) {
    if (!(x >= -87.0f)) return 0.0f;
    const float kf = __builtin_rintf(x * 1.44269504088896341f);
    float r = __builtin_fmaf(kf, -0.693145751953125f, x);
    r = __builtin_fmaf(kf, -1.428606765330187045e-06f, r);
    float p = 1.98412698412698413e-04f;
    p = __builtin_fmaf(p, r, 1.38888888888888889e-03f);
    p = __builtin_fmaf(p, r, 8.33333333333333333e-03f);
    p = __builtin_fmaf(p, r, 4.16666666666666667e-02f);
    p = __builtin_fmaf(p, r, 1.66666666666666667e-01f);
    p = __builtin_fmaf(p, r, 0.5f);
    p = __builtin_fmaf(p, r, 1.0f);
    p = __builtin_fmaf(p, r, 1.0f);
    const int k = (int)kf;
    return p * __uint_as_float((uint32_t)(k + 127) << 23);
}

// expf_repro of two values at once: the same correctly rounded operations per component, the
// multiplies and fmas on the packed fp32 pipe (v_pk_mul_f32 / v_pk_fma_f32: two results per
// instruction), so each component is bit-identical to expf_repro.
typedef float lsr_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ lsr_f2 expf_repro2(lsr_f2 x) {
    const lsr_f2 t = x * lsr_f2{1.44269504088896341f, 1.44269504088896341f};
    const lsr_f2 kf = {__builtin_rintf(t.x), __builtin_rintf(t.y)};
    lsr_f2 r = __builtin_elementwise_fma(kf, lsr_f2{-0.693145751953125f, -0.693145751953125f}, x);
    r = __builtin_elementwise_fma(kf, lsr_f2{-1.428606765330187045e-06f, -1.428606765330187045e-06f}, r);
    lsr_f2 p = {1.98412698412698413e-04f, 1.98412698412698413e-04f};
    p = __builtin_elementwise_fma(p, r, lsr_f2{1.38888888888888889e-03f, 1.38888888888888889e-03f});
    p = __builtin_elementwise_fma(p, r, lsr_f2{8.33333333333333333e-03f, 8.33333333333333333e-03f});
    p = __builtin_elementwise_fma(p, r, lsr_f2{4.16666666666666667e-02f, 4.16666666666666667e-02f});
    p = __builtin_elementwise_fma(p, r, lsr_f2{1.66666666666666667e-01f, 1.66666666666666667e-01f});
    p = __builtin_elementwise_fma(p, r, lsr_f2{0.5f, 0.5f});
    p = __builtin_elementwise_fma(p, r, lsr_f2{1.0f, 1.0f});
    p = __builtin_elementwise_fma(p, r, lsr_f2{1.0f, 1.0f});
    const lsr_f2 sc = {__uint_as_float((uint32_t)((int)kf.x + 127) << 23),
                       __uint_as_float((uint32_t)((int)kf.y + 127) << 23)};
    const lsr_f2 e = p * sc;
    return lsr_f2{x.x >= -87.0f ? e.x : 0.0f, x.y >= -87.0f ? e.y : 0.0f};
}

// Power threshold below which alpha = min(0.99, o exp(power)) < 1/255 for certain (margin 1e-3 in
// the exponent, far above float error): lets a lane skip exp without changing any decision.
__device__ __forceinline__ float skip_power(float opacity) {
    return opacity > 0.0f ? -__logf(255.0f * opacity) - 1e-3f : __builtin_inff();
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

__device__ __forceinline__ uint64_t lanemask_lt() {
    const uint32_t lane = __lane_id();
    return lane == 0 ? 0ull : (~0ull >> (64 - lane));
}

// ---- cross-lane movement without LDS ---------------------------------------------------------
// DPP controls (GFX9 encoding): quad_perm, row_mirror, row_half_mirror.
constexpr int DPP_XOR1 = 0xB1;        // quad_perm [1,0,3,2]
constexpr int DPP_XOR2 = 0x4E;        // quad_perm [2,3,0,1]
constexpr int DPP_HALF_MIRROR = 0x141;
constexpr int DPP_MIRROR = 0x140;

template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}

// v_permlane32_swap: lanes 32-63 of a <-> lanes 0-31 of b.
__device__ __forceinline__ void swap32(float& a, float& b) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}
// v_permlane16_swap: odd rows (16 lanes) of a <-> even rows of b.
__device__ __forceinline__ void swap16(float& a, float& b) {
    auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
    a = __uint_as_float(r[0]);
    b = __uint_as_float(r[1]);
}

// Transpose-reduce (reduce-scatter) of Q per-lane values over the 64 lanes of a wave.
// Six halving steps: lanes (l, l^32) via permlane32_swap, (l, l^16) via permlane16_swap, then
// inside each row of 16 the DPP involutions mirror, half-mirror, xor2, xor1.  Each step keeps
// half of the values and adds the partner's copy of them, so Q values cost ~Q swaps/adds instead
// of 6 Q.  Afterwards register k < max(1, Q/64) of lane l holds the wave total of quantity
//   q = k + (Q/64) l                    when Q >= 64,
//   q = (Q/2) b5 + (Q/4) b4 + ...       (the first log2 Q lane bits, from bit 5 down) when Q < 64.
// Values are destroyed.  Q must be a power of two >= 2.
template <int Q>
__device__ __forceinline__ void wave_transpose_reduce(float (&v)[Q]) {
    const int lane = __lane_id();
    const int r = lane & 15;
    int n = Q;
    // step 1: pairs across halves of the wave
    if constexpr (Q >= 2) {
#pragma unroll
        for (int k = 0; k < Q / 2; ++k) {
            float a = v[k], b = v[k + Q / 2];
            swap32(a, b);
            v[k] = a + b;
        }
        n = Q / 2;
    }
    // step 2: pairs across row pairs
    if constexpr (Q >= 4) {
#pragma unroll
        for (int k = 0; k < Q / 4; ++k) {
            float a = v[k], b = v[k + Q / 4];
            swap16(a, b);
            v[k] = a + b;
        }
        n = Q / 4;
    } else {
        float a = v[0], b = v[0];
        swap16(a, b);
        v[0] = a + b;
    }
    // steps 3-6 inside each row: keep the first half on the low side of the pairing
#define LSR_DPP_STEP(CTRL, DIV, HIGH)                                              \
    if constexpr (Q >= 4 * DIV) {                                                  \
        _Pragma("unroll") for (int k = 0; k < Q / (4 * DIV); ++k) {                \
            const float a = v[k], b = v[k + Q / (4 * DIV)];                        \
            const float s1 = a + dpp<CTRL>(a), s2 = b + dpp<CTRL>(b);              \
            v[k] = (HIGH) ? s2 : s1;                                               \
        }                                                                          \
    } else {                                                                       \
        v[0] = v[0] + dpp<CTRL>(v[0]);                                             \
    }
    LSR_DPP_STEP(DPP_MIRROR, 2, r >= 8)
    LSR_DPP_STEP(DPP_HALF_MIRROR, 4, (r & 7) >= 4)
    LSR_DPP_STEP(DPP_XOR2, 8, (r & 2) != 0)
    LSR_DPP_STEP(DPP_XOR1, 16, (r & 1) != 0)
#undef LSR_DPP_STEP
    (void)n;
}

// Quantity held in register 0 of `lane` after wave_transpose_reduce<Q> (Q <= 64).
template <int Q>
__device__ __forceinline__ int transpose_reduce_slot(int lane) {
    int q = 0;
    int half = Q / 2;
    const int bits[6] = {(lane >> 5) & 1, (lane >> 4) & 1, (lane >> 3) & 1, (lane >> 2) & 1, (lane >> 1) & 1, lane & 1};
#pragma unroll
    for (int s = 0; s < 6; ++s) {
        if (half >= 1) {
            q += bits[s] * half;
            half >>= 1;
        }
    }
    return q;
}

// ---- entry compaction for the per-quadrant compositor waves (render_fwd_wave / render_bwd_wave)
__device__ __forceinline__ void wave_lds_sync() {
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's LDS writes have landed
    __builtin_amdgcn_wave_barrier();
}

// May the splat (xy, conic+opacity) pass the per-pixel prefilter power >= skip_power(o) at some
// pixel centre of the box [x0, x1] x [y0, y1]?  min over the box of q(d) = a dx^2 + 2b dx dy +
// c dy^2 (power = -q/2), d = xy - p, taken on the box edges when 0 is outside.  The box
// endpoints are computed like the per-pixel dx, dy, so every pixel's (dx, dy) lies inside it; the
// margin covers the float evaluation of q at the pixels (terms up to M).  False only when the
// compositor would skip the splat at every pixel of the box.
__device__ __forceinline__ bool quad_may_touch(float2 xy, float4 co, float x0, float x1, float y0, float y1) {
    const float thr = skip_power(co.w);
    const float dxl = xy.x - x1, dxh = xy.x - x0, dyl = xy.y - y1, dyh = xy.y - y0;
    const float a = co.x, b = co.y, c = co.z;
    float mq = 0.0f;
    if (!(dxl <= 0.0f && dxh >= 0.0f && dyl <= 0.0f && dyh >= 0.0f)) {
        const float tyl = fminf(fmaxf(-b * dxl / c, dyl), dyh), tyh = fminf(fmaxf(-b * dxh / c, dyl), dyh);
        const float txl = fminf(fmaxf(-b * dyl / a, dxl), dxh), txh = fminf(fmaxf(-b * dyh / a, dxl), dxh);
        const float q1 = a * dxl * dxl + 2.0f * b * dxl * tyl + c * tyl * tyl;
        const float q2 = a * dxh * dxh + 2.0f * b * dxh * tyh + c * tyh * tyh;
        const float q3 = a * txl * txl + 2.0f * b * txl * dyl + c * dyl * dyl;
        const float q4 = a * txh * txh + 2.0f * b * txh * dyh + c * dyh * dyh;
        mq = fminf(fminf(q1, q2), fminf(q3, q4));
    }
    const float mx = fmaxf(-dxl, dxh), my = fmaxf(-dyl, dyh);
    const float M = a * mx * mx + c * my * my + 2.0f * fabsf(b) * mx * my;
    return mq <= -2.0f * thr + 1e-5f * M + 1e-4f;
}

}  // namespace lsr
