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

// Falloff exp for x <= 0: the argument clamped at -87 (exp(-87) ~ 1.6e-38: every alpha built
// from it is far below 1/255), k = rint(x log2 e) as fma(x, log2 e, 1.5 2^23) - 1.5 2^23 (one
// rounding of the exact product: the nearest integer), two-constant Cody-Waite reduction, a
// degree-5 polynomial 1 + r (1 + r (c2 + r (c3 + r (c4 + r c5)))) minimax in relative error on
// [-ln2/2, ln2/2] (1.03e-7 before rounding; tools/exp_minimax.py: LP fit, float coefficients) in
// Horner fma, and 2^k assembled from the low bits of that fma's result (bits(y) << 23 + 127 << 23).
// <= 2.16 ulp above -87 (the degree-6 polynomial it replaced: 1.02 with one fma more and an
// unfused rounding step; CUDA's expf: 2 ulp); made of correctly rounded operations only (max,
// mul, add, fma), so the host oracle (orc_exp) reproduces it bit for bit.
#define LSR_EXP_MAGIC 12582912.0f
#define LSR_EXP_C5 0.008314719423651695f
#define LSR_EXP_C4 0.041890207678079605f
#define LSR_EXP_C3 0.16667090356349945f
#define LSR_EXP_C2 0.499992311000824f
__device__ __forceinline__ float expf_repro(float x) {
    x = fmaxf(x, -87.0f);
    const float y = __builtin_fmaf(x, 1.44269504088896341f, LSR_EXP_MAGIC);
    const float kf = y - LSR_EXP_MAGIC;
    float r = __builtin_fmaf(kf, -0.693145751953125f, x);
    r = __builtin_fmaf(kf, -1.428606765330187045e-06f, r);
    float p = LSR_EXP_C5;
    p = __builtin_fmaf(p, r, LSR_EXP_C4);
    p = __builtin_fmaf(p, r, LSR_EXP_C3);
    p = __builtin_fmaf(p, r, LSR_EXP_C2);
    p = __builtin_fmaf(p, r, 1.0f);
    p = __builtin_fmaf(p, r, 1.0f);
    return p * __uint_as_float((__float_as_uint(y) << 23) + 0x3F800000u);
}

// expf_repro of two values at once: the same correctly rounded operations per component, the
// multiplies, adds and fmas on the packed fp32 pipe (v_pk_mul_f32 / v_pk_add_f32 / v_pk_fma_f32:
// two results per instruction), so each component is bit-identical to expf_repro.
typedef float lsr_f2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ lsr_f2 expf_repro2(lsr_f2 x) {
    x = lsr_f2{fmaxf(x.x, -87.0f), fmaxf(x.y, -87.0f)};
    const lsr_f2 y = __builtin_elementwise_fma(x, lsr_f2{1.44269504088896341f, 1.44269504088896341f},
                                               lsr_f2{LSR_EXP_MAGIC, LSR_EXP_MAGIC});
    const lsr_f2 kf = y - lsr_f2{LSR_EXP_MAGIC, LSR_EXP_MAGIC};
    lsr_f2 r = __builtin_elementwise_fma(kf, lsr_f2{-0.693145751953125f, -0.693145751953125f}, x);
    r = __builtin_elementwise_fma(kf, lsr_f2{-1.428606765330187045e-06f, -1.428606765330187045e-06f}, r);
    lsr_f2 p = {LSR_EXP_C5, LSR_EXP_C5};
    p = __builtin_elementwise_fma(p, r, lsr_f2{LSR_EXP_C4, LSR_EXP_C4});
    p = __builtin_elementwise_fma(p, r, lsr_f2{LSR_EXP_C3, LSR_EXP_C3});
    p = __builtin_elementwise_fma(p, r, lsr_f2{LSR_EXP_C2, LSR_EXP_C2});
    p = __builtin_elementwise_fma(p, r, lsr_f2{1.0f, 1.0f});
    p = __builtin_elementwise_fma(p, r, lsr_f2{1.0f, 1.0f});
    const lsr_f2 sc = {__uint_as_float((__float_as_uint(y.x) << 23) + 0x3F800000u),
                       __uint_as_float((__float_as_uint(y.y) << 23) + 0x3F800000u)};
    return p * sc;
}

// Gaussian falloff exponent at d = (dx, dy) = centre - pixel from the STAGED conic
// (A, B, C) = (-a/2, -b, -c/2) of the conic (a, b, c) (exact scalings):
//   power = -(a dx^2 + c dy^2)/2 - b dx dy = dx (A dx + B dy) + (C dy) dy
// in five correctly rounded operations, two of them fma; the host oracle (orc_power) evaluates
// the same sequence, so the contributor decisions stay bit-identical.
__device__ __forceinline__ float gauss_power(float A, float B, float C, float dx, float dy) {
    return __builtin_fmaf(dx, __builtin_fmaf(A, dx, B * dy), (C * dy) * dy);
}
__device__ __forceinline__ lsr_f2 gauss_power2(lsr_f2 A, lsr_f2 B, lsr_f2 C, lsr_f2 dx, lsr_f2 dy) {
    return __builtin_elementwise_fma(dx, __builtin_elementwise_fma(A, dx, B * dy), (C * dy) * dy);
}
__device__ __forceinline__ float4 stage_conic(float4 co) {   // (a, b, c, o) -> (-a/2, -b, -c/2, o)
    return make_float4(-0.5f * co.x, -co.y, -0.5f * co.z, co.w);
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

// &base[idx] as a uniform base + a 32-bit byte offset (idx * sizeof(T) < 2^32, checked on the
// host): the compiler can use the SGPR-base + VGPR-offset addressing forms instead of 64-bit
// address pairs in VGPRs (two registers and a 64-bit add per gather).
template <typename T>
__device__ __forceinline__ T* at32(T* base, uint32_t idx) {
    return reinterpret_cast<T*>(reinterpret_cast<char*>(base) + idx * (uint32_t)sizeof(T));
}
template <typename T>
__device__ __forceinline__ const T* at32(const T* base, uint32_t idx) {
    return reinterpret_cast<const T*>(reinterpret_cast<const char*>(base) + idx * (uint32_t)sizeof(T));
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

// Quadrant masks for the binning (k_emit): which 8x8 quadrants of tile (tx, ty) the splat may
// reach, for every instance.  Separable: per quadrant-row band the x-extent of the region
// R = {d : q(d) <= Q} (Q = -2 skip_power(o) plus a float margin) is computed in closed form, and
// a quadrant is kept iff its dx range meets it.  For a fixed dy, R's slice is
// dx in (-b dy -+ sqrt(a Q - det dy^2)) / a; over a dy band the minimum of the left end is at the
// ellipse's leftmost point (dy_L = b hx / c) when the band holds it, else at a band end (the left
// end is convex in dy), and symmetrically on the right.  In real arithmetic this is exactly the
// box test of quad_may_touch; in float, Q carries the same kind of margin (doubled) and the
// extents are widened by 1e-4 hx + 1e-3 px, so a quadrant where some pixel passes the
// compositors' prefilter is never dropped (tests/test_parity_gpu.py checks the bits).  The bits
// only need to be conservative: the hardware sqrt / rcp (1 ulp) sit far inside those margins.
struct EmitSplat {
    float X, Y;        // centre (pixels)
    float a, b;        // conic x^2 and xy terms (q = a dx^2 + 2 b dx dy + c dy^2)
    float inv_a, det;  // 1 / a, a c - b^2
    float Q, hx, hy;   // level, x / y half extents of R (hy < 0: R empty)
    float dyl, dyr;    // dy of R's leftmost / rightmost points
};
__device__ __forceinline__ EmitSplat emit_splat(float2 xy, float4 co) {
    EmitSplat s;
    s.X = xy.x; s.Y = xy.y;
    s.a = co.x; s.b = co.y;
    const float c = co.z;
    s.det = co.x * c - co.y * co.y;
    s.inv_a = __builtin_amdgcn_rcpf(co.x);
    const float Q0 = -2.0f * skip_power(co.w);
    float hx = 0.0f, hy = -1.0f;
    s.Q = Q0;
    if (Q0 > 0.0f && s.det > 0.0f) {
        const float rdet = __builtin_amdgcn_rcpf(s.det);
        hx = __builtin_amdgcn_sqrtf(Q0 * c * rdet);
        hy = __builtin_amdgcn_sqrtf(Q0 * co.x * rdet);
        const float M = co.x * hx * hx + c * hy * hy + 2.0f * fabsf(co.y) * hx * hy;
        s.Q = Q0 + 2e-5f * M + 2e-4f;
        hx = __builtin_amdgcn_sqrtf(s.Q * c * rdet);
        hy = __builtin_amdgcn_sqrtf(s.Q * co.x * rdet);
    }
    s.hx = hx; s.hy = hy;
    s.dyl = co.y * hx * __builtin_amdgcn_rcpf(c);
    s.dyr = -s.dyl;
    return s;
}
// R's dx extent [xmin, xmax] over the pixel rows [yb0, min(yb0 + 7, H - 1)] of one 8-row band
// (ok: the band is inside the image and meets R); shared by every tile column of a tile row
__device__ __forceinline__ void emit_band(const EmitSplat& s, int yb0, int H, float ex, bool& ok, float& xmin,
                                          float& xmax) {
    const int yb1 = min(yb0 + 7, H - 1);
    // dy = Y - y over the band's pixel rows, clipped to R's y extent
    const float u0 = fmaxf(s.Y - (float)yb1, -s.hy - ex), u1 = fminf(s.Y - (float)yb0, s.hy + ex);
    const float r0 = __builtin_amdgcn_sqrtf(fmaxf(0.0f, s.a * s.Q - s.det * u0 * u0));
    const float r1 = __builtin_amdgcn_sqrtf(fmaxf(0.0f, s.a * s.Q - s.det * u1 * u1));
    const float l0 = (-s.b * u0 - r0) * s.inv_a, l1 = (-s.b * u1 - r1) * s.inv_a;
    const float g0 = (-s.b * u0 + r0) * s.inv_a, g1 = (-s.b * u1 + r1) * s.inv_a;
    xmin = (s.dyl >= u0 && s.dyl <= u1 ? -s.hx : fminf(l0, l1)) - ex;
    xmax = (s.dyr >= u0 && s.dyr <= u1 ? s.hx : fmaxf(g0, g1)) + ex;
    ok = yb0 < H && u0 <= u1 && s.hy >= 0.0f;
}
// does the band's extent meet the 8 pixel columns from xa (dx = X - x over them)?
__device__ __forceinline__ bool emit_col_hit(const EmitSplat& s, bool band_ok, float xmin, float xmax, int xa, int W) {
    const int xb = min(xa + 7, W - 1);
    return band_ok && xa < W && s.X - (float)xb <= xmax && s.X - (float)xa >= xmin;
}
__device__ __forceinline__ float emit_margin(const EmitSplat& s) { return 1e-4f * s.hx + 1e-3f; }
// mask bit (q = (band) * 2 + (column)) for the four quadrants of the tile at pixel origin (x0, y0)
__device__ __forceinline__ uint32_t emit_quad_mask(const EmitSplat& s, int x0, int y0, int W, int H) {
    const float ex = emit_margin(s);
    uint32_t mask = 0;
#pragma unroll
    for (int band = 0; band < 2; ++band) {
        bool ok;
        float xmin, xmax;
        emit_band(s, y0 + 8 * band, H, ex, ok, xmin, xmax);
#pragma unroll
        for (int col = 0; col < 2; ++col)
            mask |= emit_col_hit(s, ok, xmin, xmax, x0 + 8 * col, W) ? 1u << (band * 2 + col) : 0u;
    }
    return mask;
}

}  // namespace lsr
