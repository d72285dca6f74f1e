// deform.hip -- the 4D deformation field: HexPlane sampling + MLP heads, fused, one block per 64
// Gaussians (include/lsr_deform.h; reference scene/hexplane.py, scene/deformation.py).
//
// Stage 1 (features): 4 threads per Gaussian, each owning 4 of the 16 channels of every plane.
//   Planes are packed channel-last ([H][W][16], lsr_deform_prepare), so a bilinear tap is one
//   float4 per thread; the 6 planes of a scale multiply, the S scales concatenate (16 S features).
// Stage 2 (MLP): Y = X W^T on v_mfma_f32_32x32x16_bf16 with fp32 accuracy from a bf16 hi/lo split
//   of both operands (hi*hi + hi*lo + lo*hi).  A comes from the block's activation rows in LDS,
//   B straight from the packed bf16 weights ([N][K] rows = the torch layout), which stay
//   L2-resident.  feature_out is a chain of max(defor_depth, 1) layers (ReLU between, and before
//   every head: the heads' first module is a ReLU); bias, ReLU and the residual adds of the heads
//   are fused into the epilogues.  The rotation head's quaternion product (apply_rotation) and the
//   discrete language combination (coff head) are per-Gaussian epilogues through LDS.  lang_deform
//   (the time-varying language field) reads only the language rows and the time: its own kernels
//   below, on the same MFMA helpers.
#include "lsr_common.h"
#include "lsr_internal.h"
#include <algorithm>
#include <cstdlib>

namespace lsr {

// Diagnostic build (-DLSR_DEFORM_DIAG): the plane scatter checks every staged tap offset and value
// and counts the bad ones (lsr_debug_deform_diag) instead of adding them.
// Diagnostic build only (-DLSR_DEFORM_STAMPS): wave 0 of every phase-A block sums per-segment
// s_memtime cycles into g_deform_stamps (lsr_debug_deform_stamps; tools/deform_stamps.py).  Shares, not
// times: the stamps cost cycles and constrain the schedule.
#ifdef LSR_DEFORM_STAMPS
__device__ unsigned long long g_deform_stamps[16];
#define DSTAMP(seg)                                                                              \
    do {                                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        unsigned long long t_;                                                                   \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");             \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        if ((seg) >= 0) ds_sum[(seg)] += t_ - ds_prev;                                           \
        ds_prev = t_;                                                                            \
    } while (0)
#else
#define DSTAMP(seg) do {} while (0)
#endif
#ifdef LSR_DEFORM_DIAG
__device__ unsigned long long g_deform_diag[8];
#endif

// LDS poison build (-DLSR_LDS_POISON, build/variants/liblsr_ldspoison.so; tests/test_deform_lds_poison_gpu.py):
// every kernel of this file fills its shared memory with all-ones words (NaN as fp32 and as bf16)
// at block entry, so a read of LDS the block never wrote turns the results into NaN instead of
// silently reusing what an earlier block on the CU left there.
#ifdef LSR_LDS_POISON
__device__ __forceinline__ void lds_poison(void* p, size_t bytes) {
    uint32_t* w = static_cast<uint32_t*>(p);
    for (size_t i = threadIdx.x; i < bytes / 4; i += blockDim.x) w[i] = 0xFFFFFFFFu;
}
#define LDS_POISON(arr) lds_poison(&(arr), sizeof(arr))
#define LDS_POISON_DONE() __syncthreads()
#else
#define LDS_POISON(arr) do {} while (0)
#define LDS_POISON_DONE() do {} while (0)
#endif

typedef __bf16 dbf16x8 __attribute__((ext_vector_type(8)));
typedef float df32x16 __attribute__((ext_vector_type(16)));
#define DMFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)
typedef float df32x4 __attribute__((ext_vector_type(4)));
#define DMFMA16(a, b, c) __builtin_amdgcn_mfma_f32_16x16x32_bf16((a), (b), (c), 0, 0, 0)

constexpr int DN = 64;            // Gaussians per block
constexpr int DWID = 128;         // MLP width
constexpr int DAP = DWID + 8;     // LDS row pitch (bf16) of the hidden rows
constexpr int DLP = 64 + 8;       // LDS row pitch (bf16) of rows of up to 64 entries
// head output widths {3, 3, 4, 1, 48} (pos, scales, rotations, opacity, SH), as arithmetic: no
// constant-memory load (a PC-relative s_getpc_b64 sequence) on the heads' paths

__device__ __forceinline__ void dsplit(float x, __bf16& hi, __bf16& lo) {
    hi = (__bf16)x;
    lo = (__bf16)(x - (float)hi);
}
__device__ __forceinline__ int head_out(const DeformArgs& a, int hd) {
    return hd < 2 ? 3 : hd == 2 ? 4 : hd == 3 ? 1 : hd == 4 ? 48 : a.centers;
}
__device__ __forceinline__ int row_of(int mt, int q, int hh) { return 32 * mt + (q & 3) + 8 * (q >> 2) + 4 * hh; }

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
// the same with K a runtime multiple of 16 in [16, 64] (the lang_deform input width)
__device__ __forceinline__ void mlp_ntile_k(int K, df32x16 (&acc)[2], const __bf16* xh, const __bf16* xl, int xp, int nt,
                                            const __bf16* wh, const __bf16* wl) {
    switch (K) {
        case 16: mlp_ntile<16>(acc, xh, xl, xp, nt, wh, wl); break;
        case 32: mlp_ntile<32>(acc, xh, xl, xp, nt, wh, wl); break;
        case 48: mlp_ntile<48>(acc, xh, xl, xp, nt, wh, wl); break;
        default: mlp_ntile<64>(acc, xh, xl, xp, nt, wh, wl); break;
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
            const int row = row_of(mt, q, h);
            const float v = fmaxf(acc[mt][q] + b, 0.0f);
            __bf16 hi, lo;
            dsplit(v, hi, lo);
            yh[row * DAP + col] = hi;
            yl[row * DAP + col] = lo;
        }
}

// normalised aabb coordinates + time of Gaussian g (normalize_aabb: (p - aabb[0]) * (2 / (aabb[1] -
// aabb[0])) - 1, aabb = [xyz_max, xyz_min])
__device__ __forceinline__ void coords(const DeformArgs& a, int g, float (&crd)[4]) {
#pragma unroll
    for (int c = 0; c < 3; ++c)
        crd[c] = (a.means3D[3 * g + c] - a.aabb[c]) * (2.0f / (a.aabb[3 + c] - a.aabb[c])) - 1.0f;
    crd[3] = a.time[g];
}
// coordinate pair (c0, c1) of plane combo ci: xy, xz, xt, yz, yt, zt.  Functions, not a table: the
// unrolled loops index the coordinate arrays with compile-time constants (a table in constant
// memory would send those arrays to scratch).
__device__ constexpr int kC0(int ci) { return ci < 3 ? 0 : (ci < 5 ? 1 : 2); }
__device__ constexpr int kC1(int ci) { return ci == 0 ? 1 : (ci == 1 || ci == 3) ? 2 : 3; }

struct Tap {
    int x0, x1, y0, y1;
    float fx, fy;
};
// bilinear tap of plane pi at the coordinate pair of combo ci (grid_sample, align_corners, border)
__device__ __forceinline__ Tap tap_of(const DeformArgs& a, int pi, int ci, const float (&crd)[4]) {
    const int W = a.pw[pi], H = a.ph[pi];
    const float ix = fminf(fmaxf((crd[kC0(ci)] + 1.0f) * 0.5f * (float)(W - 1), 0.0f), (float)(W - 1));
    const float iy = fminf(fmaxf((crd[kC1(ci)] + 1.0f) * 0.5f * (float)(H - 1), 0.0f), (float)(H - 1));
    Tap t;
    t.x0 = (int)floorf(ix); t.y0 = (int)floorf(iy);
    t.x1 = min(t.x0 + 1, W - 1); t.y1 = min(t.y0 + 1, H - 1);
    t.fx = ix - (float)t.x0; t.fy = iy - (float)t.y0;
    return t;
}
// Diagnostic builds (tools/deform_slp_bisect.sh): parts of the HexPlane sampling product's arithmetic
// as scalar VALU instructions the SLP vectorizer cannot pair (same IEEE operations, same bits), so a
// build with SLP on differs from the shipped one only there.  LSR_FEAT_SCALAR: all of it;
// LSR_FEAT_SCALAR_W: the bilinear weights; _SUM: the weighted tap sums; _PROD: the six-plane product.
#if defined(LSR_FEAT_SCALAR)
#define LSR_FEAT_SCALAR_W
#define LSR_FEAT_SCALAR_SUM
#define LSR_FEAT_SCALAR_PROD
#endif
#if defined(LSR_FEAT_SCALAR_W) || defined(LSR_FEAT_SCALAR_SUM) || defined(LSR_FEAT_SCALAR_PROD)
__device__ __forceinline__ float smul(float x, float y) { float r; asm volatile("v_mul_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y)); return r; }
__device__ __forceinline__ float sadd(float x, float y) { float r; asm volatile("v_add_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(y)); return r; }
#endif
#ifdef LSR_FEAT_SCALAR_W
#define FW_MUL(x, y) smul((x), (y))
#define FW_SUB1(x) sadd(1.0f, -(x))
#else
#define FW_MUL(x, y) ((x) * (y))
#define FW_SUB1(x) (1.0f - (x))
#endif
#ifdef LSR_FEAT_SCALAR_SUM
#define FS_MUL(x, y) smul((x), (y))
#define FS_ADD(x, y) sadd((x), (y))
#else
#define FS_MUL(x, y) ((x) * (y))
#define FS_ADD(x, y) ((x) + (y))
#endif
#ifdef LSR_FEAT_SCALAR_PROD
#define FP_MUL(x, y) smul((x), (y))
#else
#define FP_MUL(x, y) ((x) * (y))
#endif
__device__ __forceinline__ float4 sample4(const DeformArgs& a, int pi, const Tap& t, int q) {
    const int W = a.pw[pi];
    const float4* pl = reinterpret_cast<const float4*>(a.planes + a.poff[pi]) + q;
    const float4 v00 = pl[(t.y0 * W + t.x0) * 4], v01 = pl[(t.y0 * W + t.x1) * 4];
    const float4 v10 = pl[(t.y1 * W + t.x0) * 4], v11 = pl[(t.y1 * W + t.x1) * 4];
    const float ufx = FW_SUB1(t.fx), ufy = FW_SUB1(t.fy);
#ifdef LSR_FEAT_BCAST_ASM
    // Diagnostic build: the four weights as the broadcast packed products the SLP build forms
    // (v_pk_mul_f32 op_sel:[0,1] op_sel_hi:[0,1]: both halves = A.lo * B.hi), but never in place
    // (early-clobber destinations), everything else left to the vectorizer
    typedef float f2v __attribute__((ext_vector_type(2)));
    const f2v U = {ufx, ufy}, F = {t.fx, t.fy};
    f2v P00, P01, P10, P11;
#if defined(LSR_FEAT_BCAST_NOP_BEFORE)   // A/B: wait states between the operands' producers and the broadcast
#define BC_PRE "s_nop 4\n\t"
#define BC_POST ""
#elif defined(LSR_FEAT_BCAST_NOP_AFTER)  // A/B: wait states between the broadcast and its consumers
#define BC_PRE ""
#define BC_POST "\n\ts_nop 4"
#else
#define BC_PRE ""
#define BC_POST ""
#endif
    asm volatile(BC_PRE "v_pk_mul_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[0,1]" BC_POST : "=&v"(P00) : "v"(U));
    asm volatile(BC_PRE "v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[0,1]" BC_POST : "=&v"(P01) : "v"(F), "v"(U));
    asm volatile(BC_PRE "v_pk_mul_f32 %0, %1, %2 op_sel:[0,1] op_sel_hi:[0,1]" BC_POST : "=&v"(P10) : "v"(U), "v"(F));
    asm volatile(BC_PRE "v_pk_mul_f32 %0, %1, %1 op_sel:[0,1] op_sel_hi:[0,1]" BC_POST : "=&v"(P11) : "v"(F));
    const float w00 = P00.x, w01 = P01.x, w10 = P10.x, w11 = P11.x;
#else
    const float w00 = FW_MUL(ufx, ufy), w01 = FW_MUL(t.fx, ufy), w10 = FW_MUL(ufx, t.fy), w11 = FW_MUL(t.fx, t.fy);
#endif
    auto c = [&](float a0, float a1, float a2, float a3) {   // left to right, as the reference's sum
        return FS_ADD(FS_ADD(FS_ADD(FS_MUL(a0, w00), FS_MUL(a1, w01)), FS_MUL(a2, w10)), FS_MUL(a3, w11));
    };
    return make_float4(c(v00.x, v01.x, v10.x, v11.x), c(v00.y, v01.y, v10.y, v11.y), c(v00.z, v01.z, v10.z, v11.z),
                       c(v00.w, v01.w, v10.w, v11.w));
}

// Stage 1 of both passes: the block's features into LDS rows (bf16 hi/lo, pitch XP), optionally
// saved as fp32 [P, 16 S]
template <int S>
__device__ __forceinline__ void features_to_lds(const DeformArgs& a, int g0, __bf16* xh, __bf16* xl, int xp, float* save) {
    const int tid = threadIdx.x, gl = tid >> 2, q = tid & 3;
    const int g = min(g0 + gl, a.P - 1);
    float crd[4];
    coords(a, g, crd);
#pragma unroll
    for (int s = 0; s < S; ++s) {
        float4 prod = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
#pragma unroll
        for (int ci = 0; ci < 6; ++ci) {
            const int pi = 6 * s + ci;
            const float4 v = sample4(a, pi, tap_of(a, pi, ci, crd), q);
            prod.x = FP_MUL(prod.x, v.x); prod.y = FP_MUL(prod.y, v.y); prod.z = FP_MUL(prod.z, v.z);
            prod.w = FP_MUL(prod.w, v.w);
#ifdef LSR_DEFORM_FEAT_WAIT
            asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
#endif
        }
        const float f[4] = {prod.x, prod.y, prod.z, prod.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            __bf16 hi, lo;
            dsplit(f[i], hi, lo);
            xh[gl * xp + 16 * s + 4 * q + i] = hi;
            xl[gl * xp + 16 * s + 4 * q + i] = lo;
        }
        if (save && g0 + gl < a.P)
            *reinterpret_cast<float4*>(save + (size_t)(g0 + gl) * (16 * S) + 16 * s + 4 * q) = prod;
    }
}

// The quaternion product of batch_quaternion_multiply (utils/graphics_utils.py:121-124)
__device__ __forceinline__ float4 quat_mul(const float4 a, const float4 b) {
    return make_float4(a.x * b.x - a.y * b.y - a.z * b.z - a.w * b.w, a.x * b.y + a.y * b.x + a.z * b.w - a.w * b.z,
                       a.x * b.z - a.y * b.w + a.z * b.x + a.w * b.y, a.x * b.w + a.y * b.z - a.z * b.y + a.w * b.x);
}

// Discrete language combination of one Gaussian (deformation.py:156-163): centres e_c = lang rows
// [c][lang_dim] each normalised (no epsilon), m = sum_c coff_c e_c / |e_c|, out = m / (|m| + 1e-9)
__device__ __forceinline__ void discrete_combine(const DeformArgs& a, int g, const float* coff, float* out) {
    const int C = a.lang_dim, K = a.centers;
    const float* e = a.lang + (size_t)g * a.lang_in;
    float m[32];
#pragma unroll
    for (int j = 0; j < 32; ++j) m[j] = 0.0f;
    for (int c = 0; c < K; ++c) {
        float n2 = 0.0f;
        for (int j = 0; j < C; ++j) n2 += e[c * C + j] * e[c * C + j];
        const float w = coff[c] / sqrtf(n2);
#pragma unroll
        for (int j = 0; j < 32; ++j)
            if (j < C) m[j] += w * e[c * C + j];
    }
    float n2 = 0.0f;
#pragma unroll
    for (int j = 0; j < 32; ++j) n2 += m[j] * m[j];
    const float inv = 1.0f / (sqrtf(n2) + 1e-9f);
#pragma unroll
    for (int j = 0; j < 32; ++j)
        if (j < C) out[(size_t)g * C + j] = m[j] * inv;
}

// Gradient of the rotation head's output under apply_rotation, Gaussian g: out = p / |p|,
// p = q1 (x) q2 with q2 = d_rot; dp = (d - out (out . d)) / |p|; d/dq1_k of sum(p dp) =
// quat_mul(e_k, q2) . dp, likewise q2.  Writes d_rotations (the input's gradient) and the head
// output's gradient (sG_rot, the upstream of the head's backward).
__device__ __forceinline__ void quat_grad(const DeformBwdArgs& b, int g, const float* dr) {
    const float4 q1 = reinterpret_cast<const float4*>(b.f.in[2])[g];
    const float4 q2 = make_float4(dr[0], dr[1], dr[2], dr[3]);
    const float4 p = quat_mul(q1, q2);
    const float inv = 1.0f / sqrtf(p.x * p.x + p.y * p.y + p.z * p.z + p.w * p.w);
    const float4 d = reinterpret_cast<const float4*>(b.up[2])[g];
    const float4 o = make_float4(p.x * inv, p.y * inv, p.z * inv, p.w * inv);
    const float od = o.x * d.x + o.y * d.y + o.z * d.z + o.w * d.w;
    const float4 dp = make_float4((d.x - o.x * od) * inv, (d.y - o.y * od) * inv, (d.z - o.z * od) * inv,
                                  (d.w - o.w * od) * inv);
    float d1[4], d2[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const float4 ek = make_float4(k == 0, k == 1, k == 2, k == 3);
        const float4 u = quat_mul(ek, q2), w = quat_mul(q1, ek);
        d1[k] = u.x * dp.x + u.y * dp.y + u.z * dp.z + u.w * dp.w;
        d2[k] = w.x * dp.x + w.y * dp.y + w.z * dp.z + w.w * dp.w;
    }
    reinterpret_cast<float4*>(b.d_rotations)[g] = make_float4(d1[0], d1[1], d1[2], d1[3]);
    reinterpret_cast<float4*>(b.sG_rot)[g] = make_float4(d2[0], d2[1], d2[2], d2[3]);
}

// Gradient of the discrete combination (deformation.py:156-163), Gaussian g, coff = the head's
// output: dm from out = m / (|m| + eps); dcoff_c = u_c . dm (+ the upstream of coff itself);
// du_c = coff_c dm; de_c = (du_c - u_c (u_c . du_c)) / |e_c|.  m_j and dm_j are recomputed per
// pass (<= 8 terms) instead of held in registers.  Writes d_lang and sG_coff.
__device__ __forceinline__ void discrete_grad(const DeformBwdArgs& b, int g, const float* coff) {
    const DeformArgs& a = b.f;
    const int C = a.lang_dim, K = a.centers;
    const float* e = a.lang + (size_t)g * a.lang_in;
    const float* up = b.up_lang ? b.up_lang + (size_t)g * C : nullptr;
    float w[8], en[8];
    for (int c = 0; c < K; ++c) {
        float n2 = 0.0f;
        for (int j = 0; j < C; ++j) n2 += e[c * C + j] * e[c * C + j];
        en[c] = sqrtf(n2);
        w[c] = coff[c] / en[c];
    }
    auto m_at = [&](int j) {
        float m = 0.0f;
        for (int c = 0; c < K; ++c) m += w[c] * e[c * C + j];
        return m;
    };
    float n2 = 0.0f, md = 0.0f;
    for (int j = 0; j < C; ++j) {
        const float m = m_at(j);
        n2 += m * m;
        md += m * (up ? up[j] : 0.0f);
    }
    const float n = sqrtf(n2), ne = n + 1e-9f, f = md / (n * ne * ne);
    auto dm_at = [&](int j) { return (up ? up[j] : 0.0f) / ne - m_at(j) * f; };
    for (int c = 0; c < K; ++c) {
        float ud = 0.0f;
        for (int j = 0; j < C; ++j) ud += e[c * C + j] / en[c] * dm_at(j);
        b.sG_coff[(size_t)g * K + c] = ud + (b.up_coff ? b.up_coff[(size_t)g * K + c] : 0.0f);
        const float cc = coff[c];   // du_c . u_c = cc (dm . u_c) = cc ud
        for (int j = 0; j < C; ++j)
            b.d_lang[(size_t)g * a.lang_in + c * C + j] = (cc * dm_at(j) - e[c * C + j] / en[c] * (cc * ud)) / en[c];
    }
}

// GRAD = false: the forward.  GRAD = true (backward, apply_rotation / discrete only): the same
// recompute, but only the heads whose output feeds a nonlinear epilogue run, and that epilogue is
// the gradient (quat_grad, discrete_grad) the backward kernel then reads as the head's upstream.
template <int S, bool GRAD>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) k_deform_fwd(const DeformBwdArgs b) {
    const DeformArgs& a = b.f;
    constexpr int F = 16 * S, XP = F + 8;
    static_assert(XP <= DAP, "feature rows live in the second hidden buffer");
    __shared__ __attribute__((aligned(16))) __bf16 s_hh[2][DN * DAP];   // hidden rows, ping-pong
    __shared__ __attribute__((aligned(16))) __bf16 s_hl[2][DN * DAP];
    __shared__ float s_q[DN][9];                                         // per-Gaussian head outputs
    LDS_POISON(s_hh); LDS_POISON(s_hl); LDS_POISON(s_q); LDS_POISON_DONE();
    // the features are read by the first layer only, which writes buffer 0: they use buffer 1 (72 KB
    // of LDS in all: two blocks per CU)
    __bf16* const s_xh = s_hh[1];
    __bf16* const s_xl = s_hl[1];
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int g0 = blockIdx.x * DN;

    features_to_lds<S>(a, g0, s_xh, s_xl, XP, nullptr);
    __syncthreads();

    // ---- feature_out chain: hidden = relu(... relu(feat W_0^T + b_0) ... W_k^T + b_k) ------------
    int cur = 0;
    {
        df32x16 acc[2] = {df32x16{}, df32x16{}};
        mlp_ntile<F>(acc, s_xh, s_xl, XP, wave, a.wf_h[0], a.wf_l[0]);
        store_hidden(acc, wave, a.b_feat[0], s_hh[0], s_hl[0]);
    }
    __syncthreads();
    for (int k = 1; k < a.nlayers; ++k) {
        df32x16 acc[2] = {df32x16{}, df32x16{}};
        mlp_ntile<DWID>(acc, s_hh[cur], s_hl[cur], DAP, wave, a.wf_h[k], a.wf_l[k]);
        store_hidden(acc, wave, a.b_feat[k], s_hh[cur ^ 1], s_hl[cur ^ 1]);
        __syncthreads();
        cur ^= 1;
    }
    const __bf16 *ah = s_hh[cur], *al = s_hl[cur];
    __bf16 *bh = s_hh[cur ^ 1], *bl = s_hl[cur ^ 1];

    // ---- heads: out = in + (relu(hidden W1^T + b1) W2^T + b2) ---------------------------------------
    for (int hd = 0; hd < DEF_HEADS; ++hd) {
        if (!((a.heads >> hd) & 1u)) continue;                       // block-uniform
        const int nout = head_out(a, hd);
        const bool quat = hd == 2 && a.apply_rotation, coff = hd == 5;
        const bool resid_add = !quat && !coff;
        if (GRAD && resid_add) continue;
#ifndef LSR_DEFORM_FWD_W2_WIDE
        if (nout <= 16) {                                            // block-uniform
            // a head of at most 16 outputs (pos, scales, rotations, opacity, coff): its output layer as
            // 16 x 16 x 32 MFMAs, one 16-row tile per wave (the 32-column tile of one wave computed
            // 28-31 zero columns while the other three waved at the barrier)
            const int c16 = lane & 15, g4 = lane >> 4;
            float res16[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int g = g0 + 16 * wave + 4 * g4 + i;
                res16[i] = (resid_add && c16 < nout && g < a.P) ? __builtin_nontemporal_load(a.in[hd] + (size_t)g * nout + c16)
                                                               : 0.0f;
            }
            {
                df32x16 acc[2] = {df32x16{}, df32x16{}};
                mlp_ntile<DWID>(acc, ah, al, DAP, wave, a.w1_h[hd], a.w1_l[hd]);
                store_hidden(acc, wave, a.b1[hd], bh, bl);
            }
            __syncthreads();
            df32x4 o = df32x4{0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
            for (int ks = 0; ks < DWID / 32; ++ks) {
                const int k0 = 32 * ks + 8 * g4;
                const dbf16x8 xh = *reinterpret_cast<const dbf16x8*>(bh + (16 * wave + c16) * DAP + k0);
                const dbf16x8 xl = *reinterpret_cast<const dbf16x8*>(bl + (16 * wave + c16) * DAP + k0);
                const dbf16x8 wh = *reinterpret_cast<const dbf16x8*>(a.w2_h[hd] + (size_t)c16 * DWID + k0);
                const dbf16x8 wl = *reinterpret_cast<const dbf16x8*>(a.w2_l[hd] + (size_t)c16 * DWID + k0);
                o = DMFMA16(xh, wh, o);
                o = DMFMA16(xh, wl, o);
                o = DMFMA16(xl, wh, o);
            }
            if (c16 < nout) {
                const float b2 = a.b2[hd][c16];
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int r = 16 * wave + 4 * g4 + i, g = g0 + r;
                    const float v = o[i] + b2;
                    if (resid_add) {
                        if (g < a.P) __builtin_nontemporal_store(res16[i] + v, a.out[hd] + (size_t)g * nout + c16);
                    } else {
                        s_q[r][c16] = v;
                        if (!GRAD && coff && a.out_coff && g < a.P) a.out_coff[(size_t)g * nout + c16] = v;
                    }
                }
            }
            __syncthreads();   // the hidden rows read (and s_q complete) before they are reused
            if (!resid_add && wave == 0) {                           // one Gaussian per lane
                const int g = g0 + lane;
                if (GRAD && g < a.P) {
                    if (quat) quat_grad(b, g, s_q[lane]);
                    else discrete_grad(b, g, s_q[lane]);
                } else if (g < a.P) {
                    if (quat) {   // rotations = normalize(rotations (x) d_rot)  (deformation.py:135-136)
                        const float4 q1 = reinterpret_cast<const float4*>(a.in[2])[g];
                        const float4 p = quat_mul(q1, make_float4(s_q[lane][0], s_q[lane][1], s_q[lane][2], s_q[lane][3]));
                        const float inv = 1.0f / sqrtf(p.x * p.x + p.y * p.y + p.z * p.z + p.w * p.w);
                        reinterpret_cast<float4*>(a.out[2])[g] = make_float4(p.x * inv, p.y * inv, p.z * inv, p.w * inv);
                    } else {
                        discrete_combine(a, g, s_q[lane], a.out_lang);
                    }
                }
            }
            if (!resid_add) __syncthreads();   // s_q read before the next head's outputs
            continue;
        }
#endif
        const bool owner = wave < (nout + 31) / 32;     // 1 N tile, or 2 for the 48 SH coefficients
        const int col = 32 * wave + (lane & 31), h = lane >> 5;
        // the residual inputs of this wave's outputs, loaded now so the head's first layer hides
        // their latency (streamed once: non-temporal, the weights and planes keep the L2)
        float resid[2][16];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int g = g0 + row_of(mt, q, h);
                resid[mt][q] = (resid_add && owner && col < nout && g < a.P)
                                   ? __builtin_nontemporal_load(a.in[hd] + (size_t)g * nout + col) : 0.0f;
            }
        {
            df32x16 acc[2] = {df32x16{}, df32x16{}};
            mlp_ntile<DWID>(acc, ah, al, DAP, wave, a.w1_h[hd], a.w1_l[hd]);
            store_hidden(acc, wave, a.b1[hd], bh, bl);
        }
        __syncthreads();
        if (owner) {
            df32x16 acc[2] = {df32x16{}, df32x16{}};
            mlp_ntile<DWID>(acc, bh, bl, DAP, wave, a.w2_h[hd], a.w2_l[hd]);
            if (col < nout) {
                const float b = a.b2[hd][col];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const int r = row_of(mt, q, h), g = g0 + r;
                        const float v = acc[mt][q] + b;
                        if (resid_add) {
                            if (g < a.P) __builtin_nontemporal_store(resid[mt][q] + v, a.out[hd] + (size_t)g * nout + col);
                        } else {
                            s_q[r][col] = v;
                            if (!GRAD && coff && a.out_coff && g < a.P) a.out_coff[(size_t)g * nout + col] = v;
                        }
                    }
            }
            if (!resid_add) {                                        // wave 0: one Gaussian per lane
                wave_lds_sync();
                const int g = g0 + lane;
                if (GRAD && g < a.P) {
                    if (quat) quat_grad(b, g, s_q[lane]);
                    else discrete_grad(b, g, s_q[lane]);
                } else if (g < a.P) {
                    if (quat) {   // rotations = normalize(rotations (x) d_rot)  (deformation.py:135-136)
                        const float4 q1 = reinterpret_cast<const float4*>(a.in[2])[g];
                        const float4 p = quat_mul(q1, make_float4(s_q[lane][0], s_q[lane][1], s_q[lane][2], s_q[lane][3]));
                        const float inv = 1.0f / sqrtf(p.x * p.x + p.y * p.y + p.z * p.z + p.w * p.w);
                        reinterpret_cast<float4*>(a.out[2])[g] = make_float4(p.x * inv, p.y * inv, p.z * inv, p.w * inv);
                    } else {
                        discrete_combine(a, g, s_q[lane], a.out_lang);
                    }
                }
            }
        }
        __syncthreads();
    }
}

template <int S, bool GRAD>
static void go_fwd(const DeformBwdArgs& b, hipStream_t st) {
    hipLaunchKernelGGL((k_deform_fwd<S, GRAD>), dim3((b.f.P + DN - 1) / DN), dim3(256), 0, st, b);
}
template <bool GRAD>
static void go_fwd_s(const DeformBwdArgs& b, hipStream_t st) {
    switch (b.f.n_scales) {
        case 1: go_fwd<1, GRAD>(b, st); break;
        case 2: go_fwd<2, GRAD>(b, st); break;
        case 3: go_fwd<3, GRAD>(b, st); break;
        default: go_fwd<4, GRAD>(b, st); break;
    }
}
void launch_deform_fwd(const DeformArgs& a, hipStream_t st) {
    if (a.P <= 0) return;
    DeformBwdArgs b{};
    b.f = a;
    go_fwd_s<false>(b, st);
}

// The heads with at most DEF_SMALL_OUT outputs (pos, scales, rotations, opacity: 3 / 3 / 4 / 1) take
// G W2 and G^T relu(Z1) on the VALU from fp32 G rows (a float4 per row in LDS, read as a
// broadcast by the half-wave that holds the row): as 64-padded MFMA products they were 61 / 64
// zeros, with their weight fragments re-read from L2 every tile.
constexpr int DEF_SMALL_OUT = 4;
// W2 rows 0..3 of column c as fp32 (hi + lo of the forward pack; rows past nout are the pack's zeros)
__device__ __forceinline__ void w2_column(const __bf16* w2h, const __bf16* w2l, int c, float (&w)[DEF_SMALL_OUT]) {
#pragma unroll
    for (int k = 0; k < DEF_SMALL_OUT; ++k) w[k] = (float)w2h[k * DWID + c] + (float)w2l[k * DWID + c];
}
// ==== backward ====================================================================================
// Phase A, one block per 64 Gaussians (the forward's tiling): recompute the features X and the
// chain A_k = relu(H_k) (saved); per head, Z1 = A W1^T + b1, the gradient G of the head's output
// (the upstream gradient, or for the quaternion product / the discrete combination their
// per-Gaussian backward from the recomputed output), dZ1 = (G W2) * [Z1 > 0], and dA += dZ1 W1
// (the heads' Z1 / dZ1 are not saved: k_head_wgrad recomputes them for the weight gradients), all
// on the bf16 hi/lo MFMA of the forward with transposed weight
// packs; then back through the chain, dH_k = dA_k * [H_k > 0] (saved), dA_{k-1} = dH_k W_k, and
// dX = dH_0 W_0; and per Gaussian the HexPlane backward: each plane's sample gets dX times the
// product of the other five planes of its scale, scattered to the 4 bilinear taps (float atomics
// into a channel-last gradient copy: the 16 channels of a tap are one 64-byte segment), and the
// coordinate gradient (zero where border padding clips) goes to d_means3D.
constexpr int DGP = 64 + 8;   // LDS row pitch (bf16) of the upstream-gradient rows (K padded to 64)

// DEEP: a feature_out chain of more than one layer (defor_depth >= 2; runtime length).  The
// one-layer chain of every reference config gets its own instantiation: the runtime-length loops
// cost registers (spills) even when they run once.
template <int S, bool DEEP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DEEP ? 1 : 2, 2))) k_deform_bwd_a(DeformBwdArgs b) {
    constexpr int F = 16 * S, XP = F + 8;
    static_assert(XP <= DAP, "feature rows live in the second hidden buffer");
    __shared__ __attribute__((aligned(16))) __bf16 s_hh[2][DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_hl[2][DN * DAP];
    __bf16* const s_xh = s_hh[1];   // read by the first layer only, which writes buffer 0
    __bf16* const s_xl = s_hl[1];
    __shared__ __attribute__((aligned(16))) float4 s_g4[DN];   // small-output heads: fp32 G rows
    __shared__ uint32_t s_apos[DEEP ? 1 : 256];   // one layer: each thread's A_0 > 0 bits
    // Everything else lives in a hidden buffer while that buffer is dead (68 KB in all: two blocks
    // per CU): a head's G rows in the buffer its dZ1 rows take next (a barrier between the two), dX in
    // the chain's dead buffer, the plane-scatter staging in its lo half; every hand-over is a
    // __syncthreads, and the LDS-poison build checks that nothing reads a word its block never wrote.
    static_assert(DN * (F + 1) * 4 <= DN * DAP * 2, "dX rows fit one hidden buffer");
    static_assert((4 * 16 * 17 + 2 * 4 * 16 * 4) * 4 <= DN * DAP * 2, "scatter staging fits one hidden buffer");
    LDS_POISON(s_hh); LDS_POISON(s_hl); LDS_POISON(s_g4); LDS_POISON_DONE();
    const DeformArgs& a = b.f;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int g0 = blockIdx.x * DN;
    const int col = 32 * wave + (lane & 31), hh = lane >> 5;
    const int L = DEEP ? a.nlayers : 1;
#ifdef LSR_DEFORM_STAMPS
    unsigned long long ds_sum[13] = {}, ds_prev = 0;
#endif
    DSTAMP(-1);

    // ---- features (as the forward), saved as fp32 for the first layer's weight gradient ---------
    features_to_lds<S>(a, g0, s_xh, s_xl, XP, b.sX);
    __syncthreads();
    DSTAMP(0);

    // ---- chain forward, A_k = relu(H_k) saved ------------------------------------------------------
    int cur = 0;
    uint32_t apos = 0;   // one layer (!DEEP): bit 16 mt + q = A_0 > 0, the chain backward's ReLU mask,
                         // parked in LDS across the heads (a live register there spilled 38)
    for (int k = 0; k < L; ++k) {
        df32x16 acc[2] = {df32x16{}, df32x16{}};
        if (k == 0) mlp_ntile<F>(acc, s_xh, s_xl, XP, wave, a.wf_h[0], a.wf_l[0]);
        else mlp_ntile<DWID>(acc, s_hh[cur], s_hl[cur], DAP, wave, a.wf_h[k], a.wf_l[k]);
        const int dst = k == 0 ? 0 : cur ^ 1;
        store_hidden(acc, wave, a.b_feat[k], s_hh[dst], s_hl[dst]);
        const float bias = a.b_feat[k][col];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int g = g0 + row_of(mt, q, hh);
                const float av = fmaxf(acc[mt][q] + bias, 0.0f);
                if (g < a.P) b.sA[k][(size_t)g * DWID + col] = av;
                if (!DEEP) apos |= av > 0.0f ? 1u << (16 * mt + q) : 0u;
            }
        if (!DEEP) s_apos[tid] = apos;
        __syncthreads();
        cur = dst;
    }
    const __bf16 *ah = s_hh[cur], *al = s_hl[cur];
    __bf16 *bh = s_hh[cur ^ 1], *bl = s_hl[cur ^ 1];

    DSTAMP(1);
    df32x16 dA[2] = {df32x16{}, df32x16{}};
#ifdef LSR_DEFORM_ABL_NOHEADS   // timing ablation only (wrong gradients): the heads' share of phase A
    if (a.P < 0)
#endif
    for (int hd = 0; hd < DEF_HEADS; ++hd) {
        if (!((a.heads >> hd) & 1u)) continue;                       // block-uniform
        const int nout = head_out(a, hd);
        const bool quat = hd == 2 && a.apply_rotation, coff = hd == 5;
        const float* G = coff ? b.sG_coff : quat ? b.sG_rot : b.up[hd];   // saved by the GRAD pass
        // a large head's gradient rows (K padded to 64, 16 per thread) loaded before its Z1 product,
        // which hides their latency (issued after Z1, the conversion below waited for them: 12 % of
        // phase A in the stamp build)
        constexpr int NJ = DN * 64 / 256;
        float gv[NJ];
#ifndef LSR_DEFORM_SHG_LATE
        if (nout > DEF_SMALL_OUT) {                                  // block-uniform
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int i = tid + 256 * j, r = i >> 6, k = i & 63, g = g0 + r;
                gv[j] = (k < nout && g < a.P) ? G[(size_t)g * nout + k] : 0.0f;
            }
        }
#endif
        // Z1 for this wave's 32 columns (its rows finish before the sync below)
        uint32_t zpos = 0;   // bit 16 mt + q: Z1 > 0 (the ReLU mask of dZ1; Z1 itself dies here)
        {
            df32x16 z[2] = {df32x16{}, df32x16{}};
            mlp_ntile<DWID>(z, ah, al, DAP, wave, a.w1_h[hd], a.w1_l[hd]);
            const float bias = a.b1[hd][col];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 16; ++q) zpos |= z[mt][q] + bias > 0.0f ? 1u << (16 * mt + q) : 0u;
        }
        DSTAMP(2);
        if (nout <= DEF_SMALL_OUT) {                                 // block-uniform
            // dZ1 = (G W2) [Z1 > 0] on the VALU from fp32 G rows (k_head_wgrad's small-output path)
            // (loaded after Z1: issued before it, as the SH head's rows, measured 10.65-10.72 vs
            // 10.47-10.54 ms at 2M, 13 VGPRs spilled)
            if (tid < DN) {
                const int g = g0 + tid;
                float v[DEF_SMALL_OUT] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int k = 0; k < DEF_SMALL_OUT; ++k)
                    if (k < nout && g < a.P) v[k] = G[(size_t)g * nout + k];
                s_g4[tid] = make_float4(v[0], v[1], v[2], v[3]);
            }
            float w2c[DEF_SMALL_OUT];
            w2_column(a.w2_h[hd], a.w2_l[hd], col, w2c);
            DSTAMP(8);         // small head: G and W2 column loads issued, G rows stored
            __syncthreads();   // G rows complete
            DSTAMP(9);         // small head: the first barrier
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int r = row_of(mt, q, hh);
                    const float4 gv = s_g4[r];
                    float dv = gv.x * w2c[0];
                    dv = __builtin_fmaf(gv.y, w2c[1], dv);
                    dv = __builtin_fmaf(gv.z, w2c[2], dv);
                    dv = __builtin_fmaf(gv.w, w2c[3], dv);
                    const float v = (zpos >> (16 * mt + q)) & 1u ? dv : 0.0f;
                    __bf16 hi, lo;
                    dsplit(v, hi, lo);
                    bh[r * DAP + col] = hi;
                    bl[r * DAP + col] = lo;
                }
            __syncthreads();   // dZ1 rows complete
            DSTAMP(3);
            mlp_ntile<DWID>(dA, bh, bl, DAP, wave, b.w1t_h[hd], b.w1t_l[hd]);
            DSTAMP(4);
            __syncthreads();   // dZ1 rows and the G rows consumed before the next head rewrites them
            DSTAMP(5);
            continue;
        }
        // gradient rows of this head's output, K padded to 64, in the buffer dZ1 takes next: every load
        // of the thread issued before the first conversion (a load-convert-store loop waited one memory
        // latency per row)
#ifndef LSR_DEFORM_G_LOOP
        {
#ifdef LSR_DEFORM_SHG_LATE   // A/B: loaded here, after Z1
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int i = tid + 256 * j, r = i >> 6, k = i & 63, g = g0 + r;
                gv[j] = (k < nout && g < a.P) ? G[(size_t)g * nout + k] : 0.0f;
            }
#endif
#pragma unroll
            for (int j = 0; j < NJ; ++j) {
                const int i = tid + 256 * j, r = i >> 6, k = i & 63;
                __bf16 hi, lo;
                dsplit(gv[j], hi, lo);
                bh[r * DGP + k] = hi;
                bl[r * DGP + k] = lo;
            }
        }
#else   // A/B: the round-4 loop
        for (int i = tid; i < DN * 64; i += 256) {
            const int r = i >> 6, k = i & 63, g = g0 + r;
            float v = 0.0f;
            if (k < nout && g < a.P) v = G[(size_t)g * nout + k];
            __bf16 hi, lo;
            dsplit(v, hi, lo);
            bh[r * DGP + k] = hi;
            bl[r * DGP + k] = lo;
        }
#endif
        DSTAMP(10);        // SH head: G rows loaded and stored
        __syncthreads();   // G rows complete
        df32x16 d[2] = {df32x16{}, df32x16{}};
        mlp_ntile<64>(d, bh, bl, DGP, wave, b.w2t_h[hd], b.w2t_l[hd]);
        DSTAMP(11);        // SH head: barrier + G W2 product
        __syncthreads();   // every wave has read the G rows: dZ1 overwrites them
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int r = row_of(mt, q, hh);
                const float v = (zpos >> (16 * mt + q)) & 1u ? d[mt][q] : 0.0f;
                __bf16 hi, lo;
                dsplit(v, hi, lo);
                bh[r * DAP + col] = hi;
                bl[r * DAP + col] = lo;
            }
        __syncthreads();   // dZ1 rows complete
        DSTAMP(3);
        mlp_ntile<DWID>(dA, bh, bl, DAP, wave, b.w1t_h[hd], b.w1t_l[hd]);
        DSTAMP(4);
        __syncthreads();   // dZ1 rows consumed before the next head's G rows overwrite them
        DSTAMP(5);
    }

    // ---- back through the chain: dH_k = dA_k * [H_k > 0] (saved), dA_{k-1} = dH_k W_k -------------
    for (int k = L - 1; k >= 0; --k) {
        // dH_k rows into the buffer that does not hold what the MFMA below still reads
        __bf16 *dh_h = s_hh[cur ^ 1], *dh_l = s_hl[cur ^ 1];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int r = row_of(mt, q, hh), g = g0 + r;
#ifndef LSR_DEFORM_CHAIN_RELOAD
                // one layer: the mask from the registers (reloading A_0 put 32 dependent loads of rows
                // this block had just written on the chain's critical path)
                const bool on = DEEP ? (g < a.P && b.sA[k][(size_t)g * DWID + col] > 0.0f)
                                     : (g < a.P && ((s_apos[tid] >> (16 * mt + q)) & 1u));
#else
                const bool on = g < a.P && b.sA[k][(size_t)g * DWID + col] > 0.0f;   // this block wrote it
#endif
                const float v = on ? dA[mt][q] : 0.0f;
                __bf16 hi, lo;
                dsplit(v, hi, lo);
                dh_h[r * DAP + col] = hi;
                dh_l[r * DAP + col] = lo;
                if (g < a.P) b.sdH[k][(size_t)g * DWID + col] = v;
            }
        __syncthreads();
        cur ^= 1;
        if (k > 0) {
            df32x16 acc[2] = {df32x16{}, df32x16{}};
            mlp_ntile<DWID>(acc, dh_h, dh_l, DAP, wave, b.wft_h[k], b.wft_l[k]);
            dA[0] = acc[0];
            dA[1] = acc[1];
            __syncthreads();   // the dH rows read before the next iteration overwrites the other buffer
        } else if (wave < (F + 31) / 32) {
            df32x16 acc[2] = {df32x16{}, df32x16{}};
            mlp_ntile<DWID>(acc, dh_h, dh_l, DAP, wave, b.wft_h[0], b.wft_l[0]);
            const int c = 32 * wave + (lane & 31);
            // dX rows [64][F + 1] in the other hidden buffer (its rows died with the heads)
            float* dxw = reinterpret_cast<float*>(s_hh[cur ^ 1]);
            if (c < F) {
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int q = 0; q < 16; ++q) dxw[row_of(mt, q, hh) * (F + 1) + c] = acc[mt][q];
            }
        }
    }
    __syncthreads();
    DSTAMP(6);
    const float* s_dx = reinterpret_cast<const float*>(s_hh[cur ^ 1]);   // [64][F + 1]
    // plane-scatter staging in the lo half of that buffer: per wave, dv of 16 Gaussians [16][17],
    // their 4 tap offsets and bilinear weights
    float* const s_sdv = reinterpret_cast<float*>(s_hl[cur ^ 1]);
    int* const s_soff = reinterpret_cast<int*>(s_sdv + 4 * 16 * 17);
    float* const s_sw = reinterpret_cast<float*>(s_soff + 4 * 16 * 4);

    // ---- HexPlane backward: 4 threads per Gaussian, 4 channels each ----------------------------------
#ifdef LSR_DEFORM_ABL_NOHEX   // timing ablation only (wrong gradients): the HexPlane backward's share
    if (a.P < 0)
#endif
    {
        const int gl = tid >> 2, q = tid & 3;
        const bool ok = g0 + gl < a.P;
        const int g = min(g0 + gl, a.P - 1);
        float crd[4];
        coords(a, g, crd);
        float dq[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        // every Gaussian of this wave at the call's first time (a vote, no barrier)
        const bool t_row = b.trow && __all(crd[3] == a.time[0]);
        // a scale's plane gradients dv (24 registers) and its coordinate gradient: each plane's 4 taps
        // loaded once for the sample (sample4's arithmetic) and its x / y derivatives
        auto grad_scale = [&](int s, float4 (&dvo)[6]) __attribute__((always_inline)) {
            float4 v[6], gxv[6], gyv[6];
#pragma unroll
            for (int ci = 0; ci < 6; ++ci) {
                const int pi = 6 * s + ci, W = a.pw[pi];
                const Tap t = tap_of(a, pi, ci, crd);
                const float4* pl = reinterpret_cast<const float4*>(a.planes + a.poff[pi]) + q;
                const float4 t00 = pl[(t.y0 * W + t.x0) * 4], t01 = pl[(t.y0 * W + t.x1) * 4];
                const float4 t10 = pl[(t.y1 * W + t.x0) * 4], t11 = pl[(t.y1 * W + t.x1) * 4];
                const float w00 = (1.0f - t.fx) * (1.0f - t.fy), w01 = t.fx * (1.0f - t.fy), w10 = (1.0f - t.fx) * t.fy,
                            w11 = t.fx * t.fy;
                v[ci] = make_float4(t00.x * w00 + t01.x * w01 + t10.x * w10 + t11.x * w11,
                                    t00.y * w00 + t01.y * w01 + t10.y * w10 + t11.y * w11,
                                    t00.z * w00 + t01.z * w01 + t10.z * w10 + t11.z * w11,
                                    t00.w * w00 + t01.w * w01 + t10.w * w10 + t11.w * w11);
                const float ux = 1.0f - t.fy, uy = 1.0f - t.fx;
                gxv[ci] = make_float4((t01.x - t00.x) * ux + (t11.x - t10.x) * t.fy, (t01.y - t00.y) * ux + (t11.y - t10.y) * t.fy,
                                      (t01.z - t00.z) * ux + (t11.z - t10.z) * t.fy, (t01.w - t00.w) * ux + (t11.w - t10.w) * t.fy);
                gyv[ci] = make_float4((t10.x - t00.x) * uy + (t11.x - t01.x) * t.fx, (t10.y - t00.y) * uy + (t11.y - t01.y) * t.fx,
                                      (t10.z - t00.z) * uy + (t11.z - t01.z) * t.fx, (t10.w - t00.w) * uy + (t11.w - t01.w) * t.fx);
            }
            const float* dxr = s_dx + gl * (F + 1) + 16 * s + 4 * q;
            const float dxv[4] = {dxr[0], dxr[1], dxr[2], dxr[3]};
#pragma unroll
            for (int ci = 0; ci < 6; ++ci) {
                float4 oth = make_float4(1.0f, 1.0f, 1.0f, 1.0f);
#pragma unroll
                for (int cj = 0; cj < 6; ++cj)
                    if (cj != ci) {
                        oth.x *= v[cj].x; oth.y *= v[cj].y; oth.z *= v[cj].z; oth.w *= v[cj].w;
                    }
                const float dv[4] = {dxv[0] * oth.x, dxv[1] * oth.y, dxv[2] * oth.z, dxv[3] * oth.w};
                dvo[ci] = make_float4(dv[0], dv[1], dv[2], dv[3]);
                const int pi = 6 * s + ci;
                const int W = a.pw[pi], H = a.ph[pi];
                const float rx = (crd[kC0(ci)] + 1.0f) * 0.5f * (float)(W - 1);
                const float ry = (crd[kC1(ci)] + 1.0f) * 0.5f * (float)(H - 1);
                const float gx4[4] = {gxv[ci].x, gxv[ci].y, gxv[ci].z, gxv[ci].w};
                const float gy4[4] = {gyv[ci].x, gyv[ci].y, gyv[ci].z, gyv[ci].w};
                float dix = 0.0f, diy = 0.0f;
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    dix += dv[i] * gx4[i];
                    diy += dv[i] * gy4[i];
                }
                if (rx > 0.0f && rx < (float)(W - 1)) dq[kC0(ci)] += dix * 0.5f * (float)(W - 1);
                if (ry > 0.0f && ry < (float)(H - 1)) dq[kC1(ci)] += diy * 0.5f * (float)(H - 1);
            }
        };
        // scatter: stage the wave's 16 Gaussians (16 channels, 4 taps each) in LDS, then one atomic
        // instruction per Gaussian covers its 4 taps x 16 channels = four full 64-byte segments (lane =
        // 16 tap + channel) instead of 16 partial ones; blocks add into one of b.replicas copies of the
        // gradient planes (summed by the unpack), so the few cells every Gaussian of a frame shares (the
        // time planes) are not one hot spot
        auto scatter_scale = [&](int s, const float4 (&dvo)[6]) __attribute__((always_inline)) {
#pragma unroll
            for (int ci = 0; ci < 6; ++ci) {
                const int pi = 6 * s + ci, W = a.pw[pi];
                const Tap t = tap_of(a, pi, ci, crd);
                const float dv[4] = {dvo[ci].x, dvo[ci].y, dvo[ci].z, dvo[ci].w};
                const int wl = gl & 15;
                if ((ci == 2 || ci >= 4) && t_row) {   // wave-uniform
                    // a time plane of a wave at time[0]: its x-row (b.trow), 2 taps x 16 channels per
                    // Gaussian, two Gaussians per atomic instruction (half the time planes' requests)
#pragma unroll
                    for (int i = 0; i < 4; ++i) s_sdv[(wave * 16 + wl) * 17 + 4 * q + i] = ok ? dv[i] : 0.0f;
                    if (q == 0) {
                        s_soff[(wave * 16 + wl) * 4 + 0] = t.x0 * 16;
                        s_soff[(wave * 16 + wl) * 4 + 1] = t.x1 * 16;
                        s_sw[(wave * 16 + wl) * 4 + 0] = 1.0f - t.fx;
                        s_sw[(wave * 16 + wl) * 4 + 1] = t.fx;
                    }
                    wave_lds_sync();
                    float* rp = b.trow + (size_t)(blockIdx.x % b.trow_reps) * b.trow_stride + b.toff[pi];
                    const int tap = (lane >> 4) & 1, ch = lane & 15, half = lane >> 5;
#pragma unroll 4
                    for (int j = 0; j < 8; ++j) {
                        const int e = wave * 16 + 2 * j + half;
                        const float val = s_sdv[e * 17 + ch] * s_sw[e * 4 + tap];
#ifndef LSR_DEFORM_ABL_NOTIME
                        if (val != 0.0f) atomicAdd(rp + s_soff[e * 4 + tap] + ch, val);
#endif
                    }
                    wave_lds_sync();   // staging read before the next plane rewrites it
                    continue;
                }
                const float w00 = (1.0f - t.fx) * (1.0f - t.fy), w01 = t.fx * (1.0f - t.fy),
                            w10 = (1.0f - t.fx) * t.fy, w11 = t.fx * t.fy;
#pragma unroll
                for (int i = 0; i < 4; ++i) s_sdv[(wave * 16 + wl) * 17 + 4 * q + i] = ok ? dv[i] : 0.0f;
                if (q == 0) {
                    int* so = s_soff + (wave * 16 + wl) * 4;
                    float* sw = s_sw + (wave * 16 + wl) * 4;
                    so[0] = (t.y0 * W + t.x0) * 16; so[1] = (t.y0 * W + t.x1) * 16;
                    so[2] = (t.y1 * W + t.x0) * 16; so[3] = (t.y1 * W + t.x1) * 16;
                    sw[0] = w00; sw[1] = w01; sw[2] = w10; sw[3] = w11;
                }
                wave_lds_sync();
                float* gp = b.dplanes + (size_t)(blockIdx.x % b.replicas) * b.plane_stride + a.poff[pi];
                const int tap = lane >> 4, ch = lane & 15;
#pragma unroll 4
                for (int j = 0; j < 16; ++j) {
                    const float val = s_sdv[(wave * 16 + j) * 17 + ch] * s_sw[(wave * 16 + j) * 4 + tap];
#ifdef LSR_DEFORM_DIAG
                    const int off = s_soff[(wave * 16 + j) * 4 + tap];
                    const int H = a.ph[pi];
                    if (off < 0 || off >= W * H * 16 || !(fabsf(val) < 1e30f)) {
                        atomicAdd(&g_deform_diag[0], 1ull);
                        atomicAdd(&g_deform_diag[1 + tap], 1ull);
                        continue;
                    }
#endif
#ifndef LSR_DEFORM_ABL_NOSCATTER   // timing ablation only (wrong plane gradients)
#ifdef LSR_DEFORM_ABL_NOTIME        // timing ablation only: the time planes' (xt, yt, zt) atomics skipped
                    if (ci == 2 || ci >= 4) continue;
#endif
                    if (val != 0.0f) atomicAdd(gp + s_soff[(wave * 16 + j) * 4 + tap] + ch, val);
#endif
                }
                wave_lds_sync();   // staging read before the next plane rewrites it
            }
        };
#ifndef LSR_DEFORM_HEX_INTERLEAVED
        {
            // every scale's taps loaded (and its coordinate gradient formed) before the first scatter:
            // vmcnt retires in order and counts the atomics, so tap loads issued behind a scale's
            // atomics waited for them; the scales' dv (24 registers each) stay live in between
            float4 dvo[S][6];
#pragma unroll
            for (int s = 0; s < S; ++s) grad_scale(s, dvo[s]);
            DSTAMP(12);        // taps, dv and the coordinate gradient of every scale
#pragma unroll
            for (int s = 0; s < S; ++s) scatter_scale(s, dvo[s]);
        }
#else
#pragma unroll
        for (int s = 0; s < S; ++s) {
            float4 dvo[6];
            grad_scale(s, dvo);
            scatter_scale(s, dvo);
        }
#endif
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
        if (b.daabb) {   // block-uniform
            // normalize_aabb's gradient w.r.t. the box (hexplane.py:19-20): with n = (p - a0) s - 1,
            // s = 2 / (a1 - a0): dn/da0 = s (n - 1) / 2, dn/da1 = -s (n + 1) / 2, and dq = dL/dn
            float v[6];
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                const float gp = (ok && q == 0) ? dq[c] * (2.0f / (a.aabb[3 + c] - a.aabb[c])) : 0.0f;
                v[c] = 0.5f * gp * (crd[c] - 1.0f);
                v[3 + c] = -0.5f * gp * (crd[c] + 1.0f);
            }
#pragma unroll
            for (int k = 0; k < 6; ++k) {
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) v[k] += __shfl_xor(v[k], off);
            }
            if ((tid & 63) == 0) {   // one of DEF_AABB_SLOTS partial rows: every wave of a
                                     // launch adding into the same six words serialised on one L2 line
                float* row = b.daabb_part + (blockIdx.x % DEF_AABB_SLOTS) * 16;
#pragma unroll
                for (int k = 0; k < 6; ++k) atomicAdd(row + k, v[k]);
            }
        }
    }
#ifdef LSR_DEFORM_STAMPS
    DSTAMP(7);
    if (tid == 0) {
#pragma unroll
        for (int k = 0; k < 13; ++k) atomicAdd(&g_deform_stamps[k], ds_sum[k]);
        atomicAdd(&g_deform_stamps[13], 1ull);
    }
#endif
}

template <int S>
#ifndef LSR_DEFORM_BWD_DYN_LDS
#define LSR_DEFORM_BWD_DYN_LDS 0   // diagnostic builds: unused dynamic LDS per block (occupancy control)
#endif
static void go_bwd(const DeformBwdArgs& b, hipStream_t st) {
    const unsigned dyn = LSR_DEFORM_BWD_DYN_LDS;
    if (b.f.nlayers > 1) hipLaunchKernelGGL((k_deform_bwd_a<S, true>), dim3((b.f.P + DN - 1) / DN), dim3(256), dyn, st, b);
    else hipLaunchKernelGGL((k_deform_bwd_a<S, false>), dim3((b.f.P + DN - 1) / DN), dim3(256), dyn, st, b);
}
void launch_deform_bwd_a(const DeformBwdArgs& b, hipStream_t st) {
    if (b.f.P <= 0) return;
    if (b.f.apply_rotation || (b.f.heads >> 5) & 1u) go_fwd_s<true>(b, st);   // the nonlinear heads' gradients
    switch (b.f.n_scales) {
        case 1: go_bwd<1>(b, st); break;
        case 2: go_bwd<2>(b, st); break;
        case 3: go_bwd<3>(b, st); break;
        default: go_bwd<4>(b, st); break;
    }
}

// ==== lang_deform (deformation.py:68, 172-180) ====================================================
// relu([lang, t, sin(2^i t), cos(2^i t)]) -> Linear(kin, 128), ReLU, Linear(128, 128), ReLU,
// Linear(128, lang_dim); lang_out = normalize((lang +) dl).  One block per 64 Gaussians; the input
// rows are K-padded to a multiple of 16 (<= 64).
__device__ __forceinline__ float lang_in_value(const LangDeformArgs& a, int g, int k) {
    const int C = a.lang_dim;
    if (k < C) return a.lang[(size_t)g * C + k];
    const float t = a.time[g];
    if (k == C) return t;
    const int j = k - C - 1;                                          // poc_fre: sin block, cos block
    if (j < a.time_pe) return sinf(t * (float)(1 << j));
    if (j < 2 * a.time_pe) return cosf(t * (float)(1 << (j - a.time_pe)));
    return 0.0f;
}

// forward of the MLP for the block's 64 rows; leaves v = (lang +) dl in s_v[64][33] (and with
// `save`, the saved activations).  kpad = 16-padded input width.
__device__ __forceinline__ void lang_mlp_fwd(const LangDeformArgs& a, int g0, int kpad, __bf16* xh, __bf16* xl,
                                             __bf16 (*hh)[DN * DAP], __bf16 (*hl)[DN * DAP], float (*s_v)[33], bool save) {
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hh_ = lane >> 5;
    for (int i = tid; i < DN * 64; i += 256) {
        const int r = i >> 6, k = i & 63, g = g0 + r;
        const float v = (g < a.P && k < a.kin) ? fmaxf(lang_in_value(a, g, k), 0.0f) : 0.0f;
        if (k < kpad) {
            __bf16 hi, lo;
            dsplit(v, hi, lo);
            xh[r * DLP + k] = hi;
            xl[r * DLP + k] = lo;
        }
        if (save && g < a.P && k < a.kin) a.sU0[(size_t)g * a.kin + k] = v;
    }
    __syncthreads();
    const int col = 32 * wave + (lane & 31);
    for (int layer = 0; layer < 2; ++layer) {
        df32x16 acc[2] = {df32x16{}, df32x16{}};
        if (layer == 0) mlp_ntile_k(kpad, acc, xh, xl, DLP, wave, a.w_h[0], a.w_l[0]);
        else mlp_ntile<DWID>(acc, hh[0], hl[0], DAP, wave, a.w_h[1], a.w_l[1]);
        store_hidden(acc, wave, a.b[layer], hh[layer], hl[layer]);
        if (save) {
            const float bias = a.b[layer][col];
            float* dst = layer == 0 ? a.sU1 : a.sU2;
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int g = g0 + row_of(mt, q, hh_);
                    if (g < a.P) dst[(size_t)g * DWID + col] = fmaxf(acc[mt][q] + bias, 0.0f);
                }
        }
        __syncthreads();
    }
    if (wave == 0) {
        df32x16 acc[2] = {df32x16{}, df32x16{}};
        mlp_ntile<DWID>(acc, hh[1], hl[1], DAP, 0, a.w_h[2], a.w_l[2]);
        const int c = lane & 31;
        if (c < a.lang_dim) {
            const float bias = a.b[2][c];
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int r = row_of(mt, q, hh_), g = g0 + r;
                    float v = acc[mt][q] + bias;
                    if (a.residual && g < a.P) v += a.lang[(size_t)g * a.lang_dim + c];
                    s_v[r][c] = v;
                }
        }
    }
    __syncthreads();
}

__global__ void __launch_bounds__(256) k_lang_deform_fwd(LangDeformArgs a) {
    __shared__ __attribute__((aligned(16))) __bf16 s_xh[DN * DLP];
    __shared__ __attribute__((aligned(16))) __bf16 s_xl[DN * DLP];
    __shared__ __attribute__((aligned(16))) __bf16 s_hh[2][DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_hl[2][DN * DAP];
    __shared__ float s_v[DN][33];
    LDS_POISON(s_xh); LDS_POISON(s_xl); LDS_POISON(s_hh); LDS_POISON(s_hl); LDS_POISON(s_v); LDS_POISON_DONE();
    const int g0 = blockIdx.x * DN, tid = threadIdx.x;
    const int kpad = (a.kin + 15) / 16 * 16;
    lang_mlp_fwd(a, g0, kpad, s_xh, s_xl, s_hh, s_hl, s_v, false);
    if (tid < DN && g0 + tid < a.P) {   // out = v / (|v| + 1e-9)
        float n2 = 0.0f;
        for (int c = 0; c < a.lang_dim; ++c) n2 += s_v[tid][c] * s_v[tid][c];
        const float inv = 1.0f / (sqrtf(n2) + 1e-9f);
        for (int c = 0; c < a.lang_dim; ++c) a.out_lang[(size_t)(g0 + tid) * a.lang_dim + c] = s_v[tid][c] * inv;
    }
}

__global__ void __launch_bounds__(256) k_lang_deform_bwd(LangDeformArgs a) {
    __shared__ __attribute__((aligned(16))) __bf16 s_xh[DN * DLP];
    __shared__ __attribute__((aligned(16))) __bf16 s_xl[DN * DLP];
    __shared__ __attribute__((aligned(16))) __bf16 s_hh[2][DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_hl[2][DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_gh[DN * DLP];
    __shared__ __attribute__((aligned(16))) __bf16 s_gl[DN * DLP];
    __shared__ float s_v[DN][33];
    LDS_POISON(s_xh); LDS_POISON(s_xl); LDS_POISON(s_hh); LDS_POISON(s_hl); LDS_POISON(s_gh); LDS_POISON(s_gl);
    LDS_POISON(s_v); LDS_POISON_DONE();
    const int g0 = blockIdx.x * DN, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, hh = lane >> 5;
    const int col = 32 * wave + (lane & 31);
    const int C = a.lang_dim, kpad = (a.kin + 15) / 16 * 16;
    lang_mlp_fwd(a, g0, kpad, s_xh, s_xl, s_hh, s_hl, s_v, true);
    // dv = d / (|v| + eps) - v (v . d) / (|v| (|v| + eps)^2), d = the upstream language gradient
    if (tid < DN) {
        const int g = g0 + tid;
        float n2 = 0.0f, vd = 0.0f;
        for (int c = 0; c < C; ++c) {
            const float up = (g < a.P && a.up_lang) ? a.up_lang[(size_t)g * C + c] : 0.0f;
            n2 += s_v[tid][c] * s_v[tid][c];
            vd += s_v[tid][c] * up;
        }
        const float n = sqrtf(n2), ne = n + 1e-9f, f = n > 0.0f ? vd / (n * ne * ne) : 0.0f;
        for (int c = 0; c < 32; ++c) {
            float dv = 0.0f;
            if (c < C && g < a.P) dv = (a.up_lang ? a.up_lang[(size_t)g * C + c] : 0.0f) / ne - s_v[tid][c] * f;
            s_v[tid][c] = dv;
            __bf16 hi, lo;
            dsplit(dv, hi, lo);
            s_gh[tid * DLP + c] = hi;
            s_gl[tid * DLP + c] = lo;
            if (c < C && g < a.P) a.sdv[(size_t)g * C + c] = dv;
        }
    }
    __syncthreads();
    // dZ2 = (dv W3) * [U2 > 0]; dZ1 = (dZ2 W2) * [U1 > 0]   (U_k > 0 <=> Z_k > 0)
    for (int layer = 1; layer >= 0; --layer) {
        df32x16 acc[2] = {df32x16{}, df32x16{}};
        if (layer == 1) mlp_ntile<32>(acc, s_gh, s_gl, DLP, wave, a.wt_h[2], a.wt_l[2]);
        else mlp_ntile<DWID>(acc, s_hh[1], s_hl[1], DAP, wave, a.wt_h[1], a.wt_l[1]);
        const __bf16 *uh = s_hh[layer], *ul = s_hl[layer];
        float dz[2][16];
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int r = row_of(mt, q, hh);
                const bool on = (float)uh[r * DAP + col] + (float)ul[r * DAP + col] > 0.0f;
                dz[mt][q] = on ? acc[mt][q] : 0.0f;
            }
        float* save = layer == 1 ? a.sdZ2 : a.sdZ1;
        __syncthreads();   // U rows (and, for layer 0, the dZ2 rows in buffer 1) read
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int r = row_of(mt, q, hh), g = g0 + r;
                __bf16 hi, lo;
                dsplit(dz[mt][q], hi, lo);
                s_hh[1][r * DAP + col] = hi;   // dZ rows replace U2 (the next step's A operand)
                s_hl[1][r * DAP + col] = lo;
                if (g < a.P) save[(size_t)g * DWID + col] = dz[mt][q];
            }
        __syncthreads();
    }
    // dU0 = dZ1 W1 (waves owning input columns), d_lang = (dv if residual) + dU0 * [U0 > 0]
    if (wave < (kpad + 31) / 32) {
        df32x16 acc[2] = {df32x16{}, df32x16{}};
        mlp_ntile<DWID>(acc, s_hh[1], s_hl[1], DAP, wave, a.wt_h[0], a.wt_l[0]);
        const int c = 32 * wave + (lane & 31);
        if (c < C) {
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const int r = row_of(mt, q, hh), g = g0 + r;
                    if (g >= a.P) continue;
                    const bool on = (float)s_xh[r * DLP + c] + (float)s_xl[r * DLP + c] > 0.0f;
                    a.d_lang[(size_t)g * C + c] = (a.residual ? s_v[r][c] : 0.0f) + (on ? acc[mt][q] : 0.0f);
                }
        }
    }
}

void launch_lang_deform_fwd(const LangDeformArgs& a, hipStream_t st) {
    if (a.P > 0) hipLaunchKernelGGL(k_lang_deform_fwd, dim3((a.P + DN - 1) / DN), dim3(256), 0, st, a);
}
void launch_lang_deform_bwd(const LangDeformArgs& a, hipStream_t st) {
    if (a.P > 0) hipLaunchKernelGGL(k_lang_deform_bwd, dim3((a.P + DN - 1) / DN), dim3(256), 0, st, a);
}

// ==== head weight gradients by recompute ===========================================================
// Round 3 saved every head's relu(Z1) and dZ1 rows in phase A (2 x 128 floats per Gaussian per head:
// 10 GB written and read back at 2M Gaussians with five heads) for the split-K products of k_atb.
// Here a block walks its rows in tiles of 64 and recomputes them from the saved trunk activation A
// (512 B per row) and the head's output gradient G:
//   Z1 = A W1^T + b1 (mlp_ntile, as the forward),  dZ1 = (G W2) * [Z1 > 0] (as phase A),
//   dW1 += dZ1^T A,  dW2 += G^T relu(Z1),  db1 += sum dZ1,  db2 += sum G,
// accumulating the block's partial products in registers over all its tiles; one atomic per output
// element at the end.  The reduction index of the last two products is the row: wave w holds
// dZ1 and relu(Z1) for its 32 columns in the MFMA result layout, whose rows split 4 / 4 between the
// two half-waves, so one permlane32 swap per register pair turns them into the row-runs of 8 the
// 32x32x16 operands take; the A and G operands come from their LDS rows through transposing reads.
// Rows past P read as zero (their dZ1 and G vanish, so relu(b1) never reaches a product).
__device__ __forceinline__ void wg_regs_to_op(const df32x16& v, int u, dbf16x8& oh, dbf16x8& ol) {
    // rows 16u .. 16u + 15 of this 32-row M tile: lane half h gets rows 16u + 8h .. + 7
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v[8 * u + i]), __float_as_uint(v[8 * u + 4 + i]),
                                                  false, false);
        const float x0 = __uint_as_float(r[0]), x1 = __uint_as_float(r[1]);
        __bf16 h0, l0, h1, l1;
        dsplit(x0, h0, l0);
        dsplit(x1, h1, l1);
        oh[i] = h0; ol[i] = l0;
        oh[4 + i] = h1; ol[4 + i] = l1;
    }
}
// 8 consecutive rows (16 ks + 8 h ..) of column c0 + (lane & 31) of a row-major bf16 LDS array,
// through two ds_read_b64_tr_b16 (each 16-lane group reads a 4-row x 16-column block)
__device__ __forceinline__ dbf16x8 wg_lds_op(const __bf16* base, int pitch, int ks, int c0) {
    const int lane = threadIdx.x & 63, h = lane >> 5, l16 = lane & 15;
    const __bf16* p = base + (16 * ks + 8 * h + (l16 >> 2)) * pitch + c0 + 16 * ((lane >> 4) & 1) + 4 * (l16 & 3);
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    const s16x4 a0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        reinterpret_cast<__attribute__((address_space(3))) s16x4*>(reinterpret_cast<size_t>(p)));
    const s16x4 a1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        reinterpret_cast<__attribute__((address_space(3))) s16x4*>(reinterpret_cast<size_t>(p + 4 * pitch)));
    const s16x8 v = __builtin_shufflevector(a0, a1, 0, 1, 2, 3, 4, 5, 6, 7);
    return __builtin_bit_cast(dbf16x8, v);
}

// A rows of a 64-row tile into LDS as bf16 hi / lo (4 values per 8-byte store); rows past row1 are zero
__device__ __forceinline__ void a_rows_to_lds(const float* __restrict__ A, int64_t t0, int64_t row1, __bf16* ah, __bf16* al) {
    typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
    const int tid = threadIdx.x;
#pragma unroll
    for (int i = tid; i < DN * (DWID / 4); i += 256) {
        const int rr = i >> 5, c4 = (i & 31) * 4;
        const int64_t g = t0 + rr;
        const float4 v = g < row1 ? *reinterpret_cast<const float4*>(A + g * DWID + c4) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const float f[4] = {v.x, v.y, v.z, v.w};
        bf4 h4, l4;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
            __bf16 hi, lo;
            dsplit(f[e], hi, lo);
            h4[e] = hi; l4[e] = lo;
        }
        *reinterpret_cast<bf4*>(ah + rr * DAP + c4) = h4;
        *reinterpret_cast<bf4*>(al + rr * DAP + c4) = l4;
    }
}

template <bool SMALL>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2))) k_head_wgrad(HeadWgradArgs ha, int job0) {
    __shared__ __attribute__((aligned(16))) __bf16 s_ah[DN * DAP];   // A rows [64][128] hi / lo
    __shared__ __attribute__((aligned(16))) __bf16 s_al[DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_gh[SMALL ? 8 : DN * DGP];   // G rows [64][64 pad] hi / lo
    __shared__ __attribute__((aligned(16))) __bf16 s_gl[SMALL ? 8 : DN * DGP];
    __shared__ __attribute__((aligned(16))) float4 s_g4[SMALL ? DN : 1];        // SMALL: G rows fp32
    LDS_POISON(s_ah); LDS_POISON(s_al); LDS_POISON(s_gh); LDS_POISON(s_gl); LDS_POISON(s_g4); LDS_POISON_DONE();
    const HeadWgradJob& j = ha.job[job0 + blockIdx.y];
    const int64_t row0 = (int64_t)blockIdx.x * ha.rows_per_block;
    const int64_t row1 = min((int64_t)ha.P, row0 + ha.rows_per_block);
    if (row0 >= row1) return;                                            // block-uniform
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
    const int nout = j.nout, Mo = (nout + 31) / 32;                      // G^T M tiles (1 or 2)
    const int col = 32 * wave + r;
    const float b1c = j.b1[col];
    df32x16 w1acc[4] = {df32x16{}, df32x16{}, df32x16{}, df32x16{}};   // dW1 rows 32 wave .., col tiles 0..3
    df32x16 w2acc[SMALL ? 1 : 2];                                         // dW2 o tiles 0..1, col tile wave
    float w2s[DEF_SMALL_OUT] = {0.0f, 0.0f, 0.0f, 0.0f};                 // SMALL: dW2 rows 0..3, column col
    float w2c[DEF_SMALL_OUT] = {0.0f, 0.0f, 0.0f, 0.0f};                 // SMALL: W2 rows 0..3, column col
    float4 db2v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if constexpr (SMALL) w2_column(j.w2_h, j.w2_l, col, w2c);
    else { w2acc[0] = df32x16{}; w2acc[1] = df32x16{}; }
    float db1 = 0.0f, db2 = 0.0f;
    for (int64_t t0 = row0; t0 < row1; t0 += DN) {
        // ---- A and G rows of the tile into LDS; rows past P are zero ------------------------------------
        a_rows_to_lds(ha.A, t0, row1, s_ah, s_al);
        if constexpr (SMALL) {
            if (tid < DN) {   // one row per thread: db2 accumulates in its float4
                const int64_t g = t0 + tid;
                float v[DEF_SMALL_OUT] = {0.0f, 0.0f, 0.0f, 0.0f};
#pragma unroll
                for (int k = 0; k < DEF_SMALL_OUT; ++k)
                    if (k < nout && g < row1) v[k] = j.G[g * nout + k];
                const float4 gv = make_float4(v[0], v[1], v[2], v[3]);
                s_g4[tid] = gv;
                db2v.x += gv.x; db2v.y += gv.y; db2v.z += gv.z; db2v.w += gv.w;
            }
        } else {
            // G rows; a thread always holds column k = tid & 63 (256 is a multiple of 64), so db2, the
            // column sums of G, accumulate in its register (a per-tile loop of 64 dependent loads by
            // the nout threads serialised the whole block)
#pragma unroll
            for (int i = tid; i < DN * 64; i += 256) {
                const int rr = i >> 6, k = i & 63;
                const int64_t g = t0 + rr;
                const float v = (k < nout && g < row1) ? j.G[g * nout + k] : 0.0f;
                db2 += v;
                __bf16 hi, lo;
                dsplit(v, hi, lo);
                s_gh[rr * DGP + k] = hi;
                s_gl[rr * DGP + k] = lo;
            }
        }
        __syncthreads();
        // ---- Z1 for this wave's 32 columns (both row tiles), then dW2 and dZ1 ------------------------------
        uint32_t zpos = 0;   // bit 16 mt + q: Z1 > 0
        df32x16 d[2] = {df32x16{}, df32x16{}};
        {
            df32x16 z[2] = {df32x16{}, df32x16{}};
            mlp_ntile<DWID>(z, s_ah, s_al, DAP, wave, j.w1_h, j.w1_l);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const float zz = z[mt][q] + b1c;
                    zpos |= zz > 0.0f ? 1u << (16 * mt + q) : 0u;
                    z[mt][q] = fmaxf(zz, 0.0f);
                }
            if constexpr (SMALL) {
                // per row of the lane: dW2[k][col] += G[r][k] relu(Z1)[r][col], dZ1 = sum_k G[r][k] W2[k][col]
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const float4 gv = s_g4[row_of(mt, q, hh)];
                        const float zz = z[mt][q];
                        w2s[0] = __builtin_fmaf(gv.x, zz, w2s[0]); w2s[1] = __builtin_fmaf(gv.y, zz, w2s[1]);
                        w2s[2] = __builtin_fmaf(gv.z, zz, w2s[2]); w2s[3] = __builtin_fmaf(gv.w, zz, w2s[3]);
                        float dv = gv.x * w2c[0];
                        dv = __builtin_fmaf(gv.y, w2c[1], dv);
                        dv = __builtin_fmaf(gv.z, w2c[2], dv);
                        dv = __builtin_fmaf(gv.w, w2c[3], dv);
                        d[mt][q] = dv;
                    }
            } else {
#pragma unroll
                for (int ks = 0; ks < DN / 16; ++ks) {
                    dbf16x8 zh, zl;
                    wg_regs_to_op(z[ks >> 1], ks & 1, zh, zl);
#pragma unroll
                    for (int mo = 0; mo < 2; ++mo) {
                        if (mo >= Mo) break;
                        const dbf16x8 gh = wg_lds_op(s_gh, DGP, ks, 32 * mo), gl = wg_lds_op(s_gl, DGP, ks, 32 * mo);
                        w2acc[mo] = DMFMA(gh, zh, w2acc[mo]);
                        w2acc[mo] = DMFMA(gh, zl, w2acc[mo]);
                        w2acc[mo] = DMFMA(gl, zh, w2acc[mo]);
                    }
                }
            }
        }
        // ---- dZ1 = (G W2) [Z1 > 0] -> dW1 += dZ1^T A (rows 32 wave .. of dW1), db1 ------------------------
        {
            if constexpr (!SMALL) mlp_ntile<64>(d, s_gh, s_gl, DGP, wave, j.w2t_h, j.w2t_l);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    d[mt][q] = (zpos >> (16 * mt + q)) & 1u ? d[mt][q] : 0.0f;
                    db1 += d[mt][q];
                }
#pragma unroll
            for (int ks = 0; ks < DN / 16; ++ks) {
                dbf16x8 dh, dl;
                wg_regs_to_op(d[ks >> 1], ks & 1, dh, dl);
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
                    const dbf16x8 bh = wg_lds_op(s_ah, DAP, ks, 32 * nt), bl = wg_lds_op(s_al, DAP, ks, 32 * nt);
                    w1acc[nt] = DMFMA(dh, bh, w1acc[nt]);
                    w1acc[nt] = DMFMA(dh, bl, w1acc[nt]);
                    w1acc[nt] = DMFMA(dl, bh, w1acc[nt]);
                }
            }
        }
        __syncthreads();   // the tile's LDS rows read before the next tile overwrites them
    }
    // ---- the block's partial products: one atomic per element ------------------------------------------
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int m = 32 * wave + (q & 3) + 8 * (q >> 2) + 4 * hh;
            atomicAdd(j.dW1 + (size_t)m * DWID + 32 * nt + r, w1acc[nt][q]);
        }
    db1 += __shfl_xor(db1, 32);
    if (hh == 0) atomicAdd(j.db1 + col, db1);
    if constexpr (SMALL) {
#pragma unroll
        for (int k = 0; k < DEF_SMALL_OUT; ++k) {
            const float v = w2s[k] + __shfl_xor(w2s[k], 32);   // the lane pair holds the column's two row halves
            if (hh == 0 && k < nout) atomicAdd(j.dW2 + (size_t)k * DWID + col, v);
        }
        if (wave == 0) {   // db2: the 64 row threads' sums
            float v[DEF_SMALL_OUT] = {db2v.x, db2v.y, db2v.z, db2v.w};
#pragma unroll
            for (int k = 0; k < DEF_SMALL_OUT; ++k) {
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) v[k] += __shfl_xor(v[k], off);
                if (lane == 0 && k < nout) atomicAdd(j.db2 + k, v[k]);
            }
        }
    } else {
#pragma unroll
        for (int mo = 0; mo < 2; ++mo) {
            if (mo >= Mo) break;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int o = 32 * mo + (q & 3) + 8 * (q >> 2) + 4 * hh;
                if (o < nout) atomicAdd(j.dW2 + (size_t)o * DWID + col, w2acc[mo][q]);
            }
        }
        if ((tid & 63) < nout) atomicAdd(j.db2 + (tid & 63), db2);   // one partial per wave
    }
}

// Version 2 (round 6): the same products at ONE wave per SIMD, with what version 1 re-read per 64-row
// tile held in registers for the whole block -- the wave's W1 fragments (its 32 columns, K = 128: 64
// registers) and, for the wide heads, its W2^T fragments (K = 64: 32 registers) -- and the next tile's
// A and G rows loaded into registers while the current tile computes (version 1 waited on an L2 round
// trip of 64 KB of weight fragments and one of the tile's rows per tile, at 2 waves per SIMD with no
// registers left to prefetch).  The accumulators move to AGPRs (512 registers per wave at one wave
// per SIMD).  Blocks: 64 per small head (the four share each row range on one XCD: grid x is a
// multiple of 8, so their A reads meet in that XCD's L2) and 256 for a wide head, one round of 256
// CUs each.
template <bool SMALL>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) k_head_wgrad2(HeadWgradArgs ha, int job0) {
    __shared__ __attribute__((aligned(16))) __bf16 s_ah[DN * DAP];   // A rows [64][128] hi / lo
    __shared__ __attribute__((aligned(16))) __bf16 s_al[DN * DAP];
    __shared__ __attribute__((aligned(16))) __bf16 s_gh[SMALL ? 8 : DN * DGP];   // G rows [64][64 pad] hi / lo
    __shared__ __attribute__((aligned(16))) __bf16 s_gl[SMALL ? 8 : DN * DGP];
    __shared__ __attribute__((aligned(16))) float4 s_g4[SMALL ? DN : 1];        // SMALL: G rows fp32
    __shared__ __attribute__((aligned(16))) __bf16 s_w2h[SMALL ? 8 : DWID * DLP];   // !SMALL: W2^T [128][64 pad]
    __shared__ __attribute__((aligned(16))) __bf16 s_w2l[SMALL ? 8 : DWID * DLP];
    LDS_POISON(s_ah); LDS_POISON(s_al); LDS_POISON(s_gh); LDS_POISON(s_gl); LDS_POISON(s_g4); LDS_POISON(s_w2h);
    LDS_POISON(s_w2l); LDS_POISON_DONE();
    typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
    const HeadWgradJob& j = ha.job[job0 + blockIdx.y];
    const int64_t row0 = (int64_t)blockIdx.x * ha.rows_per_block;
    const int64_t row1 = min((int64_t)ha.P, row0 + ha.rows_per_block);
    if (row0 >= row1) return;                                            // block-uniform
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
    const int nout = j.nout, Mo = (nout + 31) / 32;                      // G^T M tiles (1 or 2)
    const int col = 32 * wave + r;
    const float b1c = j.b1[col];
    // ---- the wave's weight fragments, once per block ---------------------------------------------------
    dbf16x8 w1h[DWID / 16], w1l[DWID / 16];
#pragma unroll
    for (int ks = 0; ks < DWID / 16; ++ks) {
        const size_t wo = (size_t)col * DWID + 16 * ks + 8 * hh;
        w1h[ks] = *reinterpret_cast<const dbf16x8*>(j.w1_h + wo);
        w1l[ks] = *reinterpret_cast<const dbf16x8*>(j.w1_l + wo);
    }
    if constexpr (!SMALL) {   // the wide head's W2^T in LDS (registers would spill), visible after the first barrier
        for (int i = tid; i < DWID * 64 / 8; i += 256) {
            const int rr = i >> 3, c8 = (i & 7) * 8;
            *reinterpret_cast<dbf16x8*>(s_w2h + rr * DLP + c8) = *reinterpret_cast<const dbf16x8*>(j.w2t_h + rr * 64 + c8);
            *reinterpret_cast<dbf16x8*>(s_w2l + rr * DLP + c8) = *reinterpret_cast<const dbf16x8*>(j.w2t_l + rr * 64 + c8);
        }
    }
    df32x16 w1acc[4] = {df32x16{}, df32x16{}, df32x16{}, df32x16{}};   // dW1 rows 32 wave .., col tiles 0..3
    df32x16 w2acc[SMALL ? 1 : 2];                                         // dW2 o tiles 0..1, col tile wave
    float w2s[DEF_SMALL_OUT] = {0.0f, 0.0f, 0.0f, 0.0f};                 // SMALL: dW2 rows 0..3, column col
    float w2c[DEF_SMALL_OUT] = {0.0f, 0.0f, 0.0f, 0.0f};                 // SMALL: W2 rows 0..3, column col
    float4 db2v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if constexpr (SMALL) w2_column(j.w2_h, j.w2_l, col, w2c);
    else { w2acc[0] = df32x16{}; w2acc[1] = df32x16{}; }
    float db1 = 0.0f, db2 = 0.0f;
    // ---- the tile's rows in registers: A (thread: 8 float4 of rows (tid + 256 i) >> 5), G ---------------
    float4 pa[DN * DWID / 4 / 256];
    float pg[SMALL ? DEF_SMALL_OUT : DN * 64 / 256];
    auto load_tile = [&](int64_t t0) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < DN * DWID / 4 / 256; ++i) {
            const int e = tid + 256 * i, rr = e >> 5, c4 = (e & 31) * 4;
            const int64_t g = t0 + rr;
            pa[i] = g < row1 ? *reinterpret_cast<const float4*>(ha.A + g * DWID + c4) : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
        if constexpr (SMALL) {
            const int64_t g = t0 + tid;
#pragma unroll
            for (int k = 0; k < DEF_SMALL_OUT; ++k) pg[k] = (tid < DN && k < nout && g < row1) ? j.G[g * nout + k] : 0.0f;
        } else {
#pragma unroll
            for (int i = 0; i < DN * 64 / 256; ++i) {
                const int e = tid + 256 * i, rr = e >> 6, k = e & 63;
                const int64_t g = t0 + rr;
                pg[i] = (k < nout && g < row1) ? j.G[g * nout + k] : 0.0f;
            }
        }
    };
    auto store_tile = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < DN * DWID / 4 / 256; ++i) {
            const int e = tid + 256 * i, rr = e >> 5, c4 = (e & 31) * 4;
            const float f[4] = {pa[i].x, pa[i].y, pa[i].z, pa[i].w};
            bf4 h4, l4;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                __bf16 hi, lo;
                dsplit(f[q], hi, lo);
                h4[q] = hi; l4[q] = lo;
            }
            *reinterpret_cast<bf4*>(s_ah + rr * DAP + c4) = h4;
            *reinterpret_cast<bf4*>(s_al + rr * DAP + c4) = l4;
        }
        if constexpr (SMALL) {
            if (tid < DN) {
                const float4 gv = make_float4(pg[0], pg[1], pg[2], pg[3]);
                s_g4[tid] = gv;
                db2v.x += gv.x; db2v.y += gv.y; db2v.z += gv.z; db2v.w += gv.w;
            }
        } else {
#pragma unroll
            for (int i = 0; i < DN * 64 / 256; ++i) {   // column k = tid & 63 for every i: db2 in a register
                const int e = tid + 256 * i, rr = e >> 6, k = e & 63;
                db2 += pg[i];
                __bf16 hi, lo;
                dsplit(pg[i], hi, lo);
                s_gh[rr * DGP + k] = hi;
                s_gl[rr * DGP + k] = lo;
            }
        }
    };
    load_tile(row0);
    for (int64_t t0 = row0; t0 < row1; t0 += DN) {
        store_tile();
        __syncthreads();
        if (t0 + DN < row1) load_tile(t0 + DN);   // in flight while this tile computes
        // ---- Z1 for this wave's 32 columns (both row tiles), then dW2 and dZ1 ------------------------------
        uint32_t zpos = 0;   // bit 16 mt + q: Z1 > 0
        df32x16 d[2] = {df32x16{}, df32x16{}};
        {
            df32x16 z[2] = {df32x16{}, df32x16{}};
#pragma unroll
            for (int ks = 0; ks < DWID / 16; ++ks) {
                const int k0 = 16 * ks + 8 * hh;
#pragma unroll
                for (int mt = 0; mt < 2; ++mt) {
                    const dbf16x8 ah = *reinterpret_cast<const dbf16x8*>(s_ah + (32 * mt + r) * DAP + k0);
                    const dbf16x8 al = *reinterpret_cast<const dbf16x8*>(s_al + (32 * mt + r) * DAP + k0);
                    z[mt] = DMFMA(ah, w1h[ks], z[mt]);
                    z[mt] = DMFMA(ah, w1l[ks], z[mt]);
                    z[mt] = DMFMA(al, w1h[ks], z[mt]);
                }
            }
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    const float zz = z[mt][q] + b1c;
                    zpos |= zz > 0.0f ? 1u << (16 * mt + q) : 0u;
                    z[mt][q] = fmaxf(zz, 0.0f);
                }
            if constexpr (SMALL) {
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int q = 0; q < 16; ++q) {
                        const float4 gv = s_g4[row_of(mt, q, hh)];
                        const float zz = z[mt][q];
                        w2s[0] = __builtin_fmaf(gv.x, zz, w2s[0]); w2s[1] = __builtin_fmaf(gv.y, zz, w2s[1]);
                        w2s[2] = __builtin_fmaf(gv.z, zz, w2s[2]); w2s[3] = __builtin_fmaf(gv.w, zz, w2s[3]);
                        float dv = gv.x * w2c[0];
                        dv = __builtin_fmaf(gv.y, w2c[1], dv);
                        dv = __builtin_fmaf(gv.z, w2c[2], dv);
                        dv = __builtin_fmaf(gv.w, w2c[3], dv);
                        d[mt][q] = dv;
                    }
            } else {
#pragma unroll
                for (int ks = 0; ks < DN / 16; ++ks) {
                    dbf16x8 zh, zl;
                    wg_regs_to_op(z[ks >> 1], ks & 1, zh, zl);
#pragma unroll
                    for (int mo = 0; mo < 2; ++mo) {
                        if (mo >= Mo) break;
                        const dbf16x8 gh = wg_lds_op(s_gh, DGP, ks, 32 * mo), gl = wg_lds_op(s_gl, DGP, ks, 32 * mo);
                        w2acc[mo] = DMFMA(gh, zh, w2acc[mo]);
                        w2acc[mo] = DMFMA(gh, zl, w2acc[mo]);
                        w2acc[mo] = DMFMA(gl, zh, w2acc[mo]);
                    }
                }
            }
        }
        // ---- dZ1 = (G W2) [Z1 > 0] -> dW1 += dZ1^T A (rows 32 wave .. of dW1), db1 ------------------------
        {
            if constexpr (!SMALL) {
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const int k0 = 16 * ks + 8 * hh;
                    const dbf16x8 w2h = *reinterpret_cast<const dbf16x8*>(s_w2h + col * DLP + k0);
                    const dbf16x8 w2l = *reinterpret_cast<const dbf16x8*>(s_w2l + col * DLP + k0);
#pragma unroll
                    for (int mt = 0; mt < 2; ++mt) {
                        const dbf16x8 gh = *reinterpret_cast<const dbf16x8*>(s_gh + (32 * mt + r) * DGP + k0);
                        const dbf16x8 gl = *reinterpret_cast<const dbf16x8*>(s_gl + (32 * mt + r) * DGP + k0);
                        d[mt] = DMFMA(gh, w2h, d[mt]);
                        d[mt] = DMFMA(gh, w2l, d[mt]);
                        d[mt] = DMFMA(gl, w2h, d[mt]);
                    }
                }
            }
#pragma unroll
            for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                for (int q = 0; q < 16; ++q) {
                    d[mt][q] = (zpos >> (16 * mt + q)) & 1u ? d[mt][q] : 0.0f;
                    db1 += d[mt][q];
                }
#pragma unroll
            for (int ks = 0; ks < DN / 16; ++ks) {
                dbf16x8 dh, dl;
                wg_regs_to_op(d[ks >> 1], ks & 1, dh, dl);
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
                    const dbf16x8 bh = wg_lds_op(s_ah, DAP, ks, 32 * nt), bl = wg_lds_op(s_al, DAP, ks, 32 * nt);
                    w1acc[nt] = DMFMA(dh, bh, w1acc[nt]);
                    w1acc[nt] = DMFMA(dh, bl, w1acc[nt]);
                    w1acc[nt] = DMFMA(dl, bh, w1acc[nt]);
                }
            }
        }
        __syncthreads();   // the tile's LDS rows read before the next tile's are stored
    }
    // ---- the block's partial products: one atomic per element (as version 1) ---------------------------
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int m = 32 * wave + (q & 3) + 8 * (q >> 2) + 4 * hh;
            atomicAdd(j.dW1 + (size_t)m * DWID + 32 * nt + r, w1acc[nt][q]);
        }
    db1 += __shfl_xor(db1, 32);
    if (hh == 0) atomicAdd(j.db1 + col, db1);
    if constexpr (SMALL) {
#pragma unroll
        for (int k = 0; k < DEF_SMALL_OUT; ++k) {
            const float v = w2s[k] + __shfl_xor(w2s[k], 32);
            if (hh == 0 && k < nout) atomicAdd(j.dW2 + (size_t)k * DWID + col, v);
        }
        if (wave == 0) {
            float v[DEF_SMALL_OUT] = {db2v.x, db2v.y, db2v.z, db2v.w};
#pragma unroll
            for (int k = 0; k < DEF_SMALL_OUT; ++k) {
#pragma unroll
                for (int off = 32; off >= 1; off >>= 1) v[k] += __shfl_xor(v[k], off);
                if (lane == 0 && k < nout) atomicAdd(j.db2 + k, v[k]);
            }
        }
    } else {
#pragma unroll
        for (int mo = 0; mo < 2; ++mo) {
            if (mo >= Mo) break;
#pragma unroll
            for (int q = 0; q < 16; ++q) {
                const int o = 32 * mo + (q & 3) + 8 * (q >> 2) + 4 * hh;
                if (o < nout) atomicAdd(j.dW2 + (size_t)o * DWID + col, w2acc[mo][q]);
            }
        }
        if ((tid & 63) < nout) atomicAdd(j.db2 + (tid & 63), db2);
    }
}

// Version 3 (round 6, the small heads): version 2's products software-pipelined across tiles so that
// one wave per SIMD keeps its matrix core fed.  Three LDS tile buffers; iteration t runs
//   A: Z1 of tile t + 1 (MFMA, buffer t + 1)  beside  relu / dZ1 / dW2 of tile t (VALU, Z1(t) in registers)
//   B: dW1 += dZ1(t)^T A(t) (MFMA, buffer t)   beside  tile t + 2's rows into buffer t + 2 (VALU + LDS stores)
// then tile t + 3's rows are loaded into registers and one barrier ends the iteration (buffer t is
// free for tile t + 3, tile t + 2 is visible).  An iteration is branch-free (loads at clamped rows,
// zeros selected past the block's rows; Z1 past the last tile is computed and dropped) and each stage
// interleaves its two chains by hand, K step by K step, fenced by sched_barrier (sched_group_barrier
// patterns did not take: the compiler hoisted the VALU chain out of the MFMA region).  Version 2 ran
// the chains one after the other: 2.27 -> 2.03 ms for the four small heads at 2M.  W1's lo half sits
// in LDS (registers hold the hi half) so that nothing spills.
template <bool SMALL>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) k_head_wgrad3(HeadWgradArgs ha, int job0) {
    static_assert(SMALL, "version 3 covers the heads of at most DEF_SMALL_OUT outputs");
    constexpr int NB = 3;
    __shared__ __attribute__((aligned(16))) __bf16 s_ah[NB][DN * DAP];   // A rows [64][128] hi / lo
    __shared__ __attribute__((aligned(16))) __bf16 s_al[NB][DN * DAP];
    __shared__ __attribute__((aligned(16))) float4 s_g4[NB][DN];         // G rows fp32
    __shared__ __attribute__((aligned(16))) __bf16 s_w1l[DWID * DAP];    // W1 lo [128][128] (hi in registers)
    LDS_POISON(s_ah); LDS_POISON(s_al); LDS_POISON(s_g4); LDS_POISON(s_w1l); LDS_POISON_DONE();
    typedef __bf16 bf4 __attribute__((ext_vector_type(4)));
    const HeadWgradJob& j = ha.job[job0 + blockIdx.y];
    const int64_t row0 = (int64_t)blockIdx.x * ha.rows_per_block;
    const int64_t row1 = min((int64_t)ha.P, row0 + ha.rows_per_block);
    if (row0 >= row1) return;                                            // block-uniform
    const int T = (int)((row1 - row0 + DN - 1) / DN);                    // tiles of this block
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63, r = lane & 31, hh = lane >> 5;
    const int nout = j.nout;
    const int col = 32 * wave + r;
    const float b1c = j.b1[col];
    dbf16x8 w1h[DWID / 16];
#pragma unroll
    for (int ks = 0; ks < DWID / 16; ++ks)
        w1h[ks] = *reinterpret_cast<const dbf16x8*>(j.w1_h + (size_t)col * DWID + 16 * ks + 8 * hh);
    for (int i = tid; i < DWID * DWID / 8; i += 256) {   // visible after the prologue's barrier
        const int rr = i >> 4, c8 = (i & 15) * 8;
        *reinterpret_cast<dbf16x8*>(&s_w1l[rr * DAP + c8]) = *reinterpret_cast<const dbf16x8*>(j.w1_l + rr * DWID + c8);
    }
    df32x16 w1acc[4] = {df32x16{}, df32x16{}, df32x16{}, df32x16{}};
    float w2s[DEF_SMALL_OUT] = {0.0f, 0.0f, 0.0f, 0.0f};
    float w2c[DEF_SMALL_OUT] = {0.0f, 0.0f, 0.0f, 0.0f};
    float4 db2v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    w2_column(j.w2_h, j.w2_l, col, w2c);
    float db1 = 0.0f;
    float4 pa[DN * DWID / 4 / 256];
    float pg[DEF_SMALL_OUT];
    // branch-free (so that an iteration stays one scheduling region): every load is issued at a clamped
    // row and rows past row1 (tiles past the block's last included) are selected to zero
    auto load_tile = [&](int t) __attribute__((always_inline)) {
        const int64_t t0 = row0 + (int64_t)t * DN;
#pragma unroll
        for (int i = 0; i < DN * DWID / 4 / 256; ++i) {
            const int e = tid + 256 * i, rr = e >> 5, c4 = (e & 31) * 4;
            const int64_t g = t0 + rr;
            const float4 v = *reinterpret_cast<const float4*>(ha.A + min(g, row1 - 1) * DWID + c4);
            const bool ok = g < row1;
            pa[i] = make_float4(ok ? v.x : 0.0f, ok ? v.y : 0.0f, ok ? v.z : 0.0f, ok ? v.w : 0.0f);
        }
        const int64_t g = t0 + (tid & (DN - 1));
#pragma unroll
        for (int k = 0; k < DEF_SMALL_OUT; ++k) {
            const float v = j.G[min(g, row1 - 1) * nout + min(k, nout - 1)];
            pg[k] = (tid < DN && k < nout && g < row1) ? v : 0.0f;
        }
    };
    auto store_tile = [&](int b) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < DN * DWID / 4 / 256; ++i) {
            const int e = tid + 256 * i, rr = e >> 5, c4 = (e & 31) * 4;
            const float f[4] = {pa[i].x, pa[i].y, pa[i].z, pa[i].w};
            bf4 h4, l4;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                __bf16 hi, lo;
                dsplit(f[q], hi, lo);
                h4[q] = hi; l4[q] = lo;
            }
            *reinterpret_cast<bf4*>(&s_ah[b][rr * DAP + c4]) = h4;
            *reinterpret_cast<bf4*>(&s_al[b][rr * DAP + c4]) = l4;
        }
        if (tid < DN) {
            const float4 gv = make_float4(pg[0], pg[1], pg[2], pg[3]);
            s_g4[b][tid] = gv;
            db2v.x += gv.x; db2v.y += gv.y; db2v.z += gv.z; db2v.w += gv.w;
        }
    };
    auto z1 = [&](int b, df32x16 (&z)[2]) __attribute__((always_inline)) {
        z[0] = df32x16{}; z[1] = df32x16{};
#pragma unroll
        for (int ks = 0; ks < DWID / 16; ++ks) {
            const int k0 = 16 * ks + 8 * hh;
            const dbf16x8 wl = *reinterpret_cast<const dbf16x8*>(&s_w1l[col * DAP + k0]);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                const dbf16x8 ah = *reinterpret_cast<const dbf16x8*>(&s_ah[b][(32 * mt + r) * DAP + k0]);
                const dbf16x8 al = *reinterpret_cast<const dbf16x8*>(&s_al[b][(32 * mt + r) * DAP + k0]);
                z[mt] = DMFMA(ah, w1h[ks], z[mt]);
                z[mt] = DMFMA(ah, wl, z[mt]);
                z[mt] = DMFMA(al, w1h[ks], z[mt]);
            }
        }
    };
    // one element of dz1 (e = 16 mt + q)
    auto dz1_elem = [&](int b, const df32x16 (&z)[2], df32x16 (&d)[2], int mt, int q) __attribute__((always_inline)) {
        const float zz = z[mt][q] + b1c;
        const float zr = fmaxf(zz, 0.0f);
        const float4 gv = s_g4[b][row_of(mt, q, hh)];
        w2s[0] = __builtin_fmaf(gv.x, zr, w2s[0]); w2s[1] = __builtin_fmaf(gv.y, zr, w2s[1]);
        w2s[2] = __builtin_fmaf(gv.z, zr, w2s[2]); w2s[3] = __builtin_fmaf(gv.w, zr, w2s[3]);
        float dv = gv.x * w2c[0];
        dv = __builtin_fmaf(gv.y, w2c[1], dv);
        dv = __builtin_fmaf(gv.z, w2c[2], dv);
        dv = __builtin_fmaf(gv.w, w2c[3], dv);
        dv = zz > 0.0f ? dv : 0.0f;
        db1 += dv;
        d[mt][q] = dv;
    };
    // row chunk i (of 8) of store_tile's A rows, and the G row with chunk 0
    auto store_part = [&](int b, int i) __attribute__((always_inline)) {
        const int e = tid + 256 * i, rr = e >> 5, c4 = (e & 31) * 4;
        const float f[4] = {pa[i].x, pa[i].y, pa[i].z, pa[i].w};
        bf4 h4, l4;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            __bf16 hi, lo;
            dsplit(f[q], hi, lo);
            h4[q] = hi; l4[q] = lo;
        }
        *reinterpret_cast<bf4*>(&s_ah[b][rr * DAP + c4]) = h4;
        *reinterpret_cast<bf4*>(&s_al[b][rr * DAP + c4]) = l4;
        if (i == 0 && tid < DN) {
            const float4 gv = make_float4(pg[0], pg[1], pg[2], pg[3]);
            s_g4[b][tid] = gv;
            db2v.x += gv.x; db2v.y += gv.y; db2v.z += gv.z; db2v.w += gv.w;
        }
    };
    // ---- prologue: tiles 0 and 1 in LDS, tile 2's rows in registers, Z1 of tile 0 --------------------------
    load_tile(0);
    store_tile(0);
    load_tile(1);
    store_tile(1);
    load_tile(2);
    __syncthreads();
    df32x16 zc[2];
    z1(0, zc);
    for (int t = 0; t < T; ++t) {
        // one scheduling region per iteration: past the block's last tiles, Z1 runs on a buffer whose
        // result is dropped and stage B stores zero rows (load_tile's selects), so nothing branches
        const int b0 = t % NB, b1 = (t + 1) % NB, b2 = (t + 2) % NB;
        df32x16 d[2];
        df32x16 zn[2];
        // stage A: Z1(t + 1) on the matrix core, tile t's relu / dZ1 / dW2 on the VALU, interleaved by
        // hand (4 of the 32 per-lane elements after each K step's 6 MFMAs; sched_barrier keeps the chunks)
        zn[0] = df32x16{}; zn[1] = df32x16{};
#pragma unroll
        for (int ks = 0; ks < DWID / 16; ++ks) {
            const int k0 = 16 * ks + 8 * hh;
            const dbf16x8 wl = *reinterpret_cast<const dbf16x8*>(&s_w1l[col * DAP + k0]);
#pragma unroll
            for (int mt = 0; mt < 2; ++mt) {
                const dbf16x8 ah = *reinterpret_cast<const dbf16x8*>(&s_ah[b1][(32 * mt + r) * DAP + k0]);
                const dbf16x8 al = *reinterpret_cast<const dbf16x8*>(&s_al[b1][(32 * mt + r) * DAP + k0]);
                zn[mt] = DMFMA(ah, w1h[ks], zn[mt]);
                zn[mt] = DMFMA(ah, wl, zn[mt]);
                zn[mt] = DMFMA(al, w1h[ks], zn[mt]);
            }
#pragma unroll
            for (int e = 4 * ks; e < 4 * ks + 4; ++e) dz1_elem(b0, zc, d, e >> 4, e & 15);
            __builtin_amdgcn_sched_barrier(0);
        }
        // stage B: dW1(t) on the matrix core, tile t + 2's rows into LDS on the VALU (2 row chunks per K step)
#pragma unroll
        for (int ks = 0; ks < DN / 16; ++ks) {
            dbf16x8 dh, dl;
            wg_regs_to_op(d[ks >> 1], ks & 1, dh, dl);
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const dbf16x8 bh = wg_lds_op(s_ah[b0], DAP, ks, 32 * nt), bl = wg_lds_op(s_al[b0], DAP, ks, 32 * nt);
                w1acc[nt] = DMFMA(dh, bh, w1acc[nt]);
                w1acc[nt] = DMFMA(dh, bl, w1acc[nt]);
                w1acc[nt] = DMFMA(dl, bh, w1acc[nt]);
            }
            store_part(b2, 2 * ks);
            store_part(b2, 2 * ks + 1);
            __builtin_amdgcn_sched_barrier(0);
        }
        load_tile(t + 3);
        __syncthreads();
        zc[0] = zn[0]; zc[1] = zn[1];
    }
    // ---- the block's partial products: one atomic per element (as version 1) ---------------------------
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int q = 0; q < 16; ++q) {
            const int m = 32 * wave + (q & 3) + 8 * (q >> 2) + 4 * hh;
            atomicAdd(j.dW1 + (size_t)m * DWID + 32 * nt + r, w1acc[nt][q]);
        }
    db1 += __shfl_xor(db1, 32);
    if (hh == 0) atomicAdd(j.db1 + col, db1);
#pragma unroll
    for (int k = 0; k < DEF_SMALL_OUT; ++k) {
        const float v = w2s[k] + __shfl_xor(w2s[k], 32);
        if (hh == 0 && k < nout) atomicAdd(j.dW2 + (size_t)k * DWID + col, v);
    }
    if (wave == 0) {
        float v[DEF_SMALL_OUT] = {db2v.x, db2v.y, db2v.z, db2v.w};
#pragma unroll
        for (int k = 0; k < DEF_SMALL_OUT; ++k) {
#pragma unroll
            for (int off = 32; off >= 1; off >>= 1) v[k] += __shfl_xor(v[k], off);
            if (lane == 0 && k < nout) atomicAdd(j.db2 + k, v[k]);
        }
    }
}

// Rows per block of a launch, for about `blocks` blocks per head: 128 for the small-output heads
// (their per-block flush of dW1 / dW2 partials is most of their atomics), 400 for the SH head.
// Measured against the split-K default of 256 blocks per head: deformation backward 11.96-11.99
// -> 11.20-11.21 ms at 2M, configs[4] stand-in 1.449-1.454 -> 1.391-1.400 ms per iteration.
// LSR_WGRAD_ROWS_SMALL / LSR_WGRAD_ROWS_BIG override (diagnostic A/B).
static int wgrad_rows(const char* env, int P, int blocks) {
    const char* e = std::getenv(env);
    const int r = e ? std::atoi(e) : 0;
    if (r >= 64) return r / 64 * 64;
    return std::max(64, ((P + blocks - 1) / blocks + 63) / 64 * 64);
}
void launch_head_wgrad(const HeadWgradArgs& a, int njobs, hipStream_t st) {
    if (a.P <= 0 || njobs <= 0) return;
    // the small-output heads first (one launch), then the rest: jobs are reordered into two runs
    HeadWgradArgs s = a;
    int ns = 0, nbig = 0;
    for (int i = 0; i < njobs; ++i)
        if (a.job[i].nout <= DEF_SMALL_OUT) s.job[ns++] = a.job[i];
    for (int i = 0; i < njobs; ++i)
        if (a.job[i].nout > DEF_SMALL_OUT) { s.job[ns + nbig] = a.job[i]; ++nbig; }
    // version 3 for the small heads, 2 for the wide by default (2M backward 10.10 -> 9.34 (v2) -> 9.13-9.15 ms);
    // LSR_WGRAD_V=1 / 2: the earlier versions (diagnostic A/B)
    static const int ver = [] { const char* e = std::getenv("LSR_WGRAD_V"); return e ? std::atoi(e) : 3; }();
    if (ver >= 2) {   // one round of 256 CUs per launch: 64 blocks per small head, 256 for a wide head
        if (ns) {
            const int nb = ns <= 4 ? 256 / ns / 8 * 8 : 32;
            s.rows_per_block = std::max(64, ((a.P + nb - 1) / nb + 63) / 64 * 64);
            const dim3 grid((a.P + s.rows_per_block - 1) / s.rows_per_block, ns);
            if (ver == 3) hipLaunchKernelGGL(k_head_wgrad3<true>, grid, dim3(256), 0, st, s, 0);
            else hipLaunchKernelGGL(k_head_wgrad2<true>, grid, dim3(256), 0, st, s, 0);
        }
        if (nbig) {
            const int nb = std::max(8, 256 / nbig / 8 * 8);
            s.rows_per_block = std::max(64, ((a.P + nb - 1) / nb + 63) / 64 * 64);
            hipLaunchKernelGGL(k_head_wgrad2<false>, dim3((a.P + s.rows_per_block - 1) / s.rows_per_block, nbig),
                               dim3(256), 0, st, s, ns);
        }
        return;
    }
    if (ns) {
        s.rows_per_block = wgrad_rows("LSR_WGRAD_ROWS_SMALL", a.P, 128);
        const int nb = (a.P + s.rows_per_block - 1) / s.rows_per_block;
        hipLaunchKernelGGL(k_head_wgrad<true>, dim3(nb, ns), dim3(256), 0, st, s, 0);
    }
    if (nbig) {
        s.rows_per_block = wgrad_rows("LSR_WGRAD_ROWS_BIG", a.P, 400);
        const int nb = (a.P + s.rows_per_block - 1) / s.rows_per_block;
        hipLaunchKernelGGL(k_head_wgrad<false>, dim3(nb, nbig), dim3(256), 0, st, s, ns);
    }
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
    AtbArgs s = a;
    if (const char* e = std::getenv("LSR_ATB_BLOCKS")) {   // diagnostic A/B: blocks per job
        const int nbt = std::max(1, std::atoi(e));
        s.rows_per_block = std::max(64, ((a.P + nbt - 1) / nbt + 63) / 64 * 64);
    }
    const int nb = (s.P + s.rows_per_block - 1) / s.rows_per_block;
    hipLaunchKernelGGL(k_atb, dim3(nb, njobs), dim3(256), 0, st, s);
}

// packed channel-last gradient replicas [r][H][W][16] -> torch [16][H][W], summed over the replicas
// and added, every plane of a call in one launch (one per plane was 12 launches of ~10 us each at
// the Neu3D planes, mostly launch gaps).  One block per 16 texels (256 floats): each thread sums one
// float over the replicas with coalesced reads, the block transposes through LDS (pitch 17) and
// writes each channel's 16 texels as one 64-byte run.  (A thread per destination float read
// 64-byte-strided words of every replica: 0.38 ms per training iteration at configs[4]'s planes.)
// One extra block folds the box gradient's partial rows.
__global__ void __launch_bounds__(256) k_unpack_planes(const UnpackBatch u) {
    __shared__ float s_t[16][17];
    const int bid = blockIdx.x, t = threadIdx.x;
    if (bid == u.block0[u.n]) {   // block-uniform: the box gradient
        if (t < 6) {
            float acc = 0.0f;
            for (int r = 0; r < DEF_AABB_SLOTS; ++r) acc += u.daabb_part[r * 16 + t];
            u.daabb[t] += acc;
        }
        return;
    }
    LDS_POISON(s_t); LDS_POISON_DONE();
    int j = 0;
    while (j + 1 < u.n && bid >= u.block0[j + 1]) ++j;
    const int H = u.H[j], W = u.W[j], HW = H * W, base = (bid - u.block0[j]) * 16;
    const int tex = t >> 4, ch = t & 15;
    float acc = 0.0f;
    if (base + tex < HW) {
        const float* p = u.src + u.off[j] + (size_t)base * 16 + t;
        for (int r = 0; r < u.replicas; ++r) acc += p[(size_t)r * u.stride];
    }
    if (u.trow && u.toff[j] >= 0 && base + tex < HW) {   // block-uniform plane: its x-row, folded into
        // the two rows of time0 (tap_of's arithmetic for the time coordinate)
        const float iy = fminf(fmaxf((u.time0[0] + 1.0f) * 0.5f * (float)(H - 1), 0.0f), (float)(H - 1));
        const int y0 = (int)floorf(iy), y1 = min(y0 + 1, H - 1);
        const float fy = iy - (float)y0;
        const int y = (base + tex) / W, x = (base + tex) - y * W;
        if (y == y0 || y == y1) {
            float r = 0.0f;
            const float* rp = u.trow + u.toff[j] + x * 16 + ch;
            for (int k = 0; k < u.trow_reps; ++k) r += rp[(size_t)k * u.trow_stride];
            if (y == y0) acc += r * (1.0f - fy);
            if (y == y1) acc += r * fy;
        }
    }
    s_t[tex][ch] = acc;
    __syncthreads();
    const int c = t >> 4, tl = t & 15;
    if (base + tl < HW) u.dst[j][(size_t)c * HW + base + tl] += s_t[tl][c];
}

void launch_unpack_planes(const UnpackBatch& u, hipStream_t st) {
    const int nb = u.block0[u.n] + (u.daabb ? 1 : 0);
    if (nb > 0) hipLaunchKernelGGL(k_unpack_planes, dim3(nb), dim3(256), 0, st, u);
}

// ---- parameter packing ----------------------------------------------------------------------------
// plane [C=16][H][W] (torch) -> [H][W][16]
__global__ void k_pack_plane(const float* __restrict__ src, float* __restrict__ dst, int H, int W) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;   // over H * W * 16 destination floats
    if (i >= H * W * 16) return;
    const int c = i & 15, hw = i >> 4;
    dst[i] = src[(size_t)c * H * W + hw];
}

// fp32 [rows][cols] -> bf16 hi / lo [rows_pad][cols_pad], zero past `rows` / `cols`
__global__ void k_pack_weight(const float* __restrict__ src, __bf16* __restrict__ hi, __bf16* __restrict__ lo,
                              int rows, int rows_pad, int cols, int cols_pad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows_pad * cols_pad) return;
    const int r = i / cols_pad, c = i - r * cols_pad;
    const float v = (r < rows && c < cols) ? src[(size_t)r * cols + c] : 0.0f;
    __bf16 h, l;
    dsplit(v, h, l);
    hi[i] = h;
    lo[i] = l;
}

// fp32 [rows][cols] -> bf16 hi / lo [cols_pad][k_pad], dst[c][r] = src[r][c], zero for r >= rows, c >= cols
__global__ void k_pack_weight_t(const float* __restrict__ src, __bf16* __restrict__ hi, __bf16* __restrict__ lo,
                                int rows, int cols, int k_pad, int cols_pad) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= cols_pad * k_pad) return;
    const int c = i / k_pad, r = i - c * k_pad;
    const float v = (r < rows && c < cols) ? src[(size_t)r * cols + c] : 0.0f;
    __bf16 h, l;
    dsplit(v, h, l);
    hi[i] = h;
    lo[i] = l;
}

void launch_pack_weight_t(const float* src, __bf16* hi, __bf16* lo, int rows, int cols, int k_pad, int cols_pad,
                          hipStream_t st) {
    hipLaunchKernelGGL(k_pack_weight_t, dim3((cols_pad * k_pad + 255) / 256), dim3(256), 0, st, src, hi, lo, rows, cols,
                       k_pad, cols_pad);
}

// Every packing job of lsr_deform_prepare (planes, weights, transposed weights: ~34 per field) in
// one launch: block b runs job j where first[j] <= b < first[j + 1] (a scalar search over <= 48
// jobs); the element work is that of the single-job kernels above.  (One launch per job left the
// device idle between ~34 tiny kernels every training iteration.)
__global__ void __launch_bounds__(256) k_pack_batch(PackBatch pb) {
    const uint32_t b = blockIdx.x;
    int j = 0;
    while (j + 1 < pb.n && b >= pb.j[j + 1].first_block) ++j;
    const PackJob& q = pb.j[j];
    const int i = (int)(b - q.first_block) * 256 + (int)threadIdx.x;
    if (q.kind == PACK_PLANE) {   // [16][H][W] -> [H][W][16]; a = H * W
        if (i >= q.a * 16) return;
        reinterpret_cast<float*>(q.hi)[i] = q.src[(size_t)(i & 15) * q.a + (i >> 4)];
        return;
    }
    float v;
    if (q.kind == PACK_WEIGHT) {   // [rows][cols] -> [rows_pad][cols_pad]; a rows, b rows_pad, c cols, d cols_pad
        if (i >= q.b * q.d) return;
        const int r = i / q.d, c = i - r * q.d;
        v = (r < q.a && c < q.c) ? q.src[(size_t)r * q.c + c] : 0.0f;
    } else {                       // transposed: a rows, b cols, c k_pad, d cols_pad
        if (i >= q.d * q.c) return;
        const int c = i / q.c, r = i - c * q.c;
        v = (r < q.a && c < q.b) ? q.src[(size_t)r * q.b + c] : 0.0f;
    }
    __bf16 h, l;
    dsplit(v, h, l);
    reinterpret_cast<__bf16*>(q.hi)[i] = h;
    q.lo[i] = l;
}

void launch_pack_batch(PackJob* jobs, int n, hipStream_t st) {
    for (int j0 = 0; j0 < n; j0 += PACK_MAX_JOBS) {
        PackBatch pb{};
        pb.n = std::min(PACK_MAX_JOBS, n - j0);
        uint32_t blocks = 0;
        for (int k = 0; k < pb.n; ++k) {
            PackJob q = jobs[j0 + k];
            const int64_t elems = q.kind == PACK_PLANE ? (int64_t)q.a * 16
                                  : q.kind == PACK_WEIGHT ? (int64_t)q.b * q.d : (int64_t)q.d * q.c;
            q.first_block = blocks;
            blocks += (uint32_t)((elems + 255) / 256);
            pb.j[k] = q;
        }
        if (blocks) hipLaunchKernelGGL(k_pack_batch, dim3(blocks), dim3(256), 0, st, pb);
    }
}

void launch_pack_plane(const float* src, float* dst, int H, int W, hipStream_t st) {
    hipLaunchKernelGGL(k_pack_plane, dim3((H * W * 16 + 255) / 256), dim3(256), 0, st, src, dst, H, W);
}
void launch_pack_weight(const float* src, __bf16* hi, __bf16* lo, int rows, int rows_pad, int cols, int cols_pad,
                        hipStream_t st) {
    hipLaunchKernelGGL(k_pack_weight, dim3((rows_pad * cols_pad + 255) / 256), dim3(256), 0, st, src, hi, lo, rows,
                       rows_pad, cols, cols_pad);
}

}  // namespace lsr

#ifdef LSR_DEFORM_STAMPS
extern "C" int lsr_debug_deform_stamps(unsigned long long* out14) {   // 13 segments + blocks; read and reset
    if (hipMemcpyFromSymbol(out14, HIP_SYMBOL(lsr::g_deform_stamps), 14 * sizeof(unsigned long long)) != hipSuccess) return 2;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(lsr::g_deform_stamps), z, sizeof(z)) == hipSuccess ? 0 : 2;
}
#endif
#ifdef LSR_DEFORM_DIAG
// diagnostic export (not part of include/lsr_deform.h): read and reset the counters
extern "C" int lsr_debug_deform_diag(unsigned long long* out8) {
    if (hipMemcpyFromSymbol(out8, HIP_SYMBOL(lsr::g_deform_diag), 8 * sizeof(unsigned long long)) != hipSuccess) return 2;
    unsigned long long z[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(lsr::g_deform_diag), z, sizeof(z)) == hipSuccess ? 0 : 2;
}
#endif
