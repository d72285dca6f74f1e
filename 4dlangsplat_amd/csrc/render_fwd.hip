// render_fwd.hip -- per-tile front-to-back compositing of RGB + C language channels + depth.
//
// Restates the upstream renderCUDA (constants alpha <= 0.99, skip
// alpha < 1/255, stop when T (1 - alpha) < 1e-4, RGB += T bg, language channels without
// background, depth = sum z alpha T).  One 256-thread workgroup per 16x16 tile, each wave owning
// an 8x8 quadrant (compact footprint: fewer waves touched per splat).  The tile's list is streamed
// through LDS in batches; the per-Gaussian record is gathered as float2 + 2 x float4 + C floats.
// Lanes skip exp where alpha < 1/255 is certain from the power alone (skip_power).
// The workgroup stops early once every pixel has saturated.  Also writes, per tile, the largest
// n_contrib of its pixels, which bounds the backward replay.
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

template <int CPAD, int BATCH>
__global__ void __launch_bounds__(256) k_render_fwd(RenderFwdArgs a) {
    __shared__ uint32_t s_id[BATCH];
    __shared__ float2 s_xy[BATCH];
    __shared__ float4 s_co[BATCH];
    __shared__ float4 s_rgbd[BATCH];
    __shared__ float s_thr[BATCH];
    __shared__ float s_lang[CPAD > 0 ? BATCH * CPAD : 1];
    __shared__ uint32_t s_max;

    const int tile = blockIdx.x;
    const int tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int px = tx * LSR_TILE_X + (wave & 1) * 8 + (lane & 7);
    const int py = ty * LSR_TILE_Y + (wave >> 1) * 8 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pxf = (float)px, pyf = (float)py;
    const uint2 range = a.ranges[tile];
    const int C = a.C;

    if (tid == 0) s_max = 0;
    float T = 1.0f;
    uint32_t contributor = 0, last = 0;
    float acc[3] = {0.0f, 0.0f, 0.0f};
    float accL[CPAD > 0 ? CPAD : 1];
#pragma unroll
    for (int c = 0; c < (CPAD > 0 ? CPAD : 1); ++c) accL[c] = 0.0f;
    float accD = 0.0f;
    bool done = !inside;

    for (uint32_t start = range.x; start < range.y; start += BATCH) {
        if (__syncthreads_count(done) == 256) break;
        const int nb = (int)min((uint32_t)BATCH, range.y - start);
        if (tid < nb) {
            const uint32_t g = a.point_list[start + tid] & PL_ID_MASK;
            s_id[tid] = g;
            s_xy[tid] = a.xy[g];
            const float4 co = a.conic_o[g];
            s_co[tid] = co;
            s_rgbd[tid] = a.rgbd[g];
            s_thr[tid] = skip_power(co.w);
        }
        if constexpr (CPAD > 0) {
            __syncthreads();
            for (int e = tid; e < nb * CPAD; e += 256) {
                const int j = e / CPAD, c = e - j * CPAD;
                s_lang[e] = c < C ? a.lang[(size_t)s_id[j] * C + c] : 0.0f;
            }
        }
        __syncthreads();
        for (int j = 0; j < nb; ++j) {
            if (done) break;
            contributor++;
            const float2 xy = s_xy[j];
            const float4 co = s_co[j];
            const float dx = xy.x - pxf, dy = xy.y - pyf;
            const float power = gauss_power(-0.5f * co.x, -co.y, -0.5f * co.z, dx, dy);
            if (power > 0.0f || power < s_thr[j]) continue;   // the second test never changes a decision
            const float alpha = fminf(0.99f, co.w * expf_repro(power));
            if (alpha < 1.0f / 255.0f) continue;
            const float test_T = T * (1.0f - alpha);
            if (test_T < 0.0001f) { done = true; continue; }
            const float w = alpha * T;
            const float4 cd = s_rgbd[j];
            acc[0] = __builtin_fmaf(cd.x, w, acc[0]);
            acc[1] = __builtin_fmaf(cd.y, w, acc[1]);
            acc[2] = __builtin_fmaf(cd.z, w, acc[2]);
            accD = __builtin_fmaf(cd.w, w, accD);
            if constexpr (CPAD > 0) {
                const float4* f4 = reinterpret_cast<const float4*>(s_lang + j * CPAD);
#pragma unroll
                for (int c4 = 0; c4 < CPAD / 4; ++c4) {
                    const float4 f = f4[c4];
                    accL[4 * c4 + 0] = __builtin_fmaf(f.x, w, accL[4 * c4 + 0]);
                    accL[4 * c4 + 1] = __builtin_fmaf(f.y, w, accL[4 * c4 + 1]);
                    accL[4 * c4 + 2] = __builtin_fmaf(f.z, w, accL[4 * c4 + 2]);
                    accL[4 * c4 + 3] = __builtin_fmaf(f.w, w, accL[4 * c4 + 3]);
                }
            }
            T = test_T;
            last = contributor;
        }
    }
    if (inside) {
        const size_t HW = (size_t)a.H * a.W, pid = (size_t)py * a.W + px;
        a.final_T[pid] = T;
        a.n_contrib[pid] = last;
        a.out_color[pid] = acc[0] + T * a.bg[0];
        a.out_color[HW + pid] = acc[1] + T * a.bg[1];
        a.out_color[2 * HW + pid] = acc[2] + T * a.bg[2];
        a.out_depth[pid] = accD;
        if constexpr (CPAD > 0) {
#pragma unroll
            for (int c = 0; c < CPAD; ++c)
                if (c < C) a.out_lang[(size_t)c * HW + pid] = accL[c];
        }
    }
    // per-tile bound for the backward replay
    uint32_t m = last;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    __syncthreads();
    if (lane == 0) atomicMax(&s_max, m);
    __syncthreads();
    if (tid == 0) a.tile_max_contrib[tile] = s_max;
}

// ---------------------------------------------------------------------------------------------
// MFMA variant for 32 / 64 language channels.  The per-pixel serial part (alpha, T, early stop,
// RGB and depth in f32 FMAs) is unchanged and bit-identical in its decisions; the language sums
//   out^T[c][px] += sum_e F^T[c][e] W^T[e][px],   W[px][e] = alpha_e T_e
// run on v_mfma_f32_32x32x16_bf16 with a two-term bf16 split of both operands (hi = bf16(x),
// lo = bf16(x - hi); products hi*hi + hi*lo + lo*hi, ~2^-17 relative, f32 accumulation), one
// 32-entry group at a time.  A = F^T (channels x entries) comes from an LDS image written during
// staging; B = W^T (entries x pixels) comes straight from the lanes' weight registers: each
// lane holds its pixel's 32 weights, and one permlane32_swap per packed dword builds the two
// 32-pixel operand blocks (lanes 0-31 own pixels 0-31, lanes 32-63 pixels 32-63 of the wave).
// The accumulators (32 x 64 per 32 channels) live in registers for the whole tile.
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void split_bf16(float x, __bf16& hi, __bf16& lo) {
    hi = (__bf16)x;
    lo = (__bf16)(x - (float)hi);
}

// permlane32_swap of two 8 x bf16 operands (4 dwords each)
__device__ __forceinline__ void swap32_x8(bf16x8& x, bf16x8& y) {
    u32x4 a = __builtin_bit_cast(u32x4, x), b = __builtin_bit_cast(u32x4, y);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        auto r = __builtin_amdgcn_permlane32_swap(a[i], b[i], false, false);
        a[i] = r[0];
        b[i] = r[1];
    }
    x = __builtin_bit_cast(bf16x8, a);
    y = __builtin_bit_cast(bf16x8, b);
}

template <int MB>
__global__ void __launch_bounds__(256) k_render_fwd_mfma(RenderFwdArgs a) {
    constexpr int CP = 32 * MB;   // padded language channels
    constexpr int SB = 64;        // entries staged per LDS batch = 2 MFMA groups of 32
    constexpr int FP = 40;        // row pitch (bf16) of the F^T image: 32 entries + 8 pad
    __shared__ __attribute__((aligned(16))) __bf16 s_Fh[SB / 32][CP][FP];
    __shared__ __attribute__((aligned(16))) __bf16 s_Fl[SB / 32][CP][FP];
    __shared__ float4 s_co[SB];
    __shared__ float4 s_rgbd[SB];
    __shared__ float2 s_xy[SB];
    __shared__ float s_thr[SB];
    __shared__ uint32_t s_id[SB];
    __shared__ uint32_t s_max;

    const int tile = blockIdx.x;
    const int tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int qx = tx * LSR_TILE_X + (wave & 1) * 8, qy = ty * LSR_TILE_Y + (wave >> 1) * 8;   // quadrant origin
    const int px = qx + (lane & 7), py = qy + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pxf = (float)px, pyf = (float)py;
    const uint2 range = a.ranges[tile];
    const int C = a.C;
    const int lr = lane & 31, lh = lane >> 5;

    if (tid == 0) s_max = 0;
    float T = 1.0f;
    uint32_t contributor = 0, last = 0;
    float acc[3] = {0.0f, 0.0f, 0.0f}, accD = 0.0f;
    f32x16 dacc[MB][2];
#pragma unroll
    for (int m = 0; m < MB; ++m) {
        dacc[m][0] = f32x16{};
        dacc[m][1] = f32x16{};
    }
    bool done = !inside;

    for (uint32_t start = range.x; start < range.y; start += SB) {
        if (__syncthreads_count(done) == 256) break;
        const int nb = (int)min((uint32_t)SB, range.y - start);
        if (tid < nb) {
            const uint32_t g = a.point_list[start + tid] & PL_ID_MASK;
            s_id[tid] = g;
            s_xy[tid] = a.xy[g];
            const float4 co = a.conic_o[g];
            s_co[tid] = co;
            s_rgbd[tid] = a.rgbd[g];
            s_thr[tid] = skip_power(co.w);
        }
        __syncthreads();
        for (int e = tid; e < SB * CP; e += 256) {
            const int j = e / CP, c = e - j * CP;
            const float x = (j < nb && c < C) ? a.lang[(size_t)s_id[j] * C + c] : 0.0f;
            __bf16 hi, lo;
            split_bf16(x, hi, lo);
            s_Fh[j >> 5][c][j & 31] = hi;
            s_Fl[j >> 5][c][j & 31] = lo;
        }
        __syncthreads();
        for (int grp = 0; grp * 32 < nb; ++grp) {
            float w[32];
            bool any = false;
#pragma unroll
            for (int jj = 0; jj < 32; ++jj) {
                w[jj] = 0.0f;
                const int j = grp * 32 + jj;
                if (j < nb && !done) {
                    contributor++;
                    const float2 xy = s_xy[j];
                    const float4 co = s_co[j];
                    const float dx = xy.x - pxf, dy = xy.y - pyf;
                    const float power = gauss_power(-0.5f * co.x, -co.y, -0.5f * co.z, dx, dy);
                    if (!(power > 0.0f || power < s_thr[j])) {
                        const float alpha = fminf(0.99f, co.w * expf_repro(power));
                        if (alpha >= 1.0f / 255.0f) {
                            const float test_T = T * (1.0f - alpha);
                            if (test_T < 0.0001f) {
                                done = true;
                            } else {
                                const float wt = alpha * T;
                                const float4 cd = s_rgbd[j];
                                acc[0] = __builtin_fmaf(cd.x, wt, acc[0]);
                                acc[1] = __builtin_fmaf(cd.y, wt, acc[1]);
                                acc[2] = __builtin_fmaf(cd.z, wt, acc[2]);
                                accD = __builtin_fmaf(cd.w, wt, accD);
                                w[jj] = wt;
                                any = true;
                                T = test_T;
                                last = contributor;
                            }
                        }
                    }
                }
            }
            if (!__any(any)) continue;
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                bf16x8 xh, xl, yh, yl;   // entries 16ks + j (x) and 16ks + 8 + j (y) of this lane's pixel
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    __bf16 h, l;
                    split_bf16(w[16 * ks + j], h, l);
                    xh[j] = h; xl[j] = l;
                    split_bf16(w[16 * ks + 8 + j], h, l);
                    yh[j] = h; yl[j] = l;
                }
                // x -> B operand of pixels 0-31, y -> pixels 32-63 (see the header comment)
                swap32_x8(xh, yh);
                swap32_x8(xl, yl);
#pragma unroll
                for (int m = 0; m < MB; ++m) {
                    const bf16x8 ah = *reinterpret_cast<const bf16x8*>(&s_Fh[grp][32 * m + lr][16 * ks + 8 * lh]);
                    const bf16x8 al = *reinterpret_cast<const bf16x8*>(&s_Fl[grp][32 * m + lr][16 * ks + 8 * lh]);
                    dacc[m][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xh, dacc[m][0], 0, 0, 0);
                    dacc[m][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, xl, dacc[m][0], 0, 0, 0);
                    dacc[m][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, xh, dacc[m][0], 0, 0, 0);
                    dacc[m][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, yh, dacc[m][1], 0, 0, 0);
                    dacc[m][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(ah, yl, dacc[m][1], 0, 0, 0);
                    dacc[m][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(al, yh, dacc[m][1], 0, 0, 0);
                }
            }
        }
    }
    const size_t HW = (size_t)a.H * a.W;
    if (inside) {
        const size_t pid = (size_t)py * a.W + px;
        a.final_T[pid] = T;
        a.n_contrib[pid] = last;
        a.out_color[pid] = acc[0] + T * a.bg[0];
        a.out_color[HW + pid] = acc[1] + T * a.bg[1];
        a.out_color[2 * HW + pid] = acc[2] + T * a.bg[2];
        a.out_depth[pid] = accD;
    }
    // language channels: D[c][p] of pixel p = lr + 32 nb of this wave's 8 x 8 quadrant
#pragma unroll
    for (int nb2 = 0; nb2 < 2; ++nb2) {
        const int p = lr + 32 * nb2;
        const int ox = qx + (p & 7), oy = qy + (p >> 3);
        if (ox < a.W && oy < a.H) {
            const size_t pid = (size_t)oy * a.W + ox;
#pragma unroll
            for (int m = 0; m < MB; ++m)
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int c = 32 * m + (r & 3) + 8 * (r >> 2) + 4 * lh;
                    if (c < C) a.out_lang[(size_t)c * HW + pid] = dacc[m][nb2][r];
                }
        }
    }
    uint32_t mx = last;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) mx = max(mx, (uint32_t)__shfl_xor((int)mx, o));
    __syncthreads();
    if (lane == 0) atomicMax(&s_max, mx);
    __syncthreads();
    if (tid == 0) a.tile_max_contrib[tile] = s_max;
}

template <int CPAD, int BATCH>
static void go_fwd(const RenderFwdArgs& a, hipStream_t st) {
    hipLaunchKernelGGL((k_render_fwd<CPAD, BATCH>), dim3(a.grid_x * a.grid_y), dim3(256), 0, st, a);
}

void launch_render_fwd(const RenderFwdArgs& a, hipStream_t st) {
#ifndef LSR_FWD_BLOCK
    RenderFwdArgs f = a;
#ifdef LSR_FWD_ORDER
    if (f.tile_order) launch_tile_order(a.grid_x * a.grid_y, nullptr, a.ranges, f.tile_order, st);
#else
    f.tile_order = nullptr;   // tile order: the order scratch is not written
#endif
    launch_render_fwd_wave(f, st);   // compacted per-quadrant waves (render_fwd_wave.hip)
    return;
#endif
    const int C = a.include_feature ? a.C : 0;
    if (C == 0) go_fwd<0, 256>(a, st);
    else if (C <= 4) go_fwd<4, 256>(a, st);
    else if (C <= 8) go_fwd<8, 256>(a, st);
    else if (C <= 16) go_fwd<16, 128>(a, st);
    else if (C <= 32) go_fwd<32, 128>(a, st);   // VALU variant measured faster at 32 channels (serial-loop bound)
    else hipLaunchKernelGGL(k_render_fwd_mfma<2>, dim3(a.grid_x * a.grid_y), dim3(256), 0, st, a);
}

}  // namespace lsr
