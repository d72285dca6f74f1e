// render_bwd_mfma.hip -- backward compositing with the language channels on matrix cores.
//
// Same mathematics as render_bwd.hip (upstream backward).  The replay is
// cut into groups of 32 list entries.  Per group and per wave (64 pixels = one 8x8 quadrant):
//   MFMA1  S[e][px]  = sum_c F[e][c] G[px][c]        the language part of dot(c_e, dL/dpix)
//   serial           the per-pixel back-to-front recurrence (T, accum_rec . g, dL/dalpha) and the
//                    10 scalar gradients (colour, depth, mean2D, conic, opacity), which are summed
//                    over the wave by a 16-wide transpose-reduce
//   MFMA2  dF[e][c] = sum_px W[px][e] G[px][c]       the language-feature gradient, W = alpha T
// Both products use v_mfma_f32_32x32x16_bf16 with a two-term bf16 split of both operands
// (hi*hi + hi*lo + lo*hi, ~2^-17 relative, f32 accumulation).  Operand sources:
//   F (entries x channels)   LDS rows written at staging (A of MFMA1, ds_read_b128)
//   G (pixels x channels)    built once per tile from the lanes' own dL/dlanguage: B of MFMA1
//                            by permlane32_swap, B of MFMA2 (pixels on K) through a one-off LDS
//                            transpose; both kept in registers
//   W (pixels x entries)     written per group by each lane as one LDS row and read back with
//                            ds_read_b64_tr_b16 (pixels on K) as A of MFMA2
// MFMA1's result (entries in registers, pixels on lanes) is folded to one pixel per lane with one
// permlane32_swap per register.  The four waves' dF blocks meet in LDS; each (Gaussian, tile)
// then issues one atomic per language channel (contiguous 128-byte row) and one per scalar.
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ void split2(float x, __bf16& hi, __bf16& lo) {
    hi = (__bf16)x;
    lo = (__bf16)(x - (float)hi);
}

__device__ __forceinline__ void swap32_x8b(bf16x8& x, bf16x8& y) {
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

__device__ __forceinline__ bf16x4 ds_read_tr_b16(const __bf16* p) {
    // ds_read_b64_tr_b16: 16-lane groups read a 4 x 16 block of 16-bit values column-major
    typedef short s16x4 __attribute__((ext_vector_type(4)));
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        reinterpret_cast<__attribute__((address_space(3))) s16x4*>(reinterpret_cast<size_t>(p)));
    return __builtin_bit_cast(bf16x4, v);
}

#define MFMA(a, b, c) __builtin_amdgcn_mfma_f32_32x32x16_bf16((a), (b), (c), 0, 0, 0)

constexpr int BG = 32;     // entries per MFMA group
constexpr int BSB = 32;    // entries staged per LDS batch (1 group)
constexpr int FPT = 40;    // F row pitch in bf16 (32 channels + 8 pad)
constexpr int WPT = 36;    // W row pitch in bf16 (32 entries + 4 pad; 8-byte aligned rows for the tr reads)
constexpr int GTP = 72;    // G^T row pitch in bf16 (64 pixels + 8 pad)
constexpr int RQ = 12;     // scalar record: rgb 0-2, depth 3, mean2D 4-5, conic 6-8, opacity 9

template <bool DUMMY>
__global__ void __launch_bounds__(256, 3) k_render_bwd_mfma(RenderBwdArgs a) {
    __shared__ __attribute__((aligned(16))) __bf16 s_Fh[BSB][FPT];
    __shared__ __attribute__((aligned(16))) __bf16 s_Fl[BSB][FPT];
    __shared__ __attribute__((aligned(16))) __bf16 s_W[4][2][64][WPT];     // per wave: hi, lo rows [px][e]
    __shared__ float s_lrec[BSB][32];                                     // language gradient per entry
    __shared__ float s_rec[BSB][RQ];
    __shared__ float4 s_co[BSB];
    __shared__ float4 s_rgbd[BSB];
    __shared__ float2 s_xy[BSB];
    __shared__ float s_thr[BSB];
    __shared__ uint32_t s_id[BSB];
    __shared__ uint32_t s_act[BSB];

    const int tile = blockIdx.x;
    const int tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int lr = lane & 31, lh = lane >> 5;
    const int px = tx * LSR_TILE_X + (wave & 1) * 8 + (lane & 7);
    const int py = ty * LSR_TILE_Y + (wave >> 1) * 8 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pxf = (float)px, pyf = (float)py;
    const uint2 range = a.ranges[tile];
    const uint32_t nreplay = a.tile_max_contrib[tile];
    const int C = a.C;
    const size_t HW = (size_t)a.H * a.W, pid = inside ? (size_t)py * a.W + px : 0;

    const float T_final = inside ? a.final_T[pid] : 0.0f;
    float T = T_final;
    const uint32_t last_contributor = inside ? a.n_contrib[pid] : 0;
    float g0 = 0.0f, g1 = 0.0f, g2 = 0.0f, gD = 0.0f;
    if (inside) {
        g0 = a.dL_dcolor[pid]; g1 = a.dL_dcolor[HW + pid]; g2 = a.dL_dcolor[2 * HW + pid];
        if (a.dL_ddepth) gD = a.dL_ddepth[pid];
    }

    // ---- per-tile operand fragments of G (this lane's pixel, 32 language channels) ----------
    // B1[ks][nb]: MFMA1 B operand, K = channel 16 ks + 8 lh + j, column = pixel lr + 32 nb
    // B2[ks]    : MFMA2 B operand, K = pixel 16 ks + 8 lh + j, column = channel lr
    bf16x8 b1h[2][2], b1l[2][2], b2h[4], b2l[4];
    {
        float gl[32];
#pragma unroll
        for (int c = 0; c < 32; ++c)
            gl[c] = (inside && a.dL_dlang && c < C) ? a.dL_dlang[(size_t)c * HW + pid] : 0.0f;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
            bf16x8 xh, xl, yh, yl;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                __bf16 h, l;
                split2(gl[16 * ks + j], h, l); xh[j] = h; xl[j] = l;
                split2(gl[16 * ks + 8 + j], h, l); yh[j] = h; yl[j] = l;
            }
            swap32_x8b(xh, yh);
            swap32_x8b(xl, yl);
            b1h[ks][0] = xh; b1l[ks][0] = xl; b1h[ks][1] = yh; b1l[ks][1] = yl;
        }
        // one-off transpose of G through this wave's W area: rows [c][px] (hi, lo)
        __bf16* gt = &s_W[wave][0][0][0];   // 2 x 64 x 40 bf16 = room for 32 rows of pitch 72 x 2
#pragma unroll
        for (int c = 0; c < 32; ++c) {
            __bf16 h, l;
            split2(gl[c], h, l);
            gt[c * GTP + lane] = h;
            gt[32 * GTP + c * GTP + lane] = l;
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
            b2h[ks] = *reinterpret_cast<const bf16x8*>(gt + lr * GTP + 16 * ks + 8 * lh);
            b2l[ks] = *reinterpret_cast<const bf16x8*>(gt + 32 * GTP + lr * GTP + 16 * ks + 8 * lh);
        }
        __syncthreads();
    }
    const float bg_dot = a.bg[0] * g0 + a.bg[1] * g1 + a.bg[2] * g2;
    const float ddelx_dx = 0.5f * (float)a.W, ddely_dy = 0.5f * (float)a.H;
    float acc_dot = 0.0f, last_dot = 0.0f, last_alpha = 0.0f;

    for (int end = (int)nreplay; end > 0; end -= BSB) {
        const int nb = min(BSB, end);
        const int first = end - nb;                   // list position of batch slot 0
        __syncthreads();
        if (tid < BSB) {
            if (tid < nb) {
                const uint32_t gid = a.point_list[range.x + first + tid];
                const float4 co = a.conic_o[gid];
                s_id[tid] = gid;
                s_xy[tid] = a.xy[gid];
                s_co[tid] = co;
                s_rgbd[tid] = a.rgbd[gid];
                s_thr[tid] = skip_power(co.w);
            } else {
                s_co[tid] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                s_thr[tid] = __builtin_inff();
            }
            s_act[tid] = 0;
        }
        for (int e = tid; e < BSB * RQ; e += 256) (&s_rec[0][0])[e] = 0.0f;
        for (int e = tid; e < BSB * 32; e += 256) (&s_lrec[0][0])[e] = 0.0f;
        __syncthreads();
        for (int e = tid; e < BSB * 32; e += 256) {
            const int j = e >> 5, c = e & 31;
#ifdef LSR_ABL_NOLANG
            const float x = (j < nb && c < C) ? (float)(s_id[j] & 7) : 0.0f;
#else
            const float x = (j < nb && c < C) ? a.lang[(size_t)s_id[j] * C + c] : 0.0f;
#endif
            __bf16 h, l;
            split2(x, h, l);
            s_Fh[j][c] = h;
            s_Fl[j][c] = l;
        }
        __syncthreads();
        for (int grp = (nb - 1) / BG; grp >= 0; --grp) {
            const int j0 = grp * BG;
            // ---- MFMA1: S[e][px] for the group's 32 entries and the wave's 64 pixels ----------
            f32x16 d0 = f32x16{}, d1 = f32x16{};
#ifndef LSR_ABL_NOMFMA
#pragma unroll
            for (int ks = 0; ks < 2; ++ks) {
                const bf16x8 ah = *reinterpret_cast<const bf16x8*>(&s_Fh[j0 + lr][16 * ks + 8 * lh]);
                const bf16x8 al = *reinterpret_cast<const bf16x8*>(&s_Fl[j0 + lr][16 * ks + 8 * lh]);
                d0 = MFMA(ah, b1h[ks][0], d0); d0 = MFMA(ah, b1l[ks][0], d0); d0 = MFMA(al, b1h[ks][0], d0);
                d1 = MFMA(ah, b1h[ks][1], d1); d1 = MFMA(ah, b1l[ks][1], d1); d1 = MFMA(al, b1h[ks][1], d1);
            }
#endif
            // fold: afterwards S of entry (r&3) + 8(r>>2) is d0[r], of entry +4 is d1[r], own pixel
#pragma unroll
            for (int r = 0; r < 16; ++r) {
                auto v = __builtin_amdgcn_permlane32_swap(__float_as_uint(d0[r]), __float_as_uint(d1[r]), false, false);
                d0[r] = __uint_as_float(v[0]);
                d1[r] = __uint_as_float(v[1]);
            }
            // ---- serial back-to-front replay of the group ----------------------------------------
            float wv[BG];
#pragma unroll
            for (int jj = BG - 1; jj >= 0; --jj) {
                const int j = j0 + jj;
                const uint32_t k = (uint32_t)(first + j);
                const float S = ((jj >> 2) & 1) ? d1[(jj & 3) + 4 * (jj >> 3)] : d0[(jj & 3) + 4 * (jj >> 3)];
                bool active = false;
                float w = 0.0f, gm2x = 0.0f, gm2y = 0.0f, gcx = 0.0f, gcy = 0.0f, gcw = 0.0f, gop = 0.0f;
                if (j < nb && k < last_contributor) {
                    const float2 xy = s_xy[j];
                    const float4 co = s_co[j];
                    const float dx = xy.x - pxf, dy = xy.y - pyf;
                    const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                    if (power <= 0.0f && power >= s_thr[j]) {
                        const float G = expf_repro(power);
                        const float alpha = fminf(0.99f, co.w * G);
                        if (alpha >= 1.0f / 255.0f) {
                            active = true;
                            const float om = 1.0f - alpha;
                            const float rom = __builtin_amdgcn_rcpf(om);
                            T = T * rom;
                            w = alpha * T;
                            const float4 cd = s_rgbd[j];
                            float dot = cd.x * g0;
                            dot = __builtin_fmaf(cd.y, g1, dot);
                            dot = __builtin_fmaf(cd.z, g2, dot);
                            dot = __builtin_fmaf(cd.w, gD, dot);
                            dot += S;
                            acc_dot = __builtin_fmaf(last_alpha, last_dot, (1.0f - last_alpha) * acc_dot);
                            last_dot = dot;
                            float dL_dalpha = (dot - acc_dot) * T;
                            last_alpha = alpha;
                            dL_dalpha = __builtin_fmaf(-T_final * rom, bg_dot, dL_dalpha);
                            const float dL_dG = co.w * dL_dalpha;
                            const float gdx = G * dx, gdy = G * dy;
                            const float dG_ddelx = -gdx * co.x - gdy * co.y;
                            const float dG_ddely = -gdy * co.z - gdx * co.y;
                            gm2x = dL_dG * dG_ddelx * ddelx_dx;
                            gm2y = dL_dG * dG_ddely * ddely_dy;
                            gcx = -0.5f * gdx * dx * dL_dG;
                            gcy = -0.5f * gdx * dy * dL_dG;
                            gcw = -0.5f * gdy * dy * dL_dG;
                            gop = G * dL_dalpha;
                        }
                    }
                }
                wv[jj] = w;
                if (__any(active)) {
                    float v[16];
                    v[0] = w * g0; v[1] = w * g1; v[2] = w * g2; v[3] = w * gD;
                    v[4] = gm2x; v[5] = gm2y; v[6] = gcx; v[7] = gcy; v[8] = gcw; v[9] = gop;
#pragma unroll
                    for (int q = 10; q < 16; ++q) v[q] = 0.0f;
#ifdef LSR_ABL_NORED
                    float sv = 0.0f;
#pragma unroll
                    for (int q = 0; q < 10; ++q) sv += v[q];
                    if (sv == 1234.5f) atomicAdd(&s_rec[j][0], sv);
#else
                    wave_transpose_reduce<16>(v);
                    const int q = transpose_reduce_slot<16>(lane);
                    if ((lane & 3) == 0 && q < 10) atomicAdd(&s_rec[j][q], v[0]);
#endif
                    if (lane == 0) s_act[j] = 1u;
                }
            }
            // ---- MFMA2: dF[e][c] = sum_px W[px][e] G[px][c] over this wave's pixels --------------
            {
                __bf16* wh = &s_W[wave][0][0][0];
                __bf16* wl = &s_W[wave][1][0][0];
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                    bf16x8 hh, ll;
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        __bf16 h, l;
                        split2(wv[8 * q + j], h, l);
                        hh[j] = h; ll[j] = l;
                    }
                    *reinterpret_cast<bf16x8*>(wh + lane * WPT + 8 * q) = hh;
                    *reinterpret_cast<bf16x8*>(wl + lane * WPT + 8 * q) = ll;
                }
                __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's rows are in LDS
                __builtin_amdgcn_wave_barrier();
                // A operand (entries x pixels): lanes 16g'+i read rows px = 16ks + 8lh + {0..3, 4..7},
                // columns e = 16 (g' & 1) + i, via two transposing reads
                const int grpl = lane >> 4, li = lane & 15;
                const int ecol = 16 * (grpl & 1);
                const int qrow = li >> 2, pcol = 4 * (li & 3);
                f32x16 acc2 = f32x16{};
#ifndef LSR_ABL_NOMFMA
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const int r0 = 16 * ks + 8 * lh + qrow;
                    const bf16x4 h0 = ds_read_tr_b16(wh + r0 * WPT + ecol + pcol);
                    const bf16x4 h1 = ds_read_tr_b16(wh + (r0 + 4) * WPT + ecol + pcol);
                    const bf16x4 l0 = ds_read_tr_b16(wl + r0 * WPT + ecol + pcol);
                    const bf16x4 l1 = ds_read_tr_b16(wl + (r0 + 4) * WPT + ecol + pcol);
                    const bf16x8 ah = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
                    const bf16x8 al = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
                    acc2 = MFMA(ah, b2h[ks], acc2);
                    acc2 = MFMA(ah, b2l[ks], acc2);
                    acc2 = MFMA(al, b2h[ks], acc2);
                }
#endif
                // acc2[r]: entry (r&3) + 8(r>>2) + 4 lh, channel lr
#pragma unroll
                for (int r = 0; r < 16; ++r) {
                    const int e = (r & 3) + 8 * (r >> 2) + 4 * lh;
                    if (acc2[r] != 0.0f) atomicAdd(&s_lrec[j0 + e][lr], acc2[r]);
                }
            }
        }
        __syncthreads();
        // one atomic per quantity of each active (Gaussian, tile); consecutive lanes -> contiguous
        for (int e = tid; e < nb * (RQ + 32); e += 256) {
            const int j = e / (RQ + 32), q = e - j * (RQ + 32);
            if (!s_act[j]) continue;
            const uint32_t gid = s_id[j];
            if (q < 10) atomicAdd(a.acc_small + (size_t)gid * ACC_PITCH + q, s_rec[j][q]);
            else if (q >= RQ && q - RQ < C && a.acc_lang) atomicAdd(a.acc_lang + (size_t)gid * C + (q - RQ), s_lrec[j][q - RQ]);
        }
    }
}

void launch_render_bwd_mfma(const RenderBwdArgs& a, hipStream_t st) {
    hipLaunchKernelGGL(k_render_bwd_mfma<true>, dim3(a.grid_x * a.grid_y), dim3(256), 0, st, a);
}

}  // namespace lsr
