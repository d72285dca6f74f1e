// render_bwd_wave.hip -- compositor backward, one independent wave per 8x8 pixel quadrant, with
// the language channels (C <= 32) on matrix cores.
//
// Same mathematics as render_bwd.hip (upstream backward).  Measured on the
// headline scene, only a third of the replayed list entries touch any pixel of a given 8x8
// quadrant.  An entry that no pixel of the quadrant activates changes neither T nor the
// back-to-front accumulators of any of its pixels, so skipping it is exact.  Each wave therefore
//   1. scans its replay range (up to the largest n_contrib of its pixels) back to front, 64
//      entries per round, one per lane: a conservative ellipse-vs-quadrant test
//      (quad_may_touch) and a ballot compaction into a per-wave FIFO in LDS;
//   2. processes the surviving entries in groups of 16 (WG):
//        MFMA1  S[e][px]  = sum_c F[e][c] G[px][c]    the language part of dot(c_e, dL/dpix)
//        serial           the per-pixel back-to-front recurrence and the 10 scalar gradients,
//                         summed over the wave by a transpose-reduce, one global atomic each
//        MFMA2  dF[e][c]  = sum_px W[px][e] G[px][c]  the language gradient, W = alpha T,
//                         one global atomic per (entry, channel)
//      both on v_mfma_f32_16x16x32_bf16 with hi/lo bf16 splits (lsr_mfma.h).
// No block barriers: 64-thread blocks, the four quadrants of a tile on one XCD.
#include "lsr_common.h"
#include "lsr_internal.h"
#include "lsr_mfma.h"

namespace lsr {

constexpr int WG = 16;       // compacted entries per MFMA group
constexpr int WFP = 40;      // F / G row pitch in bf16 (32 channels + 8): 80-byte rows, 16-byte aligned
constexpr int WWP = 20;      // W row pitch in bf16 (16 entries + 4): 40-byte rows, 8-byte aligned
constexpr int WFIFO = 128;   // compacted entries waiting (list positions and ids); power of two

__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(3)))
k_render_bwd_wave(RenderBwdArgs a) {
    __shared__ __attribute__((aligned(16))) __bf16 s_GW[64 * WFP];      // G rows once, then W hi | lo
    __shared__ __attribute__((aligned(16))) __bf16 s_Fh[WG * WFP];
    __shared__ __attribute__((aligned(16))) __bf16 s_Fl[WG * WFP];
    __shared__ float4 s_co[WG];
    __shared__ float4 s_rgbd[WG];
    __shared__ float2 s_xy[WG];
    __shared__ float s_thr[WG];
    __shared__ uint32_t s_gid[WG];
    __shared__ uint32_t s_k[WG];
    __shared__ uint32_t s_fk[WFIFO];
    __shared__ uint32_t s_fg[WFIFO];

    const int b = blockIdx.x;
    const int tile = (b >> 5) * 8 + (b & 7), quad = (b >> 3) & 3;
    if (tile >= a.grid_x * a.grid_y) return;
    const int lane = threadIdx.x, g4 = lane >> 4, l16 = lane & 15;
    const int tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int qx0 = tx * LSR_TILE_X + (quad & 1) * 8, qy0 = ty * LSR_TILE_Y + (quad >> 1) * 8;
    const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const size_t HW = (size_t)a.H * a.W, pid = inside ? (size_t)py * a.W + px : 0;
    const uint32_t last_contributor = inside ? a.n_contrib[pid] : 0u;
    uint32_t nrep = last_contributor;
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) nrep = max(nrep, (uint32_t)__shfl_xor((int)nrep, off));
    nrep = __builtin_amdgcn_readfirstlane(nrep);
    if (nrep == 0) return;                                           // wave-uniform
    const uint2 range = a.ranges[tile];
    const int C = a.C;
    const float bx0 = (float)qx0, bx1 = (float)min(qx0 + 7, a.W - 1);
    const float by0 = (float)qy0, by1 = (float)min(qy0 + 7, a.H - 1);

    const float T_final = inside ? a.final_T[pid] : 0.0f;
    float T = T_final;
    float g0 = 0.0f, g1 = 0.0f, g2 = 0.0f, gD = 0.0f;
    if (inside) {
        g0 = a.dL_dcolor[pid]; g1 = a.dL_dcolor[HW + pid]; g2 = a.dL_dcolor[2 * HW + pid];
        if (a.dL_ddepth) gD = a.dL_ddepth[pid];
    }

    // ---- G fragments (this wave's 64 pixels x 32 channels), built once through LDS rows [px][c]
    // b1[pb]     : MFMA1 B, K = channel 8 g4 + j, N = pixel 16 pb + l16
    // b2[kb][nb] : MFMA2 B, K = pixel 32 kb + 8 g4 + j, N = channel 16 nb + l16
    bf16x8 b1h[4], b1l[4], b2h[2][2], b2l[2][2];
    {
        float gl[32];
#pragma unroll
        for (int c = 0; c < 32; ++c)
            gl[c] = (inside && a.dL_dlang && c < C) ? a.dL_dlang[(size_t)c * HW + pid] : 0.0f;
#pragma unroll
        for (int part = 0; part < 2; ++part) {
#pragma unroll
            for (int c8 = 0; c8 < 4; ++c8) {
                bf16x8 v;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    __bf16 h, l;
                    split_bf16(gl[8 * c8 + j], h, l);
                    v[j] = part == 0 ? h : l;
                }
                *reinterpret_cast<bf16x8*>(s_GW + lane * WFP + 8 * c8) = v;
            }
            wave_lds_sync();
            bf16x8* B1 = part == 0 ? b1h : b1l;
#pragma unroll
            for (int pb = 0; pb < 4; ++pb)
                B1[pb] = *reinterpret_cast<const bf16x8*>(s_GW + (16 * pb + l16) * WFP + 8 * g4);
#pragma unroll
            for (int kb = 0; kb < 2; ++kb)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    const __bf16* p = s_GW + (32 * kb + 8 * g4 + (l16 >> 2)) * WFP + 16 * nb + 4 * (l16 & 3);
                    const bf16x4 lo4 = ds_read_tr16(p), hi4 = ds_read_tr16(p + 4 * WFP);
                    const bf16x8 v = __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7);
                    if (part == 0) b2h[kb][nb] = v; else b2l[kb][nb] = v;
                }
            wave_lds_sync();
        }
    }
    __bf16* s_Wh = s_GW;
    __bf16* s_Wl = s_GW + 64 * WWP;

    const float bg_dot = a.bg[0] * g0 + a.bg[1] * g1 + a.bg[2] * g2;
    const float ddelx_dx = 0.5f * (float)a.W, ddely_dy = 0.5f * (float)a.H;
    float acc_dot = 0.0f, last_dot = 0.0f, last_alpha = 0.0f;
    const float pxf = (float)px, pyf = (float)py;

    int pos = (int)nrep;     // list positions [0, pos) not yet scanned
    int head = 0, tail = 0;  // FIFO counters (wave-uniform)
    while (true) {
        // ---- 1. scan + compaction until a group is available or the range is exhausted -----
        while (tail - head < WG && pos > 0) {
            const int base = max(pos - 64, 0);
            const int k = base + lane;
            bool cand = false;
            uint32_t gid = 0;
            if (k < pos) {
                gid = a.point_list[range.x + k];
                cand = quad_may_touch(a.xy[gid], a.conic_o[gid], bx0, bx1, by0, by1);
            }
            const uint64_t m = __ballot(cand);
            if (cand) {   // back to front: higher list positions first
                const int rank = lane == 63 ? 0 : __popcll(m >> (lane + 1));
                const int s = (tail + rank) & (WFIFO - 1);
                s_fk[s] = (uint32_t)k;
                s_fg[s] = gid;
            }
            tail += __popcll(m);
            pos = base;
        }
        const int cnt = min(WG, tail - head);
        if (cnt == 0) break;
        wave_lds_sync();
        // ---- 2. stage the group: geometry (lanes 0-15), language rows (lane -> entry lane/4) ----
        if (lane < WG) {
            const bool ok = lane < cnt;
            const int s = (head + lane) & (WFIFO - 1);
            const uint32_t gid = ok ? s_fg[s] : 0u;
            const float4 co = ok ? a.conic_o[gid] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            s_gid[lane] = gid;
            s_k[lane] = ok ? s_fk[s] : 0xFFFFFFFFu;
            s_xy[lane] = ok ? a.xy[gid] : make_float2(0.0f, 0.0f);
            s_co[lane] = co;
            s_rgbd[lane] = ok ? a.rgbd[gid] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            s_thr[lane] = ok ? skip_power(co.w) : __builtin_inff();
        }
        {
            const int e = lane >> 2, c0 = 8 * (lane & 3);
            const bool ok = e < cnt;
            const uint32_t gid = ok ? s_fg[(head + e) & (WFIFO - 1)] : 0u;
            float f[8];
            if (C == 32) {
                const float4* r = reinterpret_cast<const float4*>(a.lang + (size_t)gid * 32 + c0);
                const float4 v0 = ok ? r[0] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                const float4 v1 = ok ? r[1] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                f[0] = v0.x; f[1] = v0.y; f[2] = v0.z; f[3] = v0.w; f[4] = v1.x; f[5] = v1.y; f[6] = v1.z; f[7] = v1.w;
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] = (ok && c0 + j < C) ? a.lang[(size_t)gid * C + c0 + j] : 0.0f;
            }
            bf16x8 h8, l8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                __bf16 h, l;
                split_bf16(f[j], h, l);
                h8[j] = h; l8[j] = l;
            }
            *reinterpret_cast<bf16x8*>(s_Fh + e * WFP + c0) = h8;
            *reinterpret_cast<bf16x8*>(s_Fl + e * WFP + c0) = l8;
        }
        head += cnt;
        wave_lds_sync();

        // ---- 3. MFMA1: S[e][px], then to one pixel per lane -----------------------------------
        float S[WG];
        {
            const bf16x8 ah = *reinterpret_cast<const bf16x8*>(s_Fh + l16 * WFP + 8 * g4);
            const bf16x8 al = *reinterpret_cast<const bf16x8*>(s_Fl + l16 * WFP + 8 * g4);
            f32x4 d[4];
#pragma unroll
            for (int pb = 0; pb < 4; ++pb) {
                d[pb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
                d[pb] = LSR_MFMA16(ah, b1h[pb], d[pb]);
                d[pb] = LSR_MFMA16(ah, b1l[pb], d[pb]);
                d[pb] = LSR_MFMA16(al, b1h[pb], d[pb]);
            }
            // d[pb][i] at lane (g4, c): entry 4 g4 + i, pixel 16 pb + c
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float x[4] = {d[0][i], d[1][i], d[2][i], d[3][i]};
                transpose_lane_groups(x);
#pragma unroll
                for (int p = 0; p < 4; ++p) S[4 * p + i] = x[p];   // entry 4p + i, own pixel
            }
        }

        // ---- 4. serial back-to-front replay of the group ---------------------------------------
        float wv[WG];
#pragma unroll
        for (int e = 0; e < WG; ++e) {
            wv[e] = 0.0f;
            if (e >= cnt) continue;                                  // wave-uniform
            bool active = false;
            float w = 0.0f, gm2x = 0.0f, gm2y = 0.0f, gcx = 0.0f, gcy = 0.0f, gcw = 0.0f, gop = 0.0f;
            if (s_k[e] < last_contributor) {
                const float2 xy = s_xy[e];
                const float4 co = s_co[e];
                const float dx = xy.x - pxf, dy = xy.y - pyf;
                const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                if (power <= 0.0f && power >= s_thr[e]) {
                    const float G = expf_repro(power);
                    const float alpha = fminf(0.99f, co.w * G);
                    if (alpha >= 1.0f / 255.0f) {
                        active = true;
                        const float rom = __builtin_amdgcn_rcpf(1.0f - alpha);
                        T = T * rom;
                        w = alpha * T;
                        const float4 cd = s_rgbd[e];
                        float dot = cd.x * g0;
                        dot = __builtin_fmaf(cd.y, g1, dot);
                        dot = __builtin_fmaf(cd.z, g2, dot);
                        dot = __builtin_fmaf(cd.w, gD, dot);
                        dot += S[e];
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
            wv[e] = w;
            if (__any(active)) {
                float v[16];
                v[0] = w * g0; v[1] = w * g1; v[2] = w * g2; v[3] = w * gD;
                v[4] = gm2x; v[5] = gm2y; v[6] = gcx; v[7] = gcy; v[8] = gcw; v[9] = gop;
#pragma unroll
                for (int q = 10; q < 16; ++q) v[q] = 0.0f;
                wave_transpose_reduce<16>(v);
                const int q = transpose_reduce_slot<16>(lane);
                if ((lane & 3) == 0 && q < 10) atomicAdd(a.acc_small + (size_t)s_gid[e] * 12 + q, v[0]);
            }
        }

        // ---- 5. MFMA2: dF[e][c] = sum_px W[px][e] G[px][c] --------------------------------------
        {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                bf16x4 h4, l4;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    __bf16 h, l;
                    split_bf16(wv[4 * q + j], h, l);
                    h4[j] = h; l4[j] = l;
                }
                *reinterpret_cast<bf16x4*>(s_Wh + lane * WWP + 4 * q) = h4;
                *reinterpret_cast<bf16x4*>(s_Wl + lane * WWP + 4 * q) = l4;
            }
            wave_lds_sync();
            f32x4 dacc[2] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                const int row = 32 * kb + 8 * g4 + (l16 >> 2), col = 4 * (l16 & 3);
                const bf16x4 h0 = ds_read_tr16(s_Wh + row * WWP + col), h1 = ds_read_tr16(s_Wh + (row + 4) * WWP + col);
                const bf16x4 l0 = ds_read_tr16(s_Wl + row * WWP + col), l1 = ds_read_tr16(s_Wl + (row + 4) * WWP + col);
                const bf16x8 ah = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
                const bf16x8 al = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    dacc[nb] = LSR_MFMA16(ah, b2h[kb][nb], dacc[nb]);
                    dacc[nb] = LSR_MFMA16(ah, b2l[kb][nb], dacc[nb]);
                    dacc[nb] = LSR_MFMA16(al, b2h[kb][nb], dacc[nb]);
                }
            }
            // dacc[nb][i] at lane (g4, c): entry 4 g4 + i, channel 16 nb + c
            if (a.acc_lang) {
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int e = 4 * g4 + i;
                    if (e >= cnt) continue;
                    const size_t rowoff = (size_t)s_gid[e] * C;
#pragma unroll
                    for (int nb = 0; nb < 2; ++nb) {
                        const int ch = 16 * nb + l16;
                        if (ch < C && dacc[nb][i] != 0.0f) atomicAdd(a.acc_lang + rowoff + ch, dacc[nb][i]);
                    }
                }
            }
            wave_lds_sync();
        }
    }
}

void launch_render_bwd_wave(const RenderBwdArgs& a, hipStream_t st) {
    const int ntiles = a.grid_x * a.grid_y;
    hipLaunchKernelGGL(k_render_bwd_wave, dim3(((ntiles + 7) / 8) * 32), dim3(64), 0, st, a);
}

}  // namespace lsr
