// render_bwd.hip -- backward of the compositing.
//
// Replays each tile's list back to front, as upstream, from the last contributor: T is
// recovered by T / (1 - alpha); dL/dalpha uses the accum_rec recurrence; the 0.99 clamp is
// ignored in dL/dG; the background enters through -T_final / (1 - alpha) (bg . dL/dpix_rgb);
// means2D gradients are in NDC units (x 0.5 W, 0.5 H).
//
// Differences in mechanics (same mathematics):
//   * accum_rec is carried as one scalar per pixel, accum_rec . dL/dpix, since dL/dalpha only
//     needs that dot product: sum_ch (c_ch - accum_rec_ch) g_ch = c . g - accum_rec . g, and
//     accum_rec . g obeys the same linear recurrence.  This drops 2 (3 + C + 1) registers.
//   * the replay starts at the tile's largest n_contrib (recorded by the forward), not at the end
//     of the list;
//   * per-pixel contributions are summed over the wave before one atomic per (Gaussian, wave),
//     instead of one atomic per (Gaussian, pixel); waves with no contributing pixel skip it.
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

template <int CPAD, int BATCH>
__global__ void __launch_bounds__(256) k_render_bwd(RenderBwdArgs a) {
    __shared__ uint32_t s_id[BATCH];
    __shared__ float2 s_xy[BATCH];
    __shared__ float4 s_co[BATCH];
    __shared__ float4 s_rgbd[BATCH];
    __shared__ float s_lang[CPAD > 0 ? BATCH * CPAD : 1];

    const int tile = blockIdx.x;
    const int tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
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
    float g[3] = {0.0f, 0.0f, 0.0f}, gD = 0.0f;
    float gL[CPAD > 0 ? CPAD : 1];
#pragma unroll
    for (int c = 0; c < (CPAD > 0 ? CPAD : 1); ++c) gL[c] = 0.0f;
    if (inside) {
        g[0] = a.dL_dcolor[pid]; g[1] = a.dL_dcolor[HW + pid]; g[2] = a.dL_dcolor[2 * HW + pid];
        if (a.dL_ddepth) gD = a.dL_ddepth[pid];
        if constexpr (CPAD > 0) {
            if (a.dL_dlang) {
#pragma unroll
                for (int c = 0; c < CPAD; ++c) gL[c] = c < C ? a.dL_dlang[(size_t)c * HW + pid] : 0.0f;
            }
        }
    }
    const float bg_dot = a.bg[0] * g[0] + a.bg[1] * g[1] + a.bg[2] * g[2];
    const float ddelx_dx = 0.5f * (float)a.W, ddely_dy = 0.5f * (float)a.H;
    float acc_dot = 0.0f, last_dot = 0.0f, last_alpha = 0.0f;

    // entries [range.x, range.x + nreplay) in reverse, BATCH at a time
    for (int end = (int)nreplay; end > 0; end -= BATCH) {
        const int nb = min(BATCH, end);
        const int first = end - nb;             // list position of batch slot 0
        __syncthreads();
        if (tid < nb) {
            const uint32_t gid = a.point_list[range.x + first + tid];
            s_id[tid] = gid;
            s_xy[tid] = a.xy[gid];
            s_co[tid] = a.conic_o[gid];
            s_rgbd[tid] = a.rgbd[gid];
        }
        if constexpr (CPAD > 0) {
            __syncthreads();
            for (int e = tid; e < nb * CPAD; e += 256) {
                const int j = e / CPAD, c = e - j * CPAD;
                s_lang[e] = c < C ? a.lang[(size_t)s_id[j] * C + c] : 0.0f;
            }
        }
        __syncthreads();
        for (int j = nb - 1; j >= 0; --j) {
            const uint32_t k = (uint32_t)(first + j);   // position in the tile list (contributor index)
            bool active = false;
            float w = 0.0f, gm2x = 0.0f, gm2y = 0.0f, gcx = 0.0f, gcy = 0.0f, gcw = 0.0f, gop = 0.0f;
            if (k < last_contributor) {
                const float2 xy = s_xy[j];
                const float4 co = s_co[j];
                const float dx = xy.x - pxf, dy = xy.y - pyf;
                const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
                if (power <= 0.0f) {
                    const float G = expf_repro(power);
                    const float alpha = fminf(0.99f, co.w * G);
                    if (alpha >= 1.0f / 255.0f) {
                        active = true;
                        T = T / (1.0f - alpha);
                        w = alpha * T;
                        const float4 cd = s_rgbd[j];
                        float dot = cd.x * g[0];
                        dot = __builtin_fmaf(cd.y, g[1], dot);
                        dot = __builtin_fmaf(cd.z, g[2], dot);
                        dot = __builtin_fmaf(cd.w, gD, dot);
                        if constexpr (CPAD > 0) {
                            const float4* f4 = reinterpret_cast<const float4*>(s_lang + j * CPAD);
#pragma unroll
                            for (int c4 = 0; c4 < CPAD / 4; ++c4) {
                                const float4 f = f4[c4];
                                dot = __builtin_fmaf(f.x, gL[4 * c4 + 0], dot);
                                dot = __builtin_fmaf(f.y, gL[4 * c4 + 1], dot);
                                dot = __builtin_fmaf(f.z, gL[4 * c4 + 2], dot);
                                dot = __builtin_fmaf(f.w, gL[4 * c4 + 3], dot);
                            }
                        }
                        acc_dot = last_alpha * last_dot + (1.0f - last_alpha) * acc_dot;
                        last_dot = dot;
                        float dL_dalpha = (dot - acc_dot) * T;
                        last_alpha = alpha;
                        dL_dalpha += (-T_final / (1.0f - alpha)) * bg_dot;
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
            if (!__any(active)) continue;
            // wave sums; lane (q mod 64) of round q / 64 then issues the atomic for quantity q
            constexpr int NQ = 10 + CPAD, ROUNDS = (NQ + 63) / 64;
            const uint32_t gid = s_id[j];
            float mine[ROUNDS];
            float* dst[ROUNDS];
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r) { mine[r] = 0.0f; dst[r] = nullptr; }
#define LSR_TAKE(q, expr, ptr)                                   \
            {                                                    \
                const float v_ = wave_sum(expr);                 \
                if (lane == ((q) & 63)) { mine[(q) >> 6] = v_; dst[(q) >> 6] = (ptr); } \
            }
            LSR_TAKE(0, w * g[0], a.g_color + 3 * (size_t)gid)
            LSR_TAKE(1, w * g[1], a.g_color + 3 * (size_t)gid + 1)
            LSR_TAKE(2, w * g[2], a.g_color + 3 * (size_t)gid + 2)
            LSR_TAKE(3, gm2x, &a.g_mean2D[gid].x)
            LSR_TAKE(4, gm2y, &a.g_mean2D[gid].y)
            LSR_TAKE(5, gcx, &a.g_conic[gid].x)
            LSR_TAKE(6, gcy, &a.g_conic[gid].y)
            LSR_TAKE(7, gcw, &a.g_conic[gid].z)
            LSR_TAKE(8, w * gD, &a.g_conic[gid].w)
            LSR_TAKE(9, gop, a.g_opacity ? a.g_opacity + gid : nullptr)
            if constexpr (CPAD > 0) {
#pragma unroll
                for (int c = 0; c < CPAD; ++c)
                    LSR_TAKE(10 + c, w * gL[c], (a.g_lang && c < C) ? a.g_lang + (size_t)gid * C + c : nullptr)
            }
#undef LSR_TAKE
#pragma unroll
            for (int r = 0; r < ROUNDS; ++r)
                if (dst[r]) atomicAdd(dst[r], mine[r]);
        }
    }
}

template <int CPAD, int BATCH>
static void go_bwd(const RenderBwdArgs& a, hipStream_t st) {
    hipLaunchKernelGGL((k_render_bwd<CPAD, BATCH>), dim3(a.grid_x * a.grid_y), dim3(256), 0, st, a);
}

void launch_render_bwd(const RenderBwdArgs& a, hipStream_t st) {
    const int C = a.include_feature ? a.C : 0;
    if (C == 0) go_bwd<0, 256>(a, st);
    else if (C <= 4) go_bwd<4, 256>(a, st);
    else if (C <= 8) go_bwd<8, 256>(a, st);
    else if (C <= 16) go_bwd<16, 128>(a, st);
    else if (C <= 32) go_bwd<32, 128>(a, st);
    else go_bwd<64, 64>(a, st);
}

}  // namespace lsr
