// render_bwd.hip -- backward of the compositing.
//
// Replays each tile's list back to front, as upstream, from the last contributor: T is
// recovered by T / (1 - alpha); dL/dalpha uses the accum_rec recurrence; the 0.99 clamp is
// ignored in dL/dG; the background enters through -T_final / (1 - alpha) (bg . dL/dpix_rgb);
// means2D gradients are in NDC units (x 0.5 W, 0.5 H).
//
// Mechanics (same mathematics, different data movement):
//   * accum_rec is carried as one scalar per pixel, accum_rec . dL/dpix: dL/dalpha only needs
//     sum_ch (c_ch - accum_rec_ch) g_ch = c . g - accum_rec . g, and accum_rec . g obeys the same
//     linear recurrence.  This removes 2 (3 + C + 1) registers per pixel.
//   * the replay starts at the tile's largest n_contrib (recorded by the forward);
//   * lanes skip exp when power < ln(1 / (255 o)) - 1e-3 (alpha < 1/255 for certain);
//   * per (Gaussian, wave) the 10 + C per-pixel contributions are summed over the 64 lanes by a
//     transpose-reduce (permlane32/16 swaps + DPP), which leaves one quantity per lane; the four
//     waves of the tile add them into an LDS record (one ds_add per lane).  Then, per
//     (Gaussian, tile):
//       default        one atomic wave-instruction adds the record to the Gaussian's accumulators
//                      (10 floats + the C language floats: two contiguous segments); the atomics
//                      overlap the replay, which is VALU-bound;
//       deterministic  the record is written with plain stores at the Gaussian's instance slot
//                      and the per-Gaussian reduction (preprocess.hip) sums them in a fixed order,
//                      so the gradients are bitwise reproducible.
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

template <int CPAD, int BATCH, int Q, bool DET>
__global__ void __launch_bounds__(256) k_render_bwd(RenderBwdArgs a) {
    constexpr int RECQ = 12 + CPAD;
    static_assert(RECQ <= Q || Q == 128, "quantities must fit the transpose-reduce width");
    constexpr int NSLOT = DET ? 4 : 1;          // deterministic: one partial record per wave, summed in order
    __shared__ float s_rec[NSLOT * BATCH * RECQ];
    __shared__ float s_lang[CPAD > 0 ? BATCH * CPAD : 1];
    __shared__ float4 s_co[BATCH];
    __shared__ float4 s_rgbd[BATCH];
    __shared__ float2 s_xy[BATCH];
    __shared__ float s_thr[BATCH];
    __shared__ uint32_t s_id[BATCH];
    __shared__ uint32_t s_inst[BATCH];
    __shared__ uint32_t s_act[BATCH];

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
        __syncthreads();                        // previous batch fully written out
        if (tid < nb) {
            const uint32_t gid = a.point_list[range.x + first + tid] & PL_ID_MASK;
            const float2 xy = a.xy[gid];
            const float4 co = a.conic_o[gid];
            s_id[tid] = gid;
            s_xy[tid] = xy;
            s_co[tid] = co;
            s_rgbd[tid] = a.rgbd[gid];
            s_thr[tid] = skip_power(co.w);
            // record slot: the Gaussian's first instance + this tile's index among its emitted ones
            s_inst[tid] = a.inst_off[gid] + rect_local_index(a.rect[gid], (uint32_t)tx, (uint32_t)ty);
            s_act[tid] = 0;
        }
        for (int e = tid; e < NSLOT * BATCH * RECQ; e += 256) s_rec[e] = 0.0f;
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
                const float power = gauss_power(-0.5f * co.x, -co.y, -0.5f * co.z, dx, dy);
                if (power <= 0.0f && power >= s_thr[j]) {
                    const float G = expf_repro(power);
                    const float alpha = fminf(0.99f, co.w * G);
                    if (alpha >= 1.0f / 255.0f) {
                        active = true;
                        const float om = 1.0f - alpha;
                        T = T * __builtin_amdgcn_rcpf(om);
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
                        acc_dot = __builtin_fmaf(last_alpha, last_dot, (1.0f - last_alpha) * acc_dot);
                        last_dot = dot;
                        float dL_dalpha = (dot - acc_dot) * T;
                        last_alpha = alpha;
                        dL_dalpha = __builtin_fmaf(-T_final * __builtin_amdgcn_rcpf(om), bg_dot, dL_dalpha);
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
            float v[Q];
            v[0] = w * g[0]; v[1] = w * g[1]; v[2] = w * g[2]; v[3] = w * gD;
            v[4] = gm2x; v[5] = gm2y; v[6] = gcx; v[7] = gcy; v[8] = gcw; v[9] = gop;
            v[10] = 0.0f; v[11] = 0.0f;
#pragma unroll
            for (int c = 0; c < CPAD; ++c) v[12 + c] = w * gL[c];
#pragma unroll
            for (int q = RECQ; q < Q; ++q) v[q] = 0.0f;
            wave_transpose_reduce<Q>(v);
            float* rec = s_rec + ((DET ? wave * BATCH : 0) + j) * RECQ;
            if constexpr (Q <= 64) {
                const int q = transpose_reduce_slot<Q>(lane);
                if ((lane & (64 / Q - 1)) == 0 && q < RECQ) {
                    if constexpr (DET) rec[q] = v[0];
                    else atomicAdd(rec + q, v[0]);
                }
            } else {
#pragma unroll
                for (int kk = 0; kk < Q / 64; ++kk) {
                    const int q = kk + (Q / 64) * lane;
                    if (q < RECQ) {
                        if constexpr (DET) rec[q] = v[kk];
                        else atomicAdd(rec + q, v[kk]);
                    }
                }
            }
            if (lane == 0) s_act[j] = 1u;
        }
        __syncthreads();
        if constexpr (DET) {
            // write the batch's records (only entries with a contributing pixel), float4 at a time
            constexpr int R4 = RECQ / 4;
            for (int e = tid; e < nb * R4; e += 256) {
                const int j = e / R4, c4 = e - j * R4;
                if (s_act[j]) {
                    float4 t = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#pragma unroll
                    for (int w4 = 0; w4 < NSLOT; ++w4) {   // fixed order over the waves
                        const float4 u = reinterpret_cast<const float4*>(s_rec + (w4 * BATCH + j) * RECQ)[c4];
                        t.x += u.x; t.y += u.y; t.z += u.z; t.w += u.w;
                    }
                    reinterpret_cast<float4*>(a.rec + (size_t)s_inst[j] * RECQ)[c4] = t;
                }
            }
            if (tid < nb && s_act[tid]) a.flags[s_inst[tid]] = 1;
        } else {
            // one atomic per quantity of each active entry; consecutive lanes -> consecutive addresses
            for (int e = tid; e < nb * RECQ; e += 256) {
                const int j = e / RECQ, q = e - j * RECQ;
                if (!s_act[j] || q == 10 || q == 11) continue;
                const uint32_t gid = s_id[j];
                if (q < 12) atomicAdd(a.acc_small + (size_t)gid * ACC_PITCH + q, s_rec[e]);
                else if (a.acc_lang && q - 12 < C) atomicAdd(a.acc_lang + (size_t)gid * C + (q - 12), s_rec[e]);
            }
        }
    }
}

template <int CPAD, int BATCH, int Q>
static void go_bwd(const RenderBwdArgs& a, hipStream_t st) {
    if (a.deterministic) hipLaunchKernelGGL((k_render_bwd<CPAD, (BATCH > 32 ? 32 : BATCH), Q, true>), dim3(a.grid_x * a.grid_y), dim3(256), 0, st, a);
    else hipLaunchKernelGGL((k_render_bwd<CPAD, BATCH, Q, false>), dim3(a.grid_x * a.grid_y), dim3(256), 0, st, a);
}

void launch_render_bwd(const RenderBwdArgs& a, hipStream_t st) {
    const int C = a.include_feature ? a.C : 0;
    if (!a.deterministic && C <= 32) {
        launch_render_bwd_wave_views(&a, 1, st);   // compacted per-quadrant waves, pixel sums on matrix cores
        return;
    }
    switch (lang_pad(C)) {               // deterministic records, or 64 channels
        case 0: go_bwd<0, 64, 16>(a, st); break;
        case 4: go_bwd<4, 64, 16>(a, st); break;
        case 8: go_bwd<8, 64, 32>(a, st); break;
        case 16: go_bwd<16, 64, 32>(a, st); break;
        case 32: go_bwd<32, 64, 64>(a, st); break;
        default: go_bwd<64, 32, 128>(a, st); break;
    }
}

}  // namespace lsr
