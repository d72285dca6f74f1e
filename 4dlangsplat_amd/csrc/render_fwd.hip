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
            const uint32_t g = a.point_list[start + tid];
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
            const float power = -0.5f * (co.x * dx * dx + co.z * dy * dy) - co.y * dx * dy;
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

template <int CPAD, int BATCH>
static void go_fwd(const RenderFwdArgs& a, hipStream_t st) {
    hipLaunchKernelGGL((k_render_fwd<CPAD, BATCH>), dim3(a.grid_x * a.grid_y), dim3(256), 0, st, a);
}

void launch_render_fwd(const RenderFwdArgs& a, hipStream_t st) {
    const int C = a.include_feature ? a.C : 0;
    if (C == 0) go_fwd<0, 256>(a, st);
    else if (C <= 4) go_fwd<4, 256>(a, st);
    else if (C <= 8) go_fwd<8, 256>(a, st);
    else if (C <= 16) go_fwd<16, 128>(a, st);
    else if (C <= 32) go_fwd<32, 128>(a, st);
    else go_fwd<64, 64>(a, st);
}

}  // namespace lsr
