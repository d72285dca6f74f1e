// render_fwd_wave.hip -- front-to-back compositing, one independent wave per 8x8 pixel quadrant.
//
// The compositor forward: upstream renderCUDA restated -- alpha <= 0.99,
// skip alpha < 1/255, stop when T (1 - alpha) < 1e-4, RGB += T bg, language channels without
// background, depth = sum z alpha T; per tile the largest n_contrib of its pixels (the backward's
// replay bound).  Every channel count runs here: VALU sums for C <= 16 or > 32, and
// render_fwd_mfma_wave.hip for 17..32 channels (sums on matrix cores).  About two thirds of a tile's list entries touch no pixel of
// a given quadrant; an entry that no pixel of the quadrant blends leaves every pixel's T and
// sums unchanged, and the contributor count upstream writes to n_contrib is the list position of
// the last blended entry + 1, so skipping such entries is exact.  Each wave
//   1. scans the tile list front to back, 64 entries per round, one per lane: the entry's
//      quadrant bit (the conservative ellipse-vs-quadrant test quad_may_touch, evaluated once per
//      instance by the binning, k_emit) and a ballot compaction into a per-wave FIFO in LDS
//      (list order kept);
//   2. composites the surviving entries in groups of GF staged in LDS (geometry + language row),
//      and stops as soon as every pixel of the quadrant has saturated.
// 64-thread blocks, no block barriers; the four quadrants of a tile run on one XCD.
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

template <int CPAD>
__global__ void __launch_bounds__(64) k_render_fwd_wave(RenderFwdBatch ab) {
    const RenderFwdArgs& a = ab.v[blockIdx.y];   // grid row = view
    constexpr int GF = 32, FIFO = 128, LP = CPAD > 0 ? CPAD : 1;
    __shared__ float4 s_co[GF];
    __shared__ float4 s_rgbd[GF];
    __shared__ float2 s_xy[GF];
    __shared__ uint32_t s_k[GF];
    __shared__ __attribute__((aligned(16))) float s_lang[GF * LP];
    __shared__ uint32_t s_fk[FIFO];
    __shared__ uint32_t s_fg[FIFO];

    const int b = blockIdx.x;
    const int slot = (b >> 5) * 8 + (b & 7), quad = (b >> 3) & 3;   // a slot's 4 quadrants: one XCD
    if (slot >= a.grid_x * a.grid_y) return;
    // column by column, as k_render_fwd_wave_mfma (measured faster than raster order there)
    const int tile = a.tile_order ? (int)a.tile_order[slot] : (slot % a.grid_y) * a.grid_x + slot / a.grid_y;
    const int lane = threadIdx.x;
    const int tx = tile % a.grid_x, ty = tile / a.grid_x;
    const int qx0 = tx * LSR_TILE_X + (quad & 1) * 8, qy0 = ty * LSR_TILE_Y + (quad >> 1) * 8;
    const int px = qx0 + (lane & 7), py = qy0 + (lane >> 3);
    const bool inside = px < a.W && py < a.H;
    const float pxf = (float)px, pyf = (float)py;
    uint2 range = a.ranges[tile];
    if (range.x > range.y) {   // an empty tile: the tile sort's range atomics left the preset (~0, 0)
        range = make_uint2(0u, 0u);
        if (quad == 0 && lane == 0) a.ranges[tile] = range;   // upstream's (0, 0) for the backward
    }
    const int C = a.C;

    float T = 1.0f;
    uint32_t last = 0;
    float acc[3] = {0.0f, 0.0f, 0.0f};
    float accL[LP];
#pragma unroll
    for (int c = 0; c < LP; ++c) accL[c] = 0.0f;
    float accD = 0.0f;
    bool done = !inside;

    uint32_t pos = range.x;  // list entries [pos, range.y) not yet scanned
    int head = 0, tail = 0;  // FIFO counters (wave-uniform)
    // point-list words of the next scan round, loaded one round ahead
    uint32_t w_next = pos + lane < range.y ? *at32(a.point_list, pos + lane) : 0u;
    while (!__all(done)) {
        // ---- 1. scan + compaction -----------------------------------------------------------
        while (tail - head < GF && pos < range.y) {
            const uint32_t idx = pos + lane;
            const uint32_t word = w_next;
            w_next = idx + 64 < range.y ? *at32(a.point_list, idx + 64) : 0u;
            const uint32_t gid = word & PL_ID_MASK;
            const bool cand = idx < range.y && ((word >> (PL_QUAD_SHIFT + quad)) & 1u);
            const uint64_t m = __ballot(cand);
            if (cand) {
                const int s = (tail + __popcll(m & lanemask_lt())) & (FIFO - 1);
                s_fk[s] = idx - range.x;
                s_fg[s] = gid;
            }
            tail += __popcll(m);
            pos += 64;
        }
        const int cnt = min(GF, tail - head);
        if (cnt == 0) break;
        wave_lds_sync();
        // ---- 2. stage the group ---------------------------------------------------------------
        if (lane < GF) {
            const bool ok = lane < cnt;
            const int s = (head + lane) & (FIFO - 1);
            const uint32_t gid = ok ? s_fg[s] : 0u;
            const float4 co = ok ? a.conic_o[gid] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            s_k[lane] = ok ? s_fk[s] : 0u;
            s_xy[lane] = ok ? a.xy[gid] : make_float2(0.0f, 0.0f);
            s_co[lane] = stage_conic(co);   // (-a/2, -b, -c/2, o): gauss_power's operands
            s_rgbd[lane] = ok ? a.rgbd[gid] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        }
        if constexpr (CPAD > 0) {
            if (C == CPAD) {   // whole rows as float4, every load in flight at once
                constexpr int R4 = CPAD / 4, NQ = (GF * R4 + 63) / 64;
                float4 v[NQ];
#pragma unroll
                for (int j = 0; j < NQ; ++j) {
                    const int q = lane + 64 * j, e = q / R4, c4 = q - e * R4;
                    v[j] = q < cnt * R4 ? reinterpret_cast<const float4*>(a.lang + (size_t)s_fg[(head + e) & (FIFO - 1)] * CPAD)[c4]
                                        : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                }
#pragma unroll
                for (int j = 0; j < NQ; ++j) {
                    const int q = lane + 64 * j;
                    if (q < GF * R4) reinterpret_cast<float4*>(s_lang)[q] = v[j];
                }
            } else {
                for (int q = lane; q < cnt * CPAD; q += 64) {
                    const int e = q / CPAD, c = q - e * CPAD;
                    const uint32_t gid = s_fg[(head + e) & (FIFO - 1)];
                    s_lang[q] = c < C ? a.lang[(size_t)gid * C + c] : 0.0f;
                }
            }
        }
        head += cnt;
        wave_lds_sync();
        // ---- 3. composite the group in list order, FB entries at a time: the per-entry alphas are
        //      independent of T, so they are computed branch-free for the whole batch first (their
        //      exp chains overlap); then the serial front-to-back update uses selects, with the
        //      channel accumulation skipped only when no lane of the wave blends the entry.
        //      Per pixel the arithmetic and its order are upstream's (a skipped entry adds exact
        //      zeros nowhere: its accumulation is not executed or has w = 0 and is not applied).
        constexpr int FB = 8;
        for (int e0 = 0; e0 < cnt; e0 += FB) {
            float al[FB], pw[FB];
            bool ok[FB];
#pragma unroll
            for (int u = 0; u < FB; ++u) {
                const float2 xy = s_xy[e0 + u];
                const float4 co = s_co[e0 + u];
                const float dx = xy.x - pxf, dy = xy.y - pyf;
                pw[u] = gauss_power(co.x, co.y, co.z, dx, dy);
            }
#pragma unroll
            for (int u = 0; u < FB; u += 2) {   // two entries per packed-fp32 exp
                const lsr_f2 g2 = expf_repro2(lsr_f2{pw[u], pw[u + 1]});
                al[u] = fminf(0.99f, s_co[e0 + u].w * g2.x);
                al[u + 1] = fminf(0.99f, s_co[e0 + u + 1].w * g2.y);
            }
#pragma unroll
            for (int u = 0; u < FB; ++u) ok[u] = e0 + u < cnt && pw[u] <= 0.0f && al[u] >= 1.0f / 255.0f;
#pragma unroll
            for (int u = 0; u < FB; ++u) {
                const float alpha = al[u];
                const float test_T = T * (1.0f - alpha);
                bool blend = ok[u] && !done;
                done = done || (blend && test_T < 0.0001f);
                blend = blend && !done;
                if (!__any(blend)) continue;                       // wave-uniform
                const int e = e0 + u;
                const float w = blend ? alpha * T : 0.0f;   // w = 0: fma(c, 0, acc) == acc
                const float4 cd = s_rgbd[e];
                acc[0] = __builtin_fmaf(cd.x, w, acc[0]);
                acc[1] = __builtin_fmaf(cd.y, w, acc[1]);
                acc[2] = __builtin_fmaf(cd.z, w, acc[2]);
                accD = __builtin_fmaf(cd.w, w, accD);
                if constexpr (CPAD > 0) {
                    const float4* f4 = reinterpret_cast<const float4*>(s_lang + e * CPAD);
#pragma unroll
                    for (int c4 = 0; c4 < CPAD / 4; ++c4) {
                        const float4 f = f4[c4];
                        accL[4 * c4 + 0] = __builtin_fmaf(f.x, w, accL[4 * c4 + 0]);
                        accL[4 * c4 + 1] = __builtin_fmaf(f.y, w, accL[4 * c4 + 1]);
                        accL[4 * c4 + 2] = __builtin_fmaf(f.z, w, accL[4 * c4 + 2]);
                        accL[4 * c4 + 3] = __builtin_fmaf(f.w, w, accL[4 * c4 + 3]);
                    }
                }
                T = blend ? test_T : T;
                last = blend ? s_k[e] + 1 : last;
            }
            if (__all(done)) break;
        }
        wave_lds_sync();
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
    // per-tile bound for the backward replay (tile_max_contrib is zeroed before the launch)
    uint32_t m = last;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    if (lane == 0 && m > 0) atomicMax(a.tile_max_contrib + tile, m);
}

template <int CPAD>
static void go_fwd_wave(const RenderFwdBatch& ab, int n, hipStream_t st) {
    const int ntiles = ab.v[0].grid_x * ab.v[0].grid_y;
    hipLaunchKernelGGL(k_render_fwd_wave<CPAD>, dim3(((ntiles + 7) / 8) * 32, n), dim3(64), 0, st, ab);
}

// n <= LSR_MAX_VIEWS views sharing the image size, C and include_feature
void launch_render_fwd_wave_views(const RenderFwdArgs* a, int n, hipStream_t st) {
    const int C = a[0].include_feature ? a[0].C : 0;
    if (lang_pad(C) == 32) {   // channel sums on matrix cores
        launch_render_fwd_wave_mfma_views(a, n, st);
        return;
    }
    RenderFwdBatch ab{};
    for (int v = 0; v < n; ++v) ab.v[v] = a[v];
    switch (lang_pad(C)) {
        case 0: go_fwd_wave<0>(ab, n, st); break;
        case 4: go_fwd_wave<4>(ab, n, st); break;
        case 8: go_fwd_wave<8>(ab, n, st); break;
        case 16: go_fwd_wave<16>(ab, n, st); break;
        default: go_fwd_wave<64>(ab, n, st); break;
    }
}

// the entry point of every forward composite: the forward takes no cost order, so
// the tile-order scratch is not written
void launch_render_fwd_views(const RenderFwdArgs* a, int n, hipStream_t st) {
    RenderFwdArgs f[LSR_MAX_VIEWS];
    for (int v = 0; v < n; ++v) {
        f[v] = a[v];
        f[v].tile_order = nullptr;
    }
    launch_render_fwd_wave_views(f, n, st);
}

}  // namespace lsr
