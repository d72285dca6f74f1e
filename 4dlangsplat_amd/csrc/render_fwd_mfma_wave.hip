// render_fwd_mfma_wave.hip -- front-to-back compositing for 17..32 language channels, the channel
// sums on matrix cores.
//
// Same waves, entry compaction and per-pixel arithmetic as k_render_fwd_wave (render_fwd_wave.hip;
// upstream renderCUDA): one independent wave per 8x8 quadrant, the tile
// list scanned front to back with the conservative ellipse-vs-quadrant test, groups of 32
// compacted entries staged in LDS.  T, the contributor count, RGB and depth stay per-pixel fp32
// VALU arithmetic in upstream's order (so n_contrib, final_T and the colour are those of the
// scalar kernel).  The language channels are the dense part: per group,
//     L[c][p] += sum_e F[e][c] w[e][p],      w = alpha T (0 where the entry does not blend)
// a [32 channels x 32 entries] x [32 entries x 64 pixels] product, 8 v_mfma_f32_16x16x32_bf16
// blocks, each operand split in bf16 hi + lo (three products, ~2^-17 relative, fp32
// accumulation; lsr_mfma.h).  A = F^T comes from the group's bf16 rows [e][c] in LDS through
// transposing reads; B = w is built in registers: each lane packs its pixel's 32 weights in four
// octets and a 4x4 lane-group transpose (permlane swaps) hands every lane the octet of the pixel
// its B fragment needs.  This takes the 32 per-entry channel FMAs off the VALU.
#include "lsr_common.h"
#include "lsr_internal.h"
#include "lsr_mfma.h"

namespace lsr {

namespace {
constexpr int MG = 32;      // entries per group (= MFMA K)
constexpr int MFP = 40;     // F row pitch in bf16: 32 channels + 8 (80-byte rows)
constexpr int MFIFO = 128;  // compacted entries waiting; power of two

// pack 8 weights as bf16 hi / lo octets
__device__ __forceinline__ void pack_octet(const float (&w)[8], bf16x8& h, bf16x8& l) {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        __bf16 hh, ll;
        split_bf16(w[j], hh, ll);
        h[j] = hh;
        l[j] = ll;
    }
}

// lane group g holds octets x[0..3] (one per entry octet o) of its own pixel; afterwards it holds
// in x[nb] the octet g of pixel 16 nb + (lane & 15): the MFMA B fragments, nb = pixel block
__device__ __forceinline__ void octets_to_b(bf16x8 (&x)[4]) {
    typedef float f4v __attribute__((ext_vector_type(4)));
#pragma unroll
    for (int d = 0; d < 4; ++d) {   // per dword of the octets
        float t[4];
#pragma unroll
        for (int o = 0; o < 4; ++o) t[o] = __builtin_bit_cast(f4v, x[o])[d];
        transpose_lane_groups(t);
#pragma unroll
        for (int o = 0; o < 4; ++o) {
            f4v v = __builtin_bit_cast(f4v, x[o]);
            v[d] = t[o];
            x[o] = __builtin_bit_cast(bf16x8, v);
        }
    }
}
}  // namespace

// Diagnostic build only (-DLSR_FWD_STAMPS): per-segment s_memtime sums of the group loop into
// g_fwd_stamps (lsr_debug_fwd_stamps).  Read shares, not times.
#ifdef LSR_FWD_STAMPS
__device__ unsigned long long g_fwd_stamps[8];
#define FWD_STAMP(seg)                                                                           \
    do {                                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        unsigned long long t_;                                                                   \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");              \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        if ((seg) > 0) st_sum[(seg) - 1] += t_ - st_prev;                                         \
        st_prev = t_;                                                                            \
    } while (0)
#else
#define FWD_STAMP(seg) do {} while (0)
#endif

// Diagnostic build only (-DLSR_FWD_COUNT): (entry, pixel) pairs the waves evaluate (inside the
// image, entries of the group, while the wave runs) and the pairs that blend, summed into
// g_fwd_count (lsr_debug_fwd_count): how much of the per-pair work contributes.
#ifdef LSR_FWD_COUNT
// [0] pairs evaluated, [1] pairs blended, [2] waves, [3] compacted entries the waves processed, [4] of
// those, entries that no pixel of the quadrant blends placed BEFORE the quadrant's last blending entry
// (what the backward replays and an exact per-(entry, quadrant) activity bit would let it skip)
__device__ unsigned long long g_fwd_count[5];
#endif

#ifndef LSR_FWD_WAVES
#define LSR_FWD_WAVES 4   // waves per SIMD the register budget targets (3: 0.293 ms, 4: 0.268 ms)
#endif
// PRE: C == 32 with the language rows' bf16 hi / lo made once per batch (a.lang_split).  A variant
// that gathered every read of the group loop by LDS-DMA ran a wave's loop in 0.85x the cycles but
// was no faster (the waves then contend for issue); it was removed in round 3.
template <bool PRE>
__global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(LSR_FWD_WAVES, LSR_FWD_WAVES)))
k_render_fwd_wave_mfma(RenderFwdBatch ab) {
    const RenderFwdArgs& a = ab.v[blockIdx.y];   // grid row = view
    // group entries, one array per field (a b64 read of a pair = one packed-fp32 operand): centre
    // X, Y; staged conic -a/2, -b, -c/2 (gauss_power); opacity (0 past the group: never blends); (r, g) and (b, depth) pairs
    __shared__ __attribute__((aligned(16))) float s_X[MG], s_Y[MG], s_A[MG], s_B[MG], s_C[MG], s_O[MG];
    __shared__ lsr_f2 s_RG[MG], s_BD[MG];
    __shared__ uint32_t s_k[MG];   // list position + 1 (the n_contrib value of a blend)
    __shared__ __attribute__((aligned(16))) __bf16 s_Fh[MG * MFP];
    __shared__ __attribute__((aligned(16))) __bf16 s_Fl[MG * MFP];
    __shared__ uint32_t s_fk[MFIFO];
    __shared__ uint32_t s_fg[MFIFO];

    const int b = blockIdx.x;
    const int slot = (b >> 5) * 8 + (b & 7), quad = (b >> 3) & 3;   // a slot's 4 quadrants: one XCD
    if (slot >= a.grid_x * a.grid_y) return;
    // Slots walk the tiles column by column (no order array): measured 0.250 -> 0.232 ms against
    // raster order on the headline scene (either column direction; a per-quadrant makespan
    // simulation from the frame's composited-entry counts also favours it, 1.20 vs 1.26 of ideal).
    const int tile = a.tile_order ? (int)a.tile_order[slot] : (slot % a.grid_y) * a.grid_x + slot / a.grid_y;
    const int lane = threadIdx.x, g4 = lane >> 4, l16 = lane & 15;
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
    lsr_f2 acc_rg = {0.0f, 0.0f}, acc_bd = {0.0f, 0.0f};   // (r, g), (b, depth)
    const lsr_f2 px2 = {pxf, pxf}, py2 = {pyf, pyf};
    f32x4 L[2][4];   // L[mb][nb]: channels 16 mb + 4 g4 + i, pixels 16 nb + l16
#pragma unroll
    for (int mb = 0; mb < 2; ++mb)
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) L[mb][nb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
    bool done = !inside;
#ifdef LSR_FWD_COUNT
    uint32_t c_eval = 0, c_act = 0, c_ent = 0, c_inact_run = 0, c_inact_before = 0;
#endif

    uint32_t pos = range.x;  // list entries [pos, range.y) not yet scanned
    int head = 0, tail = 0;  // FIFO counters (wave-uniform)
    // scan prefetch: point-list words (id | quadrant bits, k_emit) of the next two rounds
    uint32_t w_c = pos + lane < range.y ? *at32(a.point_list, pos + lane) : 0u;
    uint32_t w_n = pos + 64 + lane < range.y ? *at32(a.point_list, pos + 64 + lane) : 0u;
#ifdef LSR_FWD_STAMPS
    unsigned long long st_sum[4] = {0, 0, 0, 0}, st_prev = 0;
#endif
    // scan rounds until `want` entries wait in the FIFO or the list is exhausted
    auto scan_fill = [&](int want) __attribute__((always_inline)) {
        while (tail - head < want && pos < range.y) {
            const uint32_t idx = pos + lane;
            const uint32_t word = w_c;
            w_c = w_n;
            w_n = idx + 128 < range.y ? *at32(a.point_list, idx + 128) : 0u;
            const uint32_t gid = word & PL_ID_MASK;
            const bool cand = idx < range.y && ((word >> (PL_QUAD_SHIFT + quad)) & 1u);
            const uint64_t m = __ballot(cand);
            if (cand) {
                const int s = (tail + __popcll(m & lanemask_lt())) & (MFIFO - 1);
                s_fk[s] = idx - range.x;
                s_fg[s] = gid;
            }
            tail += __popcll(m);
            pos += 64;
        }
    };
    // composite FIFO group [.., cnt) staged in the SoA arrays and F rows, then its channel sums
    auto composite = [&](int cnt) __attribute__((always_inline)) {
        // ---- 3. per pixel, front to back: alphas of 8 entries branch-free, then the serial
        //      update with selects (as k_render_fwd_wave); the weights go to octets ----------------
        bf16x8 oh[4], ol[4];
#pragma unroll
        for (int o = 0; o < 4; ++o) {
            float w8[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) w8[u] = 0.0f;
            if (8 * o < cnt && !__all(done)) {                    // wave-uniform
                float al[8];
                bool ok[8];
#ifdef LSR_FWD_SCALAR
#pragma unroll
                for (int u = 0; u < 8; ++u) {   // A/B variant: scalar VALU (build with -fno-slp-vectorize)
                    const int e = 8 * o + u;
                    const float pw = gauss_power(s_A[e], s_B[e], s_C[e], s_X[e] - pxf, s_Y[e] - pyf);
                    al[u] = fminf(0.99f, s_O[e] * expf_repro(pw));
                    ok[u] = pw <= 0.0f && al[u] >= 1.0f / 255.0f;
                }
#else
#pragma unroll
                for (int u = 0; u < 8; u += 2) {   // two entries per packed-fp32 operation
                    const int e = 8 * o + u;
                    auto ld2 = [&](const float* base) { return *reinterpret_cast<const lsr_f2*>(base + e); };
                    const lsr_f2 X = ld2(s_X), Y = ld2(s_Y), A = ld2(s_A), B = ld2(s_B), Cc = ld2(s_C), O = ld2(s_O);
                    const lsr_f2 dx = X - px2, dy = Y - py2;
                    const lsr_f2 pw = gauss_power2(A, B, Cc, dx, dy);
                    const lsr_f2 og = O * expf_repro2(pw);
                    al[u] = fminf(0.99f, og.x);
                    al[u + 1] = fminf(0.99f, og.y);
                    ok[u] = pw.x <= 0.0f && al[u] >= 1.0f / 255.0f;        // padding entries: O = 0
                    ok[u + 1] = pw.y <= 0.0f && al[u + 1] >= 1.0f / 255.0f;
                }
#endif
#pragma unroll
                for (int u = 0; u < 8; ++u) {
                    const int e = 8 * o + u;
                    const float alpha = al[u];
                    const float test_T = T * (1.0f - alpha);
                    bool blend = ok[u] && !done;
                    done = done || (blend && test_T < 0.0001f);
                    blend = blend && !done;
                    const float w = blend ? alpha * T : 0.0f;   // w = 0: fma(c, 0, acc) == acc
                    acc_rg = __builtin_elementwise_fma(s_RG[e], lsr_f2{w, w}, acc_rg);
                    acc_bd = __builtin_elementwise_fma(s_BD[e], lsr_f2{w, w}, acc_bd);
                    w8[u] = w;
#ifdef LSR_FWD_COUNT
                    c_eval += (inside && e < cnt) ? 1u : 0u;
                    c_act += blend ? 1u : 0u;
                    if (e < cnt) {   // wave-uniform
                        ++c_ent;
                        if (__ballot(blend) != 0) { c_inact_before += c_inact_run; c_inact_run = 0; }
                        else ++c_inact_run;
                    }
#endif
                    T = blend ? test_T : T;
                    last = blend ? s_k[e] : last;   // s_k holds the list position + 1
                }
            }
            pack_octet(w8, oh[o], ol[o]);
        }
        FWD_STAMP(3);
        // ---- 4. language channels on matrix cores -----------------------------------------------
        octets_to_b(oh);
        octets_to_b(ol);
#pragma unroll
        for (int mb = 0; mb < 2; ++mb) {
            // A[m = channel 16 mb + l16][k = entry 8 g4 + j] from the rows [e][c]
            const int off = (8 * g4 + (l16 >> 2)) * MFP + 16 * mb + 4 * (l16 & 3);
            const bf16x8 ah = __builtin_shufflevector(ds_read_tr16(s_Fh + off), ds_read_tr16(s_Fh + off + 4 * MFP),
                                                      0, 1, 2, 3, 4, 5, 6, 7);
            const bf16x8 alo = __builtin_shufflevector(ds_read_tr16(s_Fl + off), ds_read_tr16(s_Fl + off + 4 * MFP),
                                                       0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
            for (int nb = 0; nb < 4; ++nb) {
                L[mb][nb] = LSR_MFMA16(ah, oh[nb], L[mb][nb]);
                L[mb][nb] = LSR_MFMA16(ah, ol[nb], L[mb][nb]);
                L[mb][nb] = LSR_MFMA16(alo, oh[nb], L[mb][nb]);
            }
        }
    };
    {
        while (!__all(done)) {
            FWD_STAMP(0);
            scan_fill(MG);
            const int cnt = min(MG, tail - head);
            if (cnt == 0) break;
            wave_lds_sync();
            FWD_STAMP(1);
            // ---- 2. stage the group: geometry, and the language rows as bf16 hi / lo -------------
            // every gather of the group is issued before the first LDS store (one memory latency per
            // group instead of three in sequence)
            {
                // lane -> entry lane / 2, channels 16 (lane & 1) .. +15: four float4 loads in flight
                const int e = lane >> 1, c0 = 16 * (lane & 1);
                const bool ok = e < cnt;
                const uint32_t gid = ok ? s_fg[(head + e) & (MFIFO - 1)] : 0u;
                constexpr bool pre = PRE;   // C == 32, hi / lo made once per batch (a.lang_split)
                float f[16];   // pre: the bits of hi channels c0 .. +15 in f[0..7], lo in f[8..15]
                if constexpr (pre) {     // hi at [gid][c0], lo at [gid][32 + c0] (a uint4 holds 8 bf16)
                    const float4* q = reinterpret_cast<const float4*>(a.lang_split);
#pragma unroll
                    for (int u = 0; u < 4; ++u) {
                        const float4 v = *at32(q, gid * 8u + (uint32_t)(c0 >> 3) + (u & 1) + 4u * (u >> 1));
                        f[4 * u] = v.x; f[4 * u + 1] = v.y; f[4 * u + 2] = v.z; f[4 * u + 3] = v.w;
                    }
                } else if (C == 32) {
                    const float4* r = reinterpret_cast<const float4*>(a.lang + (size_t)gid * 32 + c0);
#pragma unroll
                    for (int q = 0; q < 4; ++q) {   // unmasked (gid 0 is a valid row), zeroed after
                        const float4 v = r[q];
                        f[4 * q] = v.x; f[4 * q + 1] = v.y; f[4 * q + 2] = v.z; f[4 * q + 3] = v.w;
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 16; ++j) f[j] = (ok && c0 + j < C) ? a.lang[(size_t)gid * C + c0 + j] : 0.0f;
                }
                float2 g_xy = make_float2(0.0f, 0.0f);
                float4 g_co = make_float4(0.0f, 0.0f, 0.0f, 0.0f), g_rgbd = g_co;
                uint32_t g_k = 0u;
                if (lane < MG && lane < cnt) {
                    const int s = (head + lane) & (MFIFO - 1);
                    const uint32_t gid = s_fg[s];
                    g_k = s_fk[s];
                    g_xy = a.xy[gid];
                    g_co = a.conic_o[gid];
                    g_rgbd = a.rgbd[gid];
                }
                if constexpr (pre) {
#pragma unroll
                    for (int j = 0; j < 16; ++j) f[j] = ok ? f[j] : 0.0f;   // +0.0 = bf16 zeros
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        *reinterpret_cast<float4*>(s_Fh + e * MFP + c0 + 8 * h) =
                            make_float4(f[4 * h], f[4 * h + 1], f[4 * h + 2], f[4 * h + 3]);
                        *reinterpret_cast<float4*>(s_Fl + e * MFP + c0 + 8 * h) =
                            make_float4(f[8 + 4 * h], f[8 + 4 * h + 1], f[8 + 4 * h + 2], f[8 + 4 * h + 3]);
                    }
                } else {
                    if (C == 32) {
#pragma unroll
                        for (int j = 0; j < 16; ++j) f[j] = ok ? f[j] : 0.0f;
                    }
#pragma unroll
                    for (int h = 0; h < 2; ++h) {
                        bf16x8 vh, vl;
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            __bf16 hh, ll;
                            split_bf16(f[8 * h + j], hh, ll);
                            vh[j] = hh;
                            vl[j] = ll;
                        }
                        *reinterpret_cast<bf16x8*>(s_Fh + e * MFP + c0 + 8 * h) = vh;
                        *reinterpret_cast<bf16x8*>(s_Fl + e * MFP + c0 + 8 * h) = vl;
                    }
                }
                if (lane < MG) {
                    s_k[lane] = g_k + 1u;
                    s_X[lane] = g_xy.x; s_Y[lane] = g_xy.y;
                    s_A[lane] = -0.5f * g_co.x; s_B[lane] = -g_co.y; s_C[lane] = -0.5f * g_co.z; s_O[lane] = g_co.w;
                    s_RG[lane] = lsr_f2{g_rgbd.x, g_rgbd.y};
                    s_BD[lane] = lsr_f2{g_rgbd.z, g_rgbd.w};
                }
            }
            head += cnt;
            wave_lds_sync();
            FWD_STAMP(2);
            composite(cnt);
            wave_lds_sync();   // the group's LDS rows are read before the next staging
            FWD_STAMP(4);
        }
    }
#ifdef LSR_FWD_COUNT
    {
        unsigned long long ve = c_eval, va = c_act;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            ve += __shfl_xor(ve, off);
            va += __shfl_xor(va, off);
        }
        if (lane == 0) {
            atomicAdd(&g_fwd_count[0], ve);
            atomicAdd(&g_fwd_count[1], va);
            atomicAdd(&g_fwd_count[2], 1ull);
            atomicAdd(&g_fwd_count[3], (unsigned long long)c_ent);
            atomicAdd(&g_fwd_count[4], (unsigned long long)c_inact_before);
        }
    }
#endif
#ifdef LSR_FWD_STAMPS
    if (lane < 4) {
        unsigned long long v = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) v = lane == k ? st_sum[k] : v;
        atomicAdd(&g_fwd_stamps[lane], v);
    }
    if (lane == 4) atomicAdd(&g_fwd_stamps[4], 1ull);
#endif
    if (inside) {
        const size_t HW = (size_t)a.H * a.W, pid = (size_t)py * a.W + px;
        a.final_T[pid] = T;
        a.n_contrib[pid] = last;
        a.out_color[pid] = acc_rg.x + T * a.bg[0];
        a.out_color[HW + pid] = acc_rg.y + T * a.bg[1];
        a.out_color[2 * HW + pid] = acc_bd.x + T * a.bg[2];
        a.out_depth[pid] = acc_bd.y;
    }
    {   // language: block (mb, nb), register i -> channel 16 mb + 4 g4 + i, pixel 16 nb + l16
        const size_t HW = (size_t)a.H * a.W;
#pragma unroll
        for (int nb = 0; nb < 4; ++nb) {
            const int p = 16 * nb + l16, qx = qx0 + (p & 7), qy = qy0 + (p >> 3);
            if (qx >= a.W || qy >= a.H) continue;
            const size_t pid = (size_t)qy * a.W + qx;
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int i = 0; i < 4; ++i) {
                    const int c = 16 * mb + 4 * g4 + i;
                    if (c < C) a.out_lang[(size_t)c * HW + pid] = L[mb][nb][i];
                }
        }
    }
    uint32_t m = last;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) m = max(m, (uint32_t)__shfl_xor((int)m, o));
    if (lane == 0 && m > 0) atomicMax(a.tile_max_contrib + tile, m);
}

// lsr_language_split: per Gaussian the 32 channels' bf16 hi then lo (split_bf16), one thread per
// 8 channels (two 16-byte loads, two 16-byte stores)
__global__ void __launch_bounds__(256) k_language_split(int P, const float* __restrict__ lang, uint16_t* __restrict__ out) {
    const uint32_t i = blockIdx.x * 256u + threadIdx.x;
    if (i >= 4u * (uint32_t)P) return;
    const uint32_t g = i >> 2, c8 = i & 3u;
    const float4* src = reinterpret_cast<const float4*>(lang);
    const float4 x = *at32(src, g * 8u + 2u * c8), y = *at32(src, g * 8u + 2u * c8 + 1u);
    const float f[8] = {x.x, x.y, x.z, x.w, y.x, y.y, y.z, y.w};
    bf16x8 h, l;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        __bf16 hh, ll;
        split_bf16(f[j], hh, ll);
        h[j] = hh;
        l[j] = ll;
    }
    bf16x8* dst = reinterpret_cast<bf16x8*>(out);
    dst[g * 8u + c8] = h;
    dst[g * 8u + 4u + c8] = l;
}

void launch_language_split(int P, const float* lang, uint16_t* out, hipStream_t st) {
    if (P > 0) hipLaunchKernelGGL(k_language_split, dim3((unsigned)((4u * (uint32_t)P + 255u) / 256u)), dim3(256), 0, st, P, lang, out);
}

void launch_render_fwd_wave_mfma_views(const RenderFwdArgs* a, int n, hipStream_t st) {
    RenderFwdBatch ab{};
    for (int v = 0; v < n; ++v) ab.v[v] = a[v];
    const int ntiles = a[0].grid_x * a[0].grid_y;
    const dim3 grid(((ntiles + 7) / 8) * 32, n);
    if (a[0].lang_split && a[0].C == 32)
        hipLaunchKernelGGL((k_render_fwd_wave_mfma<true>), grid, dim3(64), 0, st, ab);
    else
        hipLaunchKernelGGL((k_render_fwd_wave_mfma<false>), grid, dim3(64), 0, st, ab);
}

}  // namespace lsr

#ifdef LSR_FWD_COUNT
extern "C" int lsr_debug_fwd_count(unsigned long long* out5) {
    if (hipMemcpyFromSymbol(out5, HIP_SYMBOL(lsr::g_fwd_count), 5 * sizeof(unsigned long long)) != hipSuccess) return 2;
    unsigned long long z[5] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(lsr::g_fwd_count), z, sizeof(z)) == hipSuccess ? 0 : 2;
}
#endif
#ifdef LSR_FWD_STAMPS
extern "C" int lsr_debug_fwd_stamps(unsigned long long* out5) {
    if (hipMemcpyFromSymbol(out5, HIP_SYMBOL(lsr::g_fwd_stamps), 5 * sizeof(unsigned long long)) != hipSuccess) return 2;
    unsigned long long z[8] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(lsr::g_fwd_stamps), z, sizeof(z)) == hipSuccess ? 0 : 2;
}
#endif
