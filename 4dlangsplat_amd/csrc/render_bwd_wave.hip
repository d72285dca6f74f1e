// render_bwd_wave.hip -- compositor backward, one independent wave per 8x8 pixel quadrant, every
// per-Gaussian sum over pixels on matrix cores.
//
// Same mathematics as render_bwd.hip (upstream backward).  Measured on the
// headline scene, only a third of the replayed list entries touch any pixel of a given 8x8
// quadrant.  An entry that no pixel of the quadrant activates changes neither T nor the
// back-to-front accumulators of any of its pixels, so skipping it is exact.  Each wave therefore
//   1. scans its replay range (up to the largest n_contrib of its pixels) back to front, 64
//      entries per round, one per lane: the entry's quadrant bit (the conservative
//      ellipse-vs-quadrant test quad_may_touch, evaluated once per instance by the binning,
//      k_emit) and a ballot compaction into a per-wave FIFO in LDS;
//   2. processes the surviving entries in groups of 16 (WG).  Per group, with pixels p on lanes:
//        MFMA1   S[e][p] = sum_c F[e][c] G[p][c]           language part of dot(c_e, dL/dpix)
//        serial  the back-to-front recurrence per pixel: w = alpha T and t = G dL/dalpha
//        MFMA-W  sum_p w[p][e] [G[p][c] | g_rgb,depth[p]]   dL/dlanguage, dL/dcolour, dL/ddepth
//        MFMA-T  sum_p t[p][e] {1, x, y, x^2, xy, y^2}(p)   pixel moments, from which the mean2D,
//                                                         conic and opacity gradients follow exactly
//                                                         (dx = X_e - x, dy = Y_e - y in quadrant-
//                                                         local coordinates: well conditioned)
//      all on v_mfma_f32_16x16x32_bf16 with hi/lo bf16 splits (lsr_mfma.h; the moment operand is
//      small integers, exact in bf16), then one global atomic per (entry, quantity).
// No block barriers: 64-thread blocks, the four quadrants of a tile on one XCD.
#include "lsr_common.h"
#include "lsr_internal.h"
#include "lsr_mfma.h"

namespace lsr {

// Diagnostic build only (-DLSR_BWD_STAMPS): per-segment s_memtime sums of the group loop, summed
// over all waves into g_bwd_stamps (read by lsr_debug_bwd_stamps).  Read shares, not times.
#ifdef LSR_BWD_STAMPS
__device__ unsigned long long g_bwd_stamps[16];
#define BWD_STAMP(seg)                                                                           \
    do {                                                                                         \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        unsigned long long t_;                                                                   \
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");              \
        __builtin_amdgcn_sched_barrier(0);                                                       \
        if ((seg) > 0) st_sum[(seg) - 1] += t_ - st_prev;                                         \
        st_prev = t_;                                                                            \
    } while (0)
#else
#define BWD_STAMP(seg) do {} while (0)
#endif

constexpr int WG = 16;       // compacted entries per MFMA group
constexpr int WFP = 48;      // F row pitch in bf16 (32 channels + 16): the MFMA1 b128 reads conflict-free
// W / t rows [p][e]: 16 bf16 (32 B) per pixel p, unpadded and swizzled so that both the row
// writes (ds_write_b64: 16-lane groups over 32 banks) and the transposing MFMA-operand reads
// (ds_read_b64_tr_b16: 32-lane halves over 64 banks) are conflict-free: pixel p's row sits in row
// slot p ^ 4 [(p >> 3) & 1] and its 8-byte chunk q (entries 4q .. 4q + 3) in chunk q ^ ((p >> 2) & 3).
// (The padded 40-byte rows cost 2 extra LDS cycles per transposing read.)
__device__ __forceinline__ int wt_off(int p, int q) { return (p ^ (((p >> 3) & 1) << 2)) * 16 + 4 * (q ^ ((p >> 2) & 3)); }
constexpr int WFIFO = 128;   // compacted entries waiting (list positions and ids); power of two
// G rows [p][c] (the pixels' language gradients, 32 channels, bf16 hi and lo) stay in LDS for the
// whole wave instead of as 64 VGPRs of resident B fragments: 64 B per row, unpadded, with 16-byte
// chunk q of row p in chunk q ^ ((p >> 2) & 3), so both per-group reads are conflict-free -- MFMA1's
// B (row 16 pb + l16, chunk g4: 16 rows x 4 dwords over 64 banks) and MFMA-W's B through transposing
// reads (4 rows x 16 columns per 16-lane group, two groups eight rows apart per half-wave).
__device__ __forceinline__ int g_off(int p, int q) { return p * 32 + 8 * (q ^ ((p >> 2) & 3)); }

// C32: the 32-channel instantiation (headline), whose language rows are two float4 loads per lane
// with no per-channel predication.  NOL: no language channels in play (include_feature off or
// C = 0: the RGB-only training and render.py passes): the F rows, MFMA1, the language half of
// MFMA-W and its staging and atomics are compiled out, and the 64 VGPRs of B fragments they hold
// with them, so the instantiation targets twice the occupancy.
#ifndef LSR_BWD_WAVES
#define LSR_BWD_WAVES 2   // waves per SIMD the register budget targets
#endif
#ifndef LSR_BWD_WAVES_NOL
#define LSR_BWD_WAVES_NOL 3
#endif
template <bool C32, bool PRE, bool NOL>
__global__ void __launch_bounds__(64)
__attribute__((amdgpu_waves_per_eu(NOL ? LSR_BWD_WAVES_NOL : LSR_BWD_WAVES, NOL ? LSR_BWD_WAVES_NOL : LSR_BWD_WAVES)))
k_render_bwd_wave(RenderBwdBatch ab) {
    const RenderBwdArgs& a = ab.v[blockIdx.y];   // grid row = view
#ifdef LSR_BWD_STAMPS
    unsigned long long st_entry;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_entry)::"memory");
#endif
    static_assert(!(NOL && C32), "NOL has no language channels");
    __shared__ __attribute__((aligned(16))) __bf16 s_FR[64 * 32];        // bm build, then F / W / t rows
    __shared__ __attribute__((aligned(16))) __bf16 s_Gh[NOL ? 8 : 64 * 32];   // G rows (g_off), hi / lo
    __shared__ __attribute__((aligned(16))) __bf16 s_Gl[NOL ? 8 : 64 * 32];
    // group entries' screen-space data, one array per field (a b128 read gives 4 entries, a b64
    // pair the operand of a packed-fp32 instruction): centre X, Y; staged conic -a/2, -b, -c/2 (gauss_power); opacity; rgb,
    // depth; list position k (0xFFFFFFFF past the group: never active)
    __shared__ __attribute__((aligned(16))) float s_X[WG], s_Y[WG], s_A[WG], s_B[WG], s_C[WG], s_O[WG];
    __shared__ __attribute__((aligned(16))) float s_R[WG], s_Gc[WG], s_Bc[WG], s_D[WG];
    __shared__ uint32_t s_gid[WG];
    __shared__ __attribute__((aligned(16))) uint32_t s_k[WG];
    __shared__ float s_mom[WG][10];   // pitch 10: the moment stores and loads conflict-free
    // results of the previous group, staged for its atomics (issued one iteration late, see 6.)
    __shared__ float s_q[WG][17];   // per-entry scalar gradients in acc_small record order (0..9); pitch 17 (banks)
    __shared__ float s_lq[WG][36];  // dL/dlanguage rows [e][c] (pitch 36: conflict-free stores and loads)
    __shared__ uint32_t s_agid[WG];
    __shared__ uint32_t s_fk[WFIFO];
    __shared__ uint32_t s_fg[WFIFO];

    const int b = blockIdx.x;
    const int slot = (b >> 5) * 8 + (b & 7), quad = (b >> 3) & 3;   // a slot's 4 quadrants: one XCD
    if (slot >= a.grid_x * a.grid_y) return;
    // longest-first order (k_tile_order); column-major measured 0.61 vs 0.49 ms here
    const int tile = a.tile_order ? (int)a.tile_order[slot] : slot;
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
#ifdef LSR_BWD_STAMPS
    unsigned long long st_nrep;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_nrep)::"memory");
#endif
    const uint2 range = a.ranges[tile];
    const int C = C32 ? 32 : (NOL ? 0 : (a.include_feature ? a.C : 0));   // language channels in play
    const float bx0 = (float)qx0, by0 = (float)qy0;

    const float T_final = inside ? a.final_T[pid] : 0.0f;
    float T = T_final;
    float g0 = 0.0f, g1 = 0.0f, g2 = 0.0f, gD = 0.0f;
    if (inside) {
        g0 = a.dL_dcolor[pid]; g1 = a.dL_dcolor[HW + pid]; g2 = a.dL_dcolor[2 * HW + pid];
        if (a.dL_ddepth) gD = a.dL_ddepth[pid];
    }

    // ---- B operands.  The language ones are read from the G rows in LDS per group:
    // MFMA1 B   (pixel block pb): K = channel 8 g4 + j,       N = pixel 16 pb + l16      (g_b1)
    // MFMA-W B  (kb, nb)        : K = pixel 32 kb + 8 g4 + j, N = channel 16 nb + l16    (g_b2)
    // bm[kb] (resident): MFMA-T and the rgb / depth part of MFMA-W, K = pixel 32 kb + 8 g4 + j,
    //              N = l16: the moments {1, x, y, x^2, xy, y^2} (exact small integers) in columns
    //              0..5, the pixel's rgb + depth gradients as bf16 hi in 6..9 and lo in 10..13, 0 in
    //              14, 15 (one fragment for both products: each reads only its own columns)
    bf16x8 bm[2];
    {
        if constexpr (!NOL) {   // this lane's pixel row of G, hi and lo
            float gl[32];
#pragma unroll
            for (int c = 0; c < 32; ++c)
                gl[c] = (inside && a.dL_dlang && c < C) ? a.dL_dlang[(size_t)c * HW + pid] : 0.0f;
#pragma unroll
            for (int c8 = 0; c8 < 4; ++c8) {
                bf16x8 vh, vl;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    __bf16 h, l;
                    split_bf16(gl[8 * c8 + j], h, l);
                    vh[j] = h; vl[j] = l;
                }
                *reinterpret_cast<bf16x8*>(s_Gh + g_off(lane, c8)) = vh;
                *reinterpret_cast<bf16x8*>(s_Gl + g_off(lane, c8)) = vl;
            }
        }
        // bm rows [p][n], pitch 16: pixel p = lane has local x = p & 7, y = p >> 3
        {
            const float x = (float)(lane & 7), y = (float)(lane >> 3);
            const float gv[4] = {g0, g1, g2, gD};
            bf16x8 r0, r1;
            r0[0] = (__bf16)1.0f; r0[1] = (__bf16)x; r0[2] = (__bf16)y;
            r0[3] = (__bf16)(x * x); r0[4] = (__bf16)(x * y); r0[5] = (__bf16)(y * y);
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                __bf16 h, l;
                split_bf16(gv[c], h, l);
                if (c < 2) r0[6 + c] = h; else r1[c - 2] = h;
                r1[2 + c] = l;
            }
            r1[6] = (__bf16)0.0f; r1[7] = (__bf16)0.0f;
            *reinterpret_cast<bf16x8*>(s_FR + lane * 16) = r0;
            *reinterpret_cast<bf16x8*>(s_FR + lane * 16 + 8) = r1;
            wave_lds_sync();
#pragma unroll
            for (int kb = 0; kb < 2; ++kb) {
                const __bf16* p = s_FR + (32 * kb + 8 * g4 + (l16 >> 2)) * 16 + 4 * (l16 & 3);
                bm[kb] = __builtin_shufflevector(ds_read_tr16(p), ds_read_tr16(p + 4 * 16), 0, 1, 2, 3, 4, 5, 6, 7);
            }
            wave_lds_sync();
        }
    }
    // MFMA1's B: pixel rows 16 pb + l16, channels 8 g4 .. + 7
    auto g_b1 = [&](const __bf16* G, int pb) {
        return *reinterpret_cast<const bf16x8*>(G + g_off(16 * pb + l16, g4));
    };
    // MFMA-W's B: pixels 32 kb + 8 g4 + j, channel 16 nb + l16 (two transposing reads, rows +0 / +4)
    auto g_b2 = [&](const __bf16* G, int kb, int nb) {
        const int p = 32 * kb + 8 * g4 + (l16 >> 2), q = 2 * nb + ((l16 & 3) >> 1), o = 4 * (l16 & 1);
        const bf16x4 lo4 = ds_read_tr16(G + g_off(p, q) + o), hi4 = ds_read_tr16(G + g_off(p + 4, q) + o);
        return __builtin_shufflevector(lo4, hi4, 0, 1, 2, 3, 4, 5, 6, 7);
    };
    __bf16* s_Fh = s_FR;              // F rows [e][c] of the group (MFMA1 A), hi
    __bf16* s_Fl = s_FR + WG * WFP;   // lo
    __bf16* s_Rh = s_FR;              // after MFMA1: W or t rows [p][e], hi
    __bf16* s_Rl = s_FR + 64 * 16;    // lo

    const float bg_dot = a.bg[0] * g0 + a.bg[1] * g1 + a.bg[2] * g2;
    const float bg_term = -T_final * bg_dot;   // the background term's per-pixel factor
    const float ddelx_dx = 0.5f * (float)a.W, ddely_dy = 0.5f * (float)a.H;
    float acc_dot = 0.0f, last_dot = 0.0f, last_alpha = 0.0f;
    const float pxf = (float)px, pyf = (float)py;

    int pos = (int)nrep;     // list positions [0, pos) not yet scanned
    int head = 0, tail = 0;  // FIFO counters (wave-uniform)
    // scan prefetch: point-list words (id | quadrant bits) of the round at positions
    // [pos - 64, pos), loaded at the end of the round before (one register, no rotation: a copy
    // of a register whose load is in flight makes hipcc wait for every outstanding load and atomic)
    // The loads are unconditional (positions clamped to 0, a valid entry; k < 0 is masked at use):
    // a conditional load would also become a register copy.
    uint32_t sc_w = *at32(a.point_list, range.x + max(pos - 64 + lane, 0));
    // scan rounds until `want` entries wait in the FIFO or the range is exhausted
    auto scan_fill = [&](int want) {
        while (tail - head < want && pos > 0) {
            const int k = pos - 64 + lane;       // this round's positions (k < 0: before the list)
            const uint32_t word = sc_w;
            const uint32_t gid = word & PL_ID_MASK;
            const bool cand = k >= 0 && ((word >> (PL_QUAD_SHIFT + quad)) & 1u);
            const uint64_t m = __ballot(cand);
            if (cand) {   // back to front: higher list positions first
                const int rank = lane == 63 ? 0 : __popcll(m >> (lane + 1));
                const int s = (tail + rank) & (WFIFO - 1);
                s_fk[s] = (uint32_t)k;
                s_fg[s] = gid;
            }
            tail += __popcll(m);
            pos = max(pos - 64, 0);
            sc_w = *at32(a.point_list, range.x + max(k - 64, 0));
        }
        wave_lds_sync();
    };
    // group prefetch registers: geometry of entry `lane` (lanes < WG), language row slice
    // (entry lane / 4, channels 8 (lane & 3) .. +7).  The loads are unconditional (no branches
    // around them): lanes past the group read row 0 (a valid row; those entries are never active
    // and their F rows only meet zero weights).
    struct Pf {
        uint32_t gid, k;
        float2 xy;
        float4 co, rgbd, f0, f1;
    };
    auto load_group = [&](Pf& pf, int n) __attribute__((always_inline)) {   // FIFO entries [head, head + n)
        {
            const bool ok = lane < n;
            const int s = (head + lane) & (WFIFO - 1);
            pf.gid = ok ? s_fg[s] : 0u;
            pf.k = ok ? s_fk[s] : 0xFFFFFFFFu;
            pf.xy = *at32(a.xy, pf.gid);
            pf.co = *at32(a.conic_o, pf.gid);
            pf.rgbd = *at32(a.rgbd, pf.gid);
        }
        const int e = lane >> 2, c0 = 8 * (lane & 3);
        const uint32_t gid = e < n ? s_fg[(head + e) & (WFIFO - 1)] : 0u;
        if constexpr (NOL) {
            (void)gid; (void)c0;
        } else if constexpr (C32) {
            if constexpr (PRE) {   // hi / lo made once per batch (lsr_language_split): bits in f0 / f1
                const uint4* q = reinterpret_cast<const uint4*>(a.lang_split);
                pf.f0 = __builtin_bit_cast(float4, *at32(q, gid * 8u + (uint32_t)(c0 >> 3)));
                pf.f1 = __builtin_bit_cast(float4, *at32(q, gid * 8u + 4u + (uint32_t)(c0 >> 3)));
            } else {
                const float4* r = reinterpret_cast<const float4*>(at32(a.lang, gid * 32u + c0));
                pf.f0 = r[0];
                pf.f1 = r[1];
            }
        } else {
            float f[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = (c0 + j < C) ? *at32(a.lang, gid * (uint32_t)C + c0 + j) : 0.0f;
            pf.f0 = make_float4(f[0], f[1], f[2], f[3]);
            pf.f1 = make_float4(f[4], f[5], f[6], f[7]);
        }
        head += n;
    };
    auto store_group = [&](const Pf& pf) __attribute__((always_inline)) {   // prefetched group -> LDS
        if (lane < WG) {
            s_gid[lane] = pf.gid;
            s_k[lane] = pf.k;
            s_X[lane] = pf.xy.x; s_Y[lane] = pf.xy.y;
            s_A[lane] = -0.5f * pf.co.x; s_B[lane] = -pf.co.y; s_C[lane] = -0.5f * pf.co.z; s_O[lane] = pf.co.w;
            s_R[lane] = pf.rgbd.x; s_Gc[lane] = pf.rgbd.y; s_Bc[lane] = pf.rgbd.z; s_D[lane] = pf.rgbd.w;
        }
        const int e = lane >> 2, c0 = 8 * (lane & 3);
        if constexpr (NOL) {
            (void)e; (void)c0;
        } else if constexpr (C32 && PRE) {
            *reinterpret_cast<uint4*>(s_Fh + e * WFP + c0) = __builtin_bit_cast(uint4, pf.f0);
            *reinterpret_cast<uint4*>(s_Fl + e * WFP + c0) = __builtin_bit_cast(uint4, pf.f1);
        } else {
            const float f[8] = {pf.f0.x, pf.f0.y, pf.f0.z, pf.f0.w, pf.f1.x, pf.f1.y, pf.f1.z, pf.f1.w};
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
        wave_lds_sync();
    };

    // ---- 6. atomics of a group, from its staged results (s_q, s_lq, s_agid).  vmcnt retires in
    //      order and counts no-return atomics too, so a wait on any load issued after an atomic
    //      also waits for the atomic (~1-3k cycles under load).  The atomics are therefore issued
    //      one iteration late, after the scan (whose point-list loads are waited on within the
    //      iteration) and just before the next group's prefetch: the first wait behind them is
    //      the following iteration's, a whole group of compute later.  Offsets are 32-bit (P * 32
    //      floats < 2^32 bytes) so the addresses are SGPR base + VGPR offset. ---------------------
    int acnt = 0;   // entries staged
    auto issue_atomics = [&]() {
        if (acnt == 0) return;
#ifdef LSR_BWD_ABL_LANGONLY   // timing ablation only: the language rows' atomics, not the small rows'
        constexpr bool kSmall = false;
#else
        constexpr bool kSmall = true;
#endif
#ifdef LSR_BWD_ABL_NOATOMIC   // timing ablation only (no gradients): the atomics' share
        acnt = 0;
        return;
#endif
        // every staged value and row offset read from LDS first (one wait), then the atomics
        const int ch = lane & 31, q = lane & 15;
        float lv[WG / 2], sv[WG / 4];
        uint32_t lo[WG / 2], so[WG / 4];
        if constexpr (!NOL) {
#pragma unroll
            for (int j = 0; j < WG / 2; ++j) {   // lane -> channel lane & 31 of entries (lane >> 5) + 2 j
                const int e = (lane >> 5) + 2 * j;
                lv[j] = s_lq[e][ch];
                lo[j] = s_agid[e] * (uint32_t)C + ch;
            }
        }
#pragma unroll
        for (int r = 0; r < WG / 4; ++r) {   // lane -> field lane & 15 of entry (lane >> 4) + 4 r
            const int e = (lane >> 4) + 4 * r;
            sv[r] = s_q[e][q];
            so[r] = s_agid[e] * (uint32_t)ACC_PITCH + q;
        }
        // A branch-free variant (every lane, zeros for idle lanes, so that hipcc could count the
        // atomics and skip them in its waits for later loads) measured 0.70 vs 0.50 ms: with no
        // wait behind them a wave keeps several groups of atomics in flight and the memory
        // system backs up.  The wait that follows each batch throttles them.
        if (!NOL && a.acc_lang) {   // 128-byte rows
#pragma unroll
            for (int j = 0; j < WG / 2; ++j)
                if ((lane >> 5) + 2 * j < acnt && ch < C && lv[j] != 0.0f) atomicAdd(at32(a.acc_lang, lo[j]), lv[j]);
        }
#pragma unroll
        for (int r = 0; r < WG / 4; ++r)
            if (kSmall && (lane >> 4) + 4 * r < acnt && q < 10 && sv[r] != 0.0f) atomicAdd(at32(a.acc_small, so[r]), sv[r]);
        acnt = 0;
    };

#ifdef LSR_BWD_STAMPS
    unsigned long long st_scan;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_scan)::"memory");
#endif
    scan_fill(WG);
    int cnt = min(WG, tail - head);
    Pf pf;
    if (cnt > 0) load_group(pf, cnt);
#ifdef LSR_BWD_STAMPS
    unsigned long long st_sum[8] = {0, 0, 0, 0, 0, 0, 0, 0}, st_prev = 0, st_loop;
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_loop)::"memory");
#endif
    while (cnt > 0) {
        BWD_STAMP(0);
        store_group(pf);
        BWD_STAMP(1);
        scan_fill(WG);
        BWD_STAMP(2);
        issue_atomics();   // the previous group's (staging is rewritten only at this group's end)
        BWD_STAMP(3);
        // next group's loads in flight while this one computes
        const int next_cnt = min(WG, tail - head);
        if (next_cnt > 0) load_group(pf, next_cnt);
        BWD_STAMP(4);

        // ---- 3. MFMA1: S[e][p], then to one pixel per lane -------------------------------------
        float S[WG];
        if constexpr (NOL) {
#pragma unroll
            for (int e = 0; e < WG; ++e) S[e] = 0.0f;
        } else {
            const bf16x8 ah = *reinterpret_cast<const bf16x8*>(s_Fh + l16 * WFP + 8 * g4);
            const bf16x8 al = *reinterpret_cast<const bf16x8*>(s_Fl + l16 * WFP + 8 * g4);
            f32x4 d[4];
#pragma unroll
            for (int pb = 0; pb < 4; ++pb) {
                const bf16x8 bh = g_b1(s_Gh, pb), bl = g_b1(s_Gl, pb);
                d[pb] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
                d[pb] = LSR_MFMA16(ah, bh, d[pb]);
                d[pb] = LSR_MFMA16(ah, bl, d[pb]);
                d[pb] = LSR_MFMA16(al, bh, d[pb]);
            }
            wave_lds_sync();   // F read before W overwrites it
            // d[pb][i] at lane (g4, c): entry 4 g4 + i, pixel 16 pb + c
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                float x[4] = {d[0][i], d[1][i], d[2][i], d[3][i]};
                transpose_lane_groups(x);
#pragma unroll
                for (int p = 0; p < 4; ++p) S[4 * p + i] = x[p];   // entry 4p + i, own pixel
            }
        }

        BWD_STAMP(5);
        // ---- 4. serial back-to-front replay of the group: w = alpha T, t = G dL/dalpha --------
        // Per entry, everything but the T / accumulator recurrence is independent of the other
        // entries: computed branch-free for the whole group first (exp chains overlap), then the
        // recurrence.  An inactive entry (upstream skips it) runs the recurrence with alpha = 0,
        // which leaves every state exactly as the skip does: T * rcp(1 - 0) = T * 1 = T; w = 0 T
        // = 0; its fold fma(last_alpha, last_dot - acc, acc) is the one the next active entry
        // would have made (same operands), and the next entry's fold, fma(0, x, acc) = acc, adds
        // nothing.  Only alpha and t are selected; no selects on T, acc, last_dot, last_alpha or w.
        float wv[WG], tv[WG];
        constexpr int RB = 2;   // entries per branch-free batch: one packed-fp32 pair (register budget)
        const lsr_f2 px2 = {pxf, pxf}, py2 = {pyf, pyf};
        // the pairs' entry data (one broadcast b64 read per field = a packed-fp32 operand), software-
        // pipelined: the next pair's reads are issued before this pair computes, so their LDS latency
        // hides behind it (the scheduler otherwise places each read right before its first use)
        struct PairIn {
            lsr_f2 X, Y, A, B, Cc, O, R, Gc, Bc, D;
            uint2 kk;
        };
        auto ld_pair = [&](int e0) __attribute__((always_inline)) {
            auto ld2 = [&](const float* base) { return *reinterpret_cast<const lsr_f2*>(base + e0); };
            PairIn q;
            q.X = ld2(s_X); q.Y = ld2(s_Y); q.A = ld2(s_A); q.B = ld2(s_B); q.Cc = ld2(s_C); q.O = ld2(s_O);
            q.R = ld2(s_R); q.Gc = ld2(s_Gc); q.Bc = ld2(s_Bc); q.D = ld2(s_D);
            q.kk = *reinterpret_cast<const uint2*>(s_k + e0);
            return q;
        };
        // (the RGB-only instantiation, at 3 waves per SIMD, has no registers for the prefetched pair)
        constexpr bool PIPE = !NOL;
        PairIn pin = ld_pair(0);
#pragma unroll
        for (int e0 = 0; e0 < WG; e0 += RB) {
        float Gv[RB], alv[RB], romv[RB], dotv[RB];
        bool act[RB];
        PairIn pnext;
        if constexpr (PIPE) {
            if (e0 + RB < WG) pnext = ld_pair(e0 + RB);
            __builtin_amdgcn_sched_barrier(0);   // keep the next pair's reads issued here
        } else if (e0 > 0) {
            pin = ld_pair(e0);
        }
#ifdef LSR_BWD_SCALAR
        // A/B variant: the pair's alpha / dot arithmetic as scalar VALU (no packed-fp32 hazard nops
        // between the dependent steps of the exp chain; build with -fno-slp-vectorize)
#pragma unroll
        for (int u = 0; u < 2; ++u) {
            const int e = e0 + u;
            const float Xu = u ? pin.X.y : pin.X.x, Yu = u ? pin.Y.y : pin.Y.x;
            const float power = gauss_power(u ? pin.A.y : pin.A.x, u ? pin.B.y : pin.B.x, u ? pin.Cc.y : pin.Cc.x,
                                            Xu - pxf, Yu - pyf);
            const float ge = expf_repro(power);
            const float al = fminf(0.99f, (u ? pin.O.y : pin.O.x) * ge);
            float d = (u ? pin.R.y : pin.R.x) * g0;
            d = __builtin_fmaf(u ? pin.Gc.y : pin.Gc.x, g1, d);
            d = __builtin_fmaf(u ? pin.Bc.y : pin.Bc.x, g2, d);
            d = __builtin_fmaf(u ? pin.D.y : pin.D.x, gD, d);
            act[u] = (u ? pin.kk.y : pin.kk.x) < last_contributor && power <= 0.0f && al >= 1.0f / 255.0f;
            alv[u] = act[u] ? al : 0.0f;
            Gv[u] = ge;
            romv[u] = __builtin_amdgcn_rcpf(1.0f - alv[u]);
            dotv[u] = d + S[e];
        }
        if (false)
#endif
        {
            const lsr_f2 X = pin.X, Y = pin.Y, A = pin.A, B = pin.B, Cc = pin.Cc, O = pin.O;
            const uint2 kk = pin.kk;
            // the forward's operation order per component (bit-identical alpha decisions)
            const lsr_f2 dx = X - px2, dy = Y - py2;
            const lsr_f2 pw = gauss_power2(A, B, Cc, dx, dy);
            const lsr_f2 ge = expf_repro2(pw);
            const lsr_f2 og = O * ge;
            lsr_f2 dot = pin.R * g0;
            dot = __builtin_elementwise_fma(pin.Gc, lsr_f2{g1, g1}, dot);
            dot = __builtin_elementwise_fma(pin.Bc, lsr_f2{g2, g2}, dot);
            dot = __builtin_elementwise_fma(pin.D, lsr_f2{gD, gD}, dot);
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int e = e0 + u;
                const float power = u ? pw.y : pw.x;
                const float al = fminf(0.99f, u ? og.y : og.x);
                act[u] = (u ? kk.y : kk.x) < last_contributor && power <= 0.0f && al >= 1.0f / 255.0f;
                alv[u] = act[u] ? al : 0.0f;
                Gv[u] = u ? ge.y : ge.x;
                romv[u] = __builtin_amdgcn_rcpf(1.0f - alv[u]);   // rcp(1) = 1 exactly
                dotv[u] = (u ? dot.y : dot.x) + S[e];
            }
        }
#pragma unroll
        for (int u = 0; u < RB; ++u) {
            const int e = e0 + u;
            const float alpha = alv[u], rom = romv[u], dot = dotv[u];
            T = T * rom;
            // upstream's last_alpha * last_c + (1 - last_alpha) * accum_rec, as one fma on the difference
            acc_dot = __builtin_fmaf(last_alpha, last_dot - acc_dot, acc_dot);
            last_dot = dot;
            last_alpha = alpha;
            float dL_dalpha = (dot - acc_dot) * T;
            dL_dalpha = __builtin_fmaf(rom, bg_term, dL_dalpha);   // (-T_final / (1 - alpha)) bg . dL/dpix
            wv[e] = alpha * T;
            tv[e] = act[u] ? Gv[u] * dL_dalpha : 0.0f;
        }
        if constexpr (PIPE) {
            if (e0 + RB < WG) pin = pnext;
        }
        }

        BWD_STAMP(6);
        // ---- 5. sums over the wave's pixels on matrix cores -----------------------------------
        // rows [p][e] of R (W, then t) in LDS; the A operand R^T comes from transposing reads
        auto write_rows = [&](const float (&r)[WG]) {
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                bf16x4 h4, l4;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    __bf16 h, l;
                    split_bf16(r[4 * q + j], h, l);
                    h4[j] = h; l4[j] = l;
                }
                *reinterpret_cast<bf16x4*>(s_Rh + wt_off(lane, q)) = h4;
                *reinterpret_cast<bf16x4*>(s_Rl + wt_off(lane, q)) = l4;
            }
            wave_lds_sync();
        };
        auto read_a = [&](int kb, bf16x8& ah, bf16x8& al) {
            const int row = 32 * kb + 8 * g4 + (l16 >> 2), o0 = wt_off(row, l16 & 3), o1 = wt_off(row + 4, l16 & 3);
            const bf16x4 h0 = ds_read_tr16(s_Rh + o0), h1 = ds_read_tr16(s_Rh + o1);
            const bf16x4 l0 = ds_read_tr16(s_Rl + o0), l1 = ds_read_tr16(s_Rl + o1);
            ah = __builtin_shufflevector(h0, h1, 0, 1, 2, 3, 4, 5, 6, 7);
            al = __builtin_shufflevector(l0, l1, 0, 1, 2, 3, 4, 5, 6, 7);
        };
        // MFMA-W: dacc[nb][i] at lane (g4, c) = sum_p w[p][4 g4 + i] G[p][16 nb + c] (language);
        //         dacc[2][i] at lane (g4, n) = sum_p w[p][4 g4 + i] bm[p][n] (n = 6..13: rgb / depth hi, lo)
        f32x4 dacc[3] = {f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}, f32x4{0.0f, 0.0f, 0.0f, 0.0f}};
        write_rows(wv);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            bf16x8 ah, al;
            read_a(kb, ah, al);
            if constexpr (!NOL) {
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) {
                    const bf16x8 bh = g_b2(s_Gh, kb, nb), bl = g_b2(s_Gl, kb, nb);
                    dacc[nb] = LSR_MFMA16(ah, bh, dacc[nb]);
                    dacc[nb] = LSR_MFMA16(ah, bl, dacc[nb]);
                    dacc[nb] = LSR_MFMA16(al, bh, dacc[nb]);
                }
            }
            dacc[2] = LSR_MFMA16(ah, bm[kb], dacc[2]);   // w hi and lo times g hi (6..9) and lo (10..13)
            dacc[2] = LSR_MFMA16(al, bm[kb], dacc[2]);
        }
        wave_lds_sync();   // W rows read before t overwrites them
        // MFMA-T: dmom[i] at lane (g4, n) = sum_p t[p][4 g4 + i] moment_n(p)
        f32x4 dmom = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        write_rows(tv);
#pragma unroll
        for (int kb = 0; kb < 2; ++kb) {
            bf16x8 ah, al;
            read_a(kb, ah, al);
            dmom = LSR_MFMA16(ah, bm[kb], dmom);
            dmom = LSR_MFMA16(al, bm[kb], dmom);
        }
        if (l16 < 6) {
#pragma unroll
            for (int i = 0; i < 4; ++i) s_mom[4 * g4 + i][l16] = dmom[i];
        }
        {   // rgb 0-2, depth 3: hi column 6 + c plus lo column 10 + c
            float v[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) v[i] = dacc[2][i] + __shfl_down(dacc[2][i], 4, 16);
            if (l16 >= 6 && l16 < 10) {
#pragma unroll
                for (int i = 0; i < 4; ++i) s_q[4 * g4 + i][l16 - 6] = v[i];
            }
        }
        BWD_STAMP(7);
        // stage the group's results: language rows from the MFMA layout, gids
        if constexpr (!NOL) {
#pragma unroll
            for (int i = 0; i < 4; ++i)
#pragma unroll
                for (int nb = 0; nb < 2; ++nb) s_lq[4 * g4 + i][16 * nb + l16] = dacc[nb][i];
        }
        if (lane < WG) s_agid[lane] = s_gid[lane];
        wave_lds_sync();
        if (lane < cnt) {   // moments -> mean2D (4-5), conic (6-8), opacity (9)
            const int e = lane;
            const float M0 = s_mom[e][0], Mx = s_mom[e][1], My = s_mom[e][2];
            const float Mxx = s_mom[e][3], Mxy = s_mom[e][4], Myy = s_mom[e][5];
            const float2 xy = make_float2(s_X[e], s_Y[e]);
            const float4 co = make_float4(-2.0f * s_A[e], -s_B[e], -2.0f * s_C[e], s_O[e]);   // staged (-a/2, -b, -c/2)
            const float X = xy.x - bx0, Y = xy.y - by0;      // quadrant-local centre
            const float Sdx = X * M0 - Mx, Sdy = Y * M0 - My;
            const float Sdxdx = X * X * M0 - 2.0f * X * Mx + Mxx;
            const float Sdxdy = X * Y * M0 - X * My - Y * Mx + Mxy;
            const float Sdydy = Y * Y * M0 - 2.0f * Y * My + Myy;
            s_q[e][4] = -co.w * ddelx_dx * (co.x * Sdx + co.y * Sdy);
            s_q[e][5] = -co.w * ddely_dy * (co.z * Sdy + co.y * Sdx);
            s_q[e][6] = -0.5f * co.w * Sdxdx;
            s_q[e][7] = -0.5f * co.w * Sdxdy;
            s_q[e][8] = -0.5f * co.w * Sdydy;
            s_q[e][9] = M0;
        }
        wave_lds_sync();
        acnt = cnt;
        cnt = next_cnt;
        BWD_STAMP(8);
    }
    issue_atomics();   // the last group's
#ifdef LSR_BWD_STAMPS
    if (lane < 8) {   // segments 0..7 (a vector atomic per lane)
        unsigned long long v = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) v = lane == k ? st_sum[k] : v;
        atomicAdd(&g_bwd_stamps[lane], v);
    }
    if (lane == 8) atomicAdd(&g_bwd_stamps[8], 1ull);   // waves that ran groups
    {   // the wave's setup in three parts, and its whole life
        unsigned long long st_end;
        asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(st_end)::"memory");
        if (lane == 9) atomicAdd(&g_bwd_stamps[9], st_loop - st_entry);
        if (lane == 10) atomicAdd(&g_bwd_stamps[10], st_end - st_entry);
        if (lane == 11) atomicAdd(&g_bwd_stamps[11], st_nrep - st_entry);   // pixel loads, replay bound
        if (lane == 12) atomicAdd(&g_bwd_stamps[12], st_scan - st_nrep);    // G rows, B operands
        if (lane == 13) atomicAdd(&g_bwd_stamps[13], st_loop - st_scan);    // first scan + prefetch
    }
#endif
}

// Longest-first launch order.  Blocks are dispatched in launch order, so with ~10 quadrant waves
// per wave slot the tiles with the longest replays, launched last, would set the tail.  One block
// buckets the tiles by their replay bound (tile_max_contrib, written by the forward) in
// descending order: a counting sort over 1024 buckets of 2 replay entries.  The order inside a
// bucket is not fixed, which only permutes float atomic summation (this path is non-deterministic).
// One block per view of a batch.
constexpr int ORDER_BUCKETS = 1024;
struct TileOrderBatch {
    const uint32_t* tile_max[LSR_MAX_VIEWS];
    uint32_t* order[LSR_MAX_VIEWS];
};
__global__ void __launch_bounds__(1024) k_tile_order(int ntiles, TileOrderBatch tb) {
    __shared__ uint32_t s_cnt[ORDER_BUCKETS];
    __shared__ uint32_t s_wave[16];
    const uint32_t* __restrict__ tile_max = tb.tile_max[blockIdx.x];
    uint32_t* __restrict__ order = tb.order[blockIdx.x];
    if (!order || !tile_max) return;   // block-uniform: this view composites in tile order
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    s_cnt[tid] = 0;
    __syncthreads();
    auto bucket = [&](int t) {
        const uint32_t cost = tile_max[t] >> 1;
        return ORDER_BUCKETS - 1 - (int)min(cost, (uint32_t)ORDER_BUCKETS - 1);
    };
    for (int t = tid; t < ntiles; t += 1024) atomicAdd(&s_cnt[bucket(t)], 1u);
    __syncthreads();
    const uint32_t v = s_cnt[tid];
    uint32_t inc = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t y = __shfl_up(inc, o);
        if (lane >= o) inc += y;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    uint32_t off = 0;
    for (int w = 0; w < wave; ++w) off += s_wave[w];
    s_cnt[tid] = off + inc - v;   // exclusive start of bucket tid
    __syncthreads();
    for (int t = tid; t < ntiles; t += 1024) order[atomicAdd(&s_cnt[bucket(t)], 1u)] = (uint32_t)t;
}

// n <= LSR_MAX_VIEWS views sharing the image size, C, include_feature and the language operands'
// form; the tile orders of all of them in one launch, then one compositor launch
void launch_render_bwd_wave_views(const RenderBwdArgs* a, int n, hipStream_t st) {
    const int ntiles = a[0].grid_x * a[0].grid_y;
    RenderBwdBatch ab{};
    TileOrderBatch tb{};
    bool order = false;
    for (int v = 0; v < n; ++v) {
        ab.v[v] = a[v];
        tb.tile_max[v] = a[v].tile_max_contrib;
        tb.order[v] = a[v].tile_order;
        order = order || a[v].tile_order;
    }
    if (order) {
        for (int v = 0; v < n; ++v)
            if (!a[v].tile_order) { ab.v[v].tile_order = nullptr; tb.order[v] = nullptr; }
        hipLaunchKernelGGL(k_tile_order, dim3(n), dim3(1024), 0, st, ntiles, tb);
    }
    const bool c32 = a[0].include_feature && a[0].C == 32;
    const bool nol = !a[0].include_feature || a[0].C == 0;
    const dim3 grid(((ntiles + 7) / 8) * 32, n);
    if (c32 && a[0].lang_split) hipLaunchKernelGGL((k_render_bwd_wave<true, true, false>), grid, dim3(64), 0, st, ab);
    else if (c32) hipLaunchKernelGGL((k_render_bwd_wave<true, false, false>), grid, dim3(64), 0, st, ab);
    else if (nol) hipLaunchKernelGGL((k_render_bwd_wave<false, false, true>), grid, dim3(64), 0, st, ab);
    else hipLaunchKernelGGL((k_render_bwd_wave<false, false, false>), grid, dim3(64), 0, st, ab);
}

}  // namespace lsr

#ifdef LSR_BWD_STAMPS
// diagnostic export (not part of include/lsr.h): read and reset the stamp sums
extern "C" int lsr_debug_bwd_stamps(unsigned long long* out14) {   // 8 segments, waves, setup, life, setup parts
    if (hipMemcpyFromSymbol(out14, HIP_SYMBOL(lsr::g_bwd_stamps), 14 * sizeof(unsigned long long)) != hipSuccess) return 2;
    unsigned long long z[16] = {};
    return hipMemcpyToSymbol(HIP_SYMBOL(lsr::g_bwd_stamps), z, sizeof(z)) == hipSuccess ? 0 : 2;
}
#endif
