// tilebin.hip -- tile-bucket binning: the per-tile lists built without a depth sort of the Gaussians.
//
// Upstream sorts 64-bit (tile << 32 | depth bits) keys of all instances; the
// sort path of this library (sort.hip, binning.hip) sorts the Gaussians by depth, emits instances in
// that order and stable-sorts them by tile (13 bits).  Here the instances go straight to their tile's
// bucket, and each bucket is sorted on its own in LDS:
//   1. k_tb_count    blocks of TB_GPB consecutive Gaussians (index order) walk their instance slots
//                    (the exclusive scan of the per-Gaussian counts, as k_emit walks depth ranks) and
//                    count the listed instances per tile in an LDS histogram, one row of the
//                    [blocks][tiles] table per block (no atomics);
//   2. k_tb_colscan  per tile, the exclusive scan of its column over the blocks, and its total;
//   3. k_tb_tilescan per view, the exclusive scan of the tile totals: the tile ranges;
//   4. k_tb_scatter  the same walk again: each listed instance takes the next slot of its tile inside
//                    the block's reserved run (an LDS counter) and writes its 64-bit key
//                    (depth bits << 32 | id << 4 | quadrant bits);
//   5. k_tb_sort     one block per tile sorts its keys in LDS (8-key register runs, then merge-path
//                    passes; buckets longer than TB_CAP go through LDS-sorted chunks and merge passes
//                    in global memory) and writes the point list words (id | quadrant bits << 28).
// Sorting a bucket by (depth bits, id) reproduces upstream's order exactly (its radix sort is
// stable over instances emitted in id order), so the lists equal the sort path's: the same entries
// (instances that reach no quadrant are not listed, emit_quad_mask), in the same order.
#include <mutex>

#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

namespace {
constexpr int TB_WAVES = 16;                  // waves per count / scatter block
constexpr int TB_THREADS = 64 * TB_WAVES;
constexpr int TB_CHUNKS = 16;                 // 64-Gaussian chunks per wave
constexpr int TB_GPB = TB_THREADS * TB_CHUNKS;   // Gaussians per count / scatter block (16384: ~8
                                                 // listed instances per tile and block on the headline
                                                 // scene, so the scatter's runs fill whole 64-byte lines)
constexpr int TB_CAP = 2048;                  // bucket length sorted in LDS at once (2 x 16 KB)
constexpr int TB_SEG = 16;                    // column-scan segments (and tiles) per block

__device__ __forceinline__ uint64_t tb_key(uint32_t depth_bits, uint32_t id, uint32_t quads) {
    return ((uint64_t)depth_bits << 32) | ((uint64_t)id << 4) | (uint64_t)quads;
}
__device__ __forceinline__ uint32_t tb_word(uint64_t k) {
    return (uint32_t)((k >> 4) & PL_ID_MASK) | ((uint32_t)(k & 0xFu) << PL_QUAD_SHIFT);
}

// The instance walk shared by the count and the scatter: wave w of block b takes chunks of 64
// consecutive Gaussians; per chunk it walks the chunk's instance slots (consecutive lanes, a binary
// search over the 64 start offsets) and calls f(tile, id, quads) for every instance that reaches a
// quadrant of its tile -- the slot order and the quadrant bits of k_emit.
template <typename F>
__device__ __forceinline__ void tb_walk(const TbBatch& tb, const TbView& tv, F&& f) {
    __shared__ uint32_t s_off[TB_WAVES][64];
    __shared__ uint2 s_rc[TB_WAVES][64];
    __shared__ EmitSplat s_sp[TB_WAVES][64];
    const int P = tb.P, gx = tb.grid_x;
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    for (int ch = 0; ch < TB_CHUNKS; ++ch) {
        const int base = blockIdx.x * TB_GPB + (ch * TB_WAVES + w) * 64;
        if (base >= P) break;                               // wave-uniform
        const int g = base + lane;
        const bool ok = g < P;
        const uint32_t cnt = ok ? tv.counts[g] : 0u;
        const uint32_t off = ok ? tv.offsets[g] : 0u;
        const int last = min(P - 1 - base, 63);
        const uint32_t end = __shfl(off + cnt, last);
        const uint32_t start = __shfl(off, 0);
        const uint2 rc = ok ? tv.rect[g] : make_uint2(0u, 0u);
        s_off[w][lane] = ok ? off : end;                    // past-the-end lanes never own a slot
        s_rc[w][lane] = rc;
        uint32_t ox0, oy0, ox1, oy1;
        rect_unpack(rc, ox0, oy0, ox1, oy1);
        if (ok && cnt > 0 && (ox1 - ox0 > 2 || oy1 - oy0 > 2)) s_sp[w][lane] = emit_splat(tv.xy[g], tv.conic_o[g]);
        __builtin_amdgcn_wave_barrier();
        for (uint32_t j = start + lane; j < end; j += 64) {
            int k = 0;                                      // last chunk lane with s_off <= j
#pragma unroll
            for (int step = 32; step >= 1; step >>= 1)
                if (s_off[w][k + step] <= j) k += step;
            const uint2 r = s_rc[w][k];
            uint32_t x0, y0, x1, y1;
            rect_unpack(r, x0, y0, x1, y1);
            const uint32_t loc = j - s_off[w][k];
            uint32_t dx, dy, quads;
            if (rect_small(x0, y0, x1, y1)) {
                const uint32_t map = rect_quad_map(r);
                uint32_t m = rect_tile_mask(map);
                for (uint32_t i = 0; i < loc; ++i) m &= m - 1u;
                const uint32_t pos = (uint32_t)__builtin_ctz(m);
                dx = pos & 1u;
                dy = pos >> 1;
                const uint32_t sh = 8 * dy + 2 * dx;
                quads = ((map >> sh) & 3u) | (((map >> (sh + 4)) & 3u) << 2);
            } else {
                const uint32_t wd = x1 - x0;
                dy = loc / wd;
                dx = loc - dy * wd;
                quads = emit_quad_mask(s_sp[w][k], (int)(x0 + dx) * LSR_TILE_X, (int)(y0 + dy) * LSR_TILE_Y, tb.W, tb.H);
            }
            if (quads) f((y0 + dy) * (uint32_t)gx + (x0 + dx), (uint32_t)(base + k), quads);
        }
        __builtin_amdgcn_wave_barrier();                    // the staging arrays are rewritten next chunk
    }
}
}  // namespace

__global__ void __launch_bounds__(TB_THREADS) k_tb_count(const TbBatch tb) {
    extern __shared__ uint32_t s_hist[];   // [ntiles]
    const TbView& tv = tb.v[blockIdx.y];
    for (int t = threadIdx.x; t < tb.ntiles; t += TB_THREADS) s_hist[t] = 0u;
    __syncthreads();
    tb_walk(tb, tv, [&](uint32_t tile, uint32_t, uint32_t) { atomicAdd(&s_hist[tile], 1u); });
    __syncthreads();
    uint32_t* row = tv.table + (size_t)blockIdx.x * tb.ntiles;
    for (int t = threadIdx.x; t < tb.ntiles; t += TB_THREADS) row[t] = s_hist[t];
}

// per tile (TB_SEG tiles x TB_SEG segments of block rows per 256-thread block): the column's
// exclusive scan in place, and its total
__global__ void __launch_bounds__(256) k_tb_colscan(const TbBatch tb, int nblocks) {
    __shared__ uint32_t s_part[TB_SEG][TB_SEG + 1];
    const TbView& tv = tb.v[blockIdx.y];
    const int tl = threadIdx.x % TB_SEG, seg = threadIdx.x / TB_SEG;
    const int t = blockIdx.x * TB_SEG + tl;
    const int per = (nblocks + TB_SEG - 1) / TB_SEG, b0 = seg * per, b1 = min(nblocks, b0 + per);
    uint32_t sum = 0;
    if (t < tb.ntiles)
        for (int b = b0; b < b1; ++b) sum += tv.table[(size_t)b * tb.ntiles + t];
    s_part[seg][tl] = sum;
    __syncthreads();
    if (seg == 0) {
        uint32_t run = 0;
        for (int s = 0; s < TB_SEG; ++s) {
            const uint32_t v = s_part[s][tl];
            s_part[s][tl] = run;
            run += v;
        }
        if (t < tb.ntiles) tv.tile_total[t] = run;
    }
    __syncthreads();
    if (t < tb.ntiles) {
        uint32_t run = s_part[seg][tl];
        for (int b = b0; b < b1; ++b) {
            uint32_t* p = tv.table + (size_t)b * tb.ntiles + t;
            const uint32_t v = *p;
            *p = run;
            run += v;
        }
    }
}

// per view: the tile totals' exclusive scan -> tile starts (tile_start) and ranges
__global__ void __launch_bounds__(1024) k_tb_tilescan(const TbBatch tb) {
    __shared__ uint32_t s_wave[16];
    __shared__ uint32_t s_carry;
    const TbView& tv = tb.v[blockIdx.x];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) s_carry = 0u;
    __syncthreads();
    for (int t0 = 0; t0 < tb.ntiles; t0 += 1024) {
        const int t = t0 + tid;
        const uint32_t v = t < tb.ntiles ? tv.tile_total[t] : 0u;
        uint32_t inc = v;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t y = __shfl_up(inc, o);
            if (lane >= o) inc += y;
        }
        if (lane == 63) s_wave[wave] = inc;
        __syncthreads();
        uint32_t off = s_carry;
        for (int w2 = 0; w2 < wave; ++w2) off += s_wave[w2];
        const uint32_t start = off + inc - v;
        if (t < tb.ntiles) {
            tv.tile_start[t] = start;
            tv.ranges[t] = v ? make_uint2(start, start + v) : make_uint2(0u, 0u);   // upstream's empty range
        }
        __syncthreads();
        if (tid == 1023) s_carry = start + v;
        __syncthreads();
    }
}

__global__ void __launch_bounds__(TB_THREADS) k_tb_scatter(const TbBatch tb) {
    extern __shared__ uint32_t s_cur[];   // [ntiles]: the next slot of each tile in this block's run
    const TbView& tv = tb.v[blockIdx.y];
    const uint32_t* row = tv.table + (size_t)blockIdx.x * tb.ntiles;
    for (int t = threadIdx.x; t < tb.ntiles; t += TB_THREADS) s_cur[t] = tv.tile_start[t] + row[t];
    __syncthreads();
    tb_walk(tb, tv, [&](uint32_t tile, uint32_t id, uint32_t quads) {
        const uint32_t pos = atomicAdd(&s_cur[tile], 1u);
        tv.keys[pos] = tb_key(tv.depth[id], id, quads);
    });
}

namespace {
// LDS slot of key i: one unused slot after every 8 keys, so that a thread's run of 8 (the register
// sort, the merge outputs) starts 9 slots after its neighbour's: 2-way bank conflicts, not 16-way.
__device__ __forceinline__ int pad8(int i) { return i + (i >> 3); }
constexpr int TB_CAP_PAD = TB_CAP + TB_CAP / 8;

// Sorts keys 0..n8-1 (slots pad8(i) of s; n8 a multiple of 8, 8 <= n8 <= TB_CAP) ascending with the
// block's 256 threads; returns the buffer holding the result (s or t, both [TB_CAP_PAD] in LDS).
// Each thread sorts a run of 8 keys in registers, then merge passes double the runs (the last run of
// a pass may be short): thread i makes outputs [8 i, 8 i + 8) of its pair of runs, finding where they
// start by a binary search along the merge path and merging 8 steps from there.  Keys are unique
// apart from the ~0 padding (equal, so either order is right).
__device__ __forceinline__ uint64_t* lds_merge_sort(uint64_t* s, uint64_t* t, int n8) {
    const int nt = n8 / 8, tid = threadIdx.x;
    if (tid < nt) {
        uint64_t x[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) x[k] = s[9 * tid + k];
        // odd-even transposition network on 8 registers (28 compare-exchanges, fully unrolled)
#pragma unroll
        for (int r = 0; r < 8; ++r)
#pragma unroll
            for (int k = r & 1; k + 1 < 8; k += 2) {
                const uint64_t lo = x[k] < x[k + 1] ? x[k] : x[k + 1];
                const uint64_t hi = x[k] < x[k + 1] ? x[k + 1] : x[k];
                x[k] = lo;
                x[k + 1] = hi;
            }
#pragma unroll
        for (int k = 0; k < 8; ++k) s[9 * tid + k] = x[k];
    }
    __syncthreads();
    uint64_t* src = s;
    uint64_t* dst = t;
    for (int w = 8; w < n8; w <<= 1) {
        if (tid < nt) {
            const int o = 8 * tid, lo = o & ~(2 * w - 1), d = o - lo;
            const int na = min(w, n8 - lo), nb = max(0, min(w, n8 - lo - w)), bo = lo + na;
            int a0 = max(0, d - nb), a1 = min(d, na);   // keys taken from A = [lo, lo + na) among the first d
            while (a0 < a1) {
                const int m = (a0 + a1) >> 1;
                if (src[pad8(lo + m)] < src[pad8(bo + d - m - 1)]) a0 = m + 1;
                else a1 = m;
            }
            int i = a0, j = d - a0;
            uint64_t av = i < na ? src[pad8(lo + i)] : ~0ull, bv = j < nb ? src[pad8(bo + j)] : ~0ull;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
                const bool ta = j >= nb || (i < na && av < bv);
                dst[9 * tid + k] = ta ? av : bv;
                if (ta) {
                    ++i;
                    av = i < na ? src[pad8(lo + i)] : ~0ull;
                } else {
                    ++j;
                    bv = j < nb ? src[pad8(bo + j)] : ~0ull;
                }
            }
        }
        __syncthreads();
        uint64_t* x = src; src = dst; dst = x;
    }
    return src;
}
// merge runs a[0, na) and b[0, nb) into out (global memory, unique keys): each output index takes its
// element by a binary search along the merge path (the rare buckets longer than TB_CAP)
__device__ __forceinline__ void merge_runs(const uint64_t* a, int na, const uint64_t* b, int nb, uint64_t* out) {
    for (int o = threadIdx.x; o < na + nb; o += 256) {
        int lo = max(0, o - nb), hi = min(o, na);   // i = elements taken from a among the first o
        while (lo < hi) {
            const int i = (lo + hi) >> 1;
            if (a[i] < b[o - i - 1]) lo = i + 1;
            else hi = i;
        }
        const int i = lo, jb = o - i;
        const bool take_a = jb >= nb || (i < na && a[i] < b[jb]);
        out[o] = take_a ? a[i] : b[jb];
    }
}
__device__ __forceinline__ int round8(int n) { return (n + 7) & ~7; }
}  // namespace

__global__ void __launch_bounds__(256) k_tb_sort(const TbBatch tb) {
    __shared__ uint64_t s_a[TB_CAP_PAD];
    __shared__ uint64_t s_b[TB_CAP_PAD];
    const TbView& tv = tb.v[blockIdx.y];
    const int tile = blockIdx.x;
    const uint2 r = tv.ranges[tile];
    const int n = (int)(r.y - r.x);
    uint64_t* keys = tv.keys + r.x;
    uint32_t* words = tv.words + r.x;
    if (n > 0 && n <= TB_CAP) {
        const int n8 = round8(n);
        for (int i = threadIdx.x; i < n8; i += 256) s_a[pad8(i)] = i < n ? keys[i] : ~0ull;
        __syncthreads();
        const uint64_t* res = lds_merge_sort(s_a, s_b, n8);
        for (int i = threadIdx.x; i < n; i += 256) words[i] = tb_word(res[pad8(i)]);
    } else if (n > TB_CAP) {
        // long bucket: LDS-sorted chunks of TB_CAP, then merge passes between keys and tmp
        for (int c0 = 0; c0 < n; c0 += TB_CAP) {
            const int m = min(TB_CAP, n - c0), m8 = round8(m);
            for (int i = threadIdx.x; i < m8; i += 256) s_a[pad8(i)] = i < m ? keys[c0 + i] : ~0ull;
            __syncthreads();
            const uint64_t* res = lds_merge_sort(s_a, s_b, m8);
            for (int i = threadIdx.x; i < m; i += 256) keys[c0 + i] = res[pad8(i)];
            __syncthreads();
        }
        __threadfence_block();
        uint64_t* src = keys;
        uint64_t* dst = tv.tmp + r.x;
        for (int wdt = TB_CAP; wdt < n; wdt <<= 1) {
            for (int lo = 0; lo < n; lo += 2 * wdt) {
                const int na = min(wdt, n - lo), nb = max(0, min(wdt, n - lo - wdt));
                merge_runs(src + lo, na, src + lo + na, nb, dst + lo);
            }
            __threadfence_block();
            __syncthreads();
            uint64_t* t = src; src = dst; dst = t;
        }
        for (int i = threadIdx.x; i < n; i += 256) words[i] = tb_word(src[i]);
    }
    if (threadIdx.x == 0) tv.tile_max[tile] = 0u;   // the forward's atomicMax bound starts at 0
}

int tb_blocks(int P) { return (P + TB_GPB - 1) / TB_GPB; }

hipError_t launch_tile_bucket_binning(const TbBatch& tb, int nv, hipStream_t st) {
    if (tb.P == 0 || nv <= 0) return hipSuccess;
    const int nb = tb_blocks(tb.P);
    const size_t hist = (size_t)tb.ntiles * sizeof(uint32_t);
    // dynamic LDS beyond 64 KiB beside the walk's static staging arrays: a per-function attribute that
    // HIP keeps per device, so it is set once per device (thread-safe) and its result kept
    constexpr int kMaxDev = 64;
    static std::once_flag once[kMaxDev];
    static hipError_t attr_err[kMaxDev];
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    if (dev < 0 || dev >= kMaxDev) return hipErrorInvalidDevice;
    std::call_once(once[dev], [dev] {
        hipError_t r = hipFuncSetAttribute(reinterpret_cast<const void*>(k_tb_count),
                                           hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        if (r == hipSuccess)
            r = hipFuncSetAttribute(reinterpret_cast<const void*>(k_tb_scatter),
                                    hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        attr_err[dev] = r;
    });
    if (attr_err[dev] != hipSuccess) return attr_err[dev];
    hipLaunchKernelGGL(k_tb_count, dim3(nb, nv), dim3(TB_THREADS), hist, st, tb);
    hipLaunchKernelGGL(k_tb_colscan, dim3((tb.ntiles + TB_SEG - 1) / TB_SEG, nv), dim3(256), 0, st, tb, nb);
    hipLaunchKernelGGL(k_tb_tilescan, dim3(nv), dim3(1024), 0, st, tb);
    hipLaunchKernelGGL(k_tb_scatter, dim3(nb, nv), dim3(TB_THREADS), hist, st, tb);
    hipLaunchKernelGGL(k_tb_sort, dim3(tb.ntiles, nv), dim3(256), 0, st, tb);
    return hipSuccess;
}

}  // namespace lsr
