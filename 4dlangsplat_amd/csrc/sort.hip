// sort.hip -- device-wide exclusive scan and stable LSD radix sort of (u32 key, u32 value) pairs,
// written for wave64: per-wave digit matching by ballots (one 64-bit ballot per key bit), per-wave
// digit counts in LDS, and per-digit running offsets, so every pass is stable.
//
// Used twice per frame by the binning (binning.hip):
//   1. depth order of all P Gaussians: key = view-space depth bits (culled = 0xFFFFFFFF), 8 + 9 + 9
//      bits above the kept keys' 256-aligned minimum when they span < 2^26 of it, else 4 x 8 bits;
//   2. tile order of the K (Gaussian, tile) instances emitted in depth order: key = tile id,
//      ceil(log2(tiles)) bits (2 passes at 5,440 tiles).
// Stable tile sort of depth-ordered instances == the upstream sort of (tile << 32 | depth) keys.
#include "lsr_common.h"
#include "lsr_internal.h"
#include <cstdlib>

namespace lsr {

constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = 256 * SCAN_ITEMS;

static inline size_t align_up(size_t x, size_t a) { return (x + a - 1) / a * a; }

// ---- scan -------------------------------------------------------------------------------------
__device__ __forceinline__ void block_exclusive_scan8(uint32_t (&v)[SCAN_ITEMS], uint32_t* s_wave,
                                                      uint32_t& block_total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t local = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) { const uint32_t x = v[i]; v[i] = local; local += x; }
    uint32_t inc = local;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o);
        if (lane >= o) inc += t;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    uint32_t wave_off = 0, total = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        const uint32_t s = s_wave[w];
        wave_off += (w < wave) ? s : 0u;
        total += s;
    }
    const uint32_t off = wave_off + inc - local;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) v[i] += off;
    block_total = total;
}

__global__ void __launch_bounds__(256) k_scan_reduce(const uint32_t* __restrict__ in, size_t n,
                                                     uint32_t* __restrict__ partials) {
    __shared__ uint32_t s_wave[4];
    const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) s += (base + i < n) ? in[base + i] : 0u;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) s_wave[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
}

__global__ void __launch_bounds__(256) k_scan_down(const uint32_t* __restrict__ in, uint32_t* __restrict__ out,
                                                   size_t n, const uint32_t* __restrict__ bases,
                                                   uint32_t* __restrict__ total) {
    __shared__ uint32_t s_wave[4];
    const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) v[i] = (base + i < n) ? in[base + i] : 0u;
    uint32_t block_total;
    block_exclusive_scan8(v, s_wave, block_total);
    const uint32_t b0 = bases ? bases[blockIdx.x] : 0u;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i)
        if (base + i < n) out[base + i] = v[i] + b0;
    if (total && threadIdx.x == 0 && gridDim.x == 1) *total = block_total;
}

// SCAN_ITEMS consecutive values from `base` (zeros past n): two 16-byte loads when aligned
static_assert(SCAN_ITEMS == 8, "load_items reads two uint4");
__device__ __forceinline__ void load_items(const uint32_t* __restrict__ in, size_t base, size_t n,
                                           uint32_t (&v)[SCAN_ITEMS]) {
    if (base + SCAN_ITEMS <= n && (reinterpret_cast<uintptr_t>(in + base) & 15u) == 0) {
        const uint4 a = reinterpret_cast<const uint4*>(in + base)[0], c = reinterpret_cast<const uint4*>(in + base)[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = c.x; v[5] = c.y; v[6] = c.z; v[7] = c.w;
    } else {
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i) v[i] = (base + i < n) ? in[base + i] : 0u;
    }
}

// Two-kernel scan of up to 4096 tiles, for a batch of segments (blockIdx.y): the first kernel
// writes every tile's sum; in the second, block b sums the partials of blocks [0, b) itself (no
// separate scan of the partials: one dependent launch less), then scans its tile.  Block 0 also
// writes the grand total.  Blocks past a segment's own tile count return at once.
__global__ void __launch_bounds__(256) k_scan_reduce_seg(const ScanBatch bt) {
    __shared__ uint32_t s_wave[4];
    const ScanSeg& sg = bt.s[blockIdx.y];
    const size_t n = sg.n;
    if ((size_t)blockIdx.x * SCAN_TILE >= n) return;                  // block-uniform
    const size_t base = (size_t)blockIdx.x * SCAN_TILE + (size_t)threadIdx.x * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    load_items(sg.in, base, n, v);
    uint32_t s = 0;
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) s += v[i];
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) s += __shfl_xor(s, o);
    if ((threadIdx.x & 63) == 0) s_wave[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) sg.partials[blockIdx.x] = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
}

__global__ void __launch_bounds__(256) k_scan_down_sum(const ScanBatch bt) {
    __shared__ uint32_t s_wave[4];
    __shared__ uint32_t s_base[2];
    const ScanSeg& sg = bt.s[blockIdx.y];
    const size_t n = sg.n;
    const int nb = (int)((n + SCAN_TILE - 1) / SCAN_TILE);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.x;
    if (b >= nb) return;                                               // block-uniform
    // this tile's items are loaded first: their latency overlaps the partials' sum
    const size_t base = (size_t)b * SCAN_TILE + (size_t)tid * SCAN_ITEMS;
    uint32_t v[SCAN_ITEMS];
    load_items(sg.in, base, n, v);
    uint32_t pre = 0, all = 0;
    const int upto = b == 0 ? nb : b;   // block 0 also sums them all for the grand total
    for (int i = tid; i < upto; i += 256) {
        const uint32_t x = sg.partials[i];
        pre += i < b ? x : 0u;
        all += x;
    }
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        pre += __shfl_xor(pre, o);
        all += __shfl_xor(all, o);
    }
    if (lane == 0) s_wave[wave] = pre;
    __syncthreads();
    if (tid == 0) s_base[0] = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    __syncthreads();
    if (lane == 0) s_wave[wave] = all;
    __syncthreads();
    if (tid == 0) s_base[1] = s_wave[0] + s_wave[1] + s_wave[2] + s_wave[3];
    __syncthreads();
    const uint32_t b0 = s_base[0];
    if (b == 0 && tid == 0) {
        if (sg.total) *sg.total = s_base[1];
        if (sg.host_total) sg.host_total[0] = s_base[1];   // host-mapped: visible once the kernel completed
    }
    uint32_t block_total;
    block_exclusive_scan8(v, s_wave, block_total);
#pragma unroll
    for (int i = 0; i < SCAN_ITEMS; ++i) v[i] += b0;
    if (base + SCAN_ITEMS <= n && (reinterpret_cast<uintptr_t>(sg.out + base) & 15u) == 0) {
        uint4* o = reinterpret_cast<uint4*>(sg.out + base);
        o[0] = make_uint4(v[0], v[1], v[2], v[3]);
        o[1] = make_uint4(v[4], v[5], v[6], v[7]);
    } else {
#pragma unroll
        for (int i = 0; i < SCAN_ITEMS; ++i)
            if (base + i < n) sg.out[base + i] = v[i];
    }
}

size_t scan_temp_bytes(size_t n) {
    if (n <= (size_t)SCAN_TILE) return 0;
    const size_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    return align_up(nb * sizeof(uint32_t), 256) * 2 + scan_temp_bytes(nb);
}

void exclusive_scan_u32(const uint32_t* in, uint32_t* out, size_t n, uint32_t* total, void* temp, hipStream_t st) {
    if (n == 0) {
        if (total) (void)hipMemsetAsync(total, 0, sizeof(uint32_t), st);
        return;
    }
    if (n <= (size_t)SCAN_TILE) {
        hipLaunchKernelGGL(k_scan_down, dim3(1), dim3(256), 0, st, in, out, n, (const uint32_t*)nullptr, total);
        return;
    }
    const size_t nb = (n + SCAN_TILE - 1) / SCAN_TILE;
    uint32_t* partials = reinterpret_cast<uint32_t*>(temp);
    if (nb <= (size_t)SCAN_SEG_TILES) {   // up to 8M values: the scan of the partials is folded into the second pass
        const ScanSeg sg{in, out, total, partials, n};
        exclusive_scan_batch(&sg, 1, st);
        return;
    }
    uint32_t* scanned = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(temp) + align_up(nb * 4, 256));
    void* deeper = reinterpret_cast<char*>(temp) + 2 * align_up(nb * 4, 256);
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(256), 0, st, in, n, partials);
    exclusive_scan_u32(partials, scanned, nb, total, deeper, st);
    hipLaunchKernelGGL(k_scan_down, dim3((unsigned)nb), dim3(256), 0, st, in, out, n, (const uint32_t*)scanned,
                       (uint32_t*)nullptr);
}

uint32_t exclusive_scan_batch(const ScanSeg* segs, int nseg, hipStream_t st) {
    ScanBatch bt{};
    int ns = 0;
    size_t nbmax = 0;
    uint32_t wrote = 0;
    for (int i = 0; i < nseg; ++i) {
        const ScanSeg& g = segs[i];
        const size_t nb = (g.n + SCAN_TILE - 1) / SCAN_TILE;
        if (g.n > (size_t)SCAN_TILE && nb <= (size_t)SCAN_SEG_TILES) {
            bt.s[ns++] = g;
            nbmax = std::max(nbmax, nb);
            if (g.host_total) wrote |= 1u << i;
        } else {
            exclusive_scan_u32(g.in, g.out, g.n, g.total, g.partials, st);   // one tile, or beyond 8M values
        }
    }
    if (ns == 0) return wrote;
    hipLaunchKernelGGL(k_scan_reduce_seg, dim3((unsigned)nbmax, ns), dim3(256), 0, st, bt);
    hipLaunchKernelGGL(k_scan_down_sum, dim3((unsigned)nbmax, ns), dim3(256), 0, st, bt);
    return wrote;
}

// ---- radix sort ---------------------------------------------------------------------------------
// Reduce-then-scan LSD passes, 8 keys per thread (12 above 4M keys): per pass a count kernel writes
// every block's digit counts, a scan kernel turns them into each block's offset inside its digit
// and the digit totals, and the scatter kernel ranks the block's keys again (ballot digit matching
// per wave, stable), places them digit-sorted in LDS and writes runs (coalesced stores).
// There is no inter-block chain: a decoupled look-back (one pass kernel, blocks waiting on their
// predecessors' published counts) crossed the 8 XCDs' non-coherent L2s at every hop and bounded a
// pass by the chain length; it was removed in round 3.
//
// Digits are up to 9 bits (RDX = 512).  Host-planned sorts (the tile sort) give every launch its
// shift / width; the depth sort (SortSeg::vals_c set) plans on the device: its first pass takes
// the low 8 bits and records each block's smallest and largest kept key, its scan fixes
// kbase = min & ~0xFF, and when the kept keys span less than 2^26 above kbase (depths within a
// factor of 256) the sort finishes in two 9-bit passes over key - kbase instead of three 8-bit
// ones.  Both plans leave the result in the (a) buffers: the three-pass plan's middle pass writes
// its values to vals_c (free scratch) so that its last pass can gather into vals_a.
constexpr int OS_ITEMS = 8;                   // keys per thread per pass (4 / 8 / 16 swept)
constexpr int OS_TILE = 256 * OS_ITEMS;       // keys per block
constexpr int RDX = 512;                      // digits of the widest pass (count rows' stride)

// Peers of this lane's digit inside the wave (lanes with the same digit among the valid lanes).
__device__ __forceinline__ uint64_t match_digit(uint32_t d, bool valid, int nbits) {
    uint64_t peers = __ballot(valid);
    for (int bit = 0; bit < nbits; ++bit) {
        const bool b = (d >> bit) & 1u;
        const uint64_t m = __ballot(b);
        peers &= b ? m : ~m;
    }
    return peers;
}

// exclusive scan of one value per thread over a 256-thread block
__device__ __forceinline__ uint32_t block_excl_scan256(uint32_t x, uint32_t* s_wave) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    uint32_t inc = x;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t t = __shfl_up(inc, o);
        if (lane >= o) inc += t;
    }
    if (lane == 63) s_wave[wave] = inc;
    __syncthreads();
    uint32_t off = 0;
#pragma unroll
    for (int w = 0; w < 4; ++w) off += (w < wave) ? s_wave[w] : 0u;
    __syncthreads();
    return off + inc - x;
}

// ---- reduce-then-scan passes ------------------------------------------------------------------
//   drop (first pass of a sort with a kept-count word): keys equal to 0xFFFFFFFF are not counted
//   and not placed; the scatter's block 0 writes the number of kept keys to *kept_out.
//   n_dev (later passes): the number of keys is *n_dev (<= n); blocks past it write zero counts
//   and place nothing.
__device__ __forceinline__ size_t rts_n(size_t n, const uint32_t* n_dev) {
    return n_dev ? min(n, (size_t)*n_dev) : n;
}
// A segment's workspace: digit totals [pass][RDX], the depth plan (kbase, three-pass flag), then
// the per-pass count rows [pass][block][RDX] (the first pass's rows also carry the block's smallest
// and largest kept key in words 256 / 257 when the plan is made on the device).
constexpr size_t RTS_PLAN_OFF = 4 * RDX * 4;
constexpr size_t RTS_ROWS_OFF = RTS_PLAN_OFF + 256;
__device__ __forceinline__ size_t rts_blocks(size_t n, int it) { return (n + 256 * (size_t)it - 1) / (256 * (size_t)it); }
__device__ __forceinline__ uint32_t* rts_rows(const SortSeg& g, int pass, size_t nbi) {
    return reinterpret_cast<uint32_t*>(static_cast<char*>(g.temp) + RTS_ROWS_OFF) + (size_t)pass * nbi * RDX;
}
__device__ __forceinline__ uint32_t* rts_totals(const SortSeg& g, int pass) {
    return static_cast<uint32_t*>(g.temp) + pass * RDX;
}
__device__ __forceinline__ uint32_t* rts_plan(const SortSeg& g) {
    return reinterpret_cast<uint32_t*>(static_cast<char*>(g.temp) + RTS_PLAN_OFF);
}

// One pass of one segment: digit = ((key - kbase) >> shift) & (2^nbits - 1); buffers by id
// (0: a, 1: b, 2: keys a with values in vals_c).
struct PassDesc {
    int active, shift, nbits, last, src, dst;
    uint32_t kbase;
};
__device__ __forceinline__ PassDesc pass_desc(const SortSeg& sg, int pass, int in_b, int shift, int nbits, int last) {
    PassDesc d{1, shift, nbits, last, in_b, in_b ^ 1, 0u};
    if (!sg.vals_c) return d;                                      // host plan
    if (pass == 0) return PassDesc{1, 0, 8, 0, 0, 1, 0u};
    const uint32_t* pl = rts_plan(sg);
    const uint32_t kbase = pl[0], three = pl[1];
    if (three) {
        if (pass == 1) return PassDesc{1, 8, 9, 0, 1, 2, kbase};
        if (pass == 2) return PassDesc{1, 17, 9, 1, 2, 0, kbase};
        return PassDesc{0, 0, 8, 0, 0, 0, kbase};
    }
    return PassDesc{1, 8 * pass, 8, pass == 3, pass & 1, (pass & 1) ^ 1, 0u};
}
__device__ __forceinline__ const uint32_t* keys_of(const SortSeg& g, int id) { return id == 1 ? g.keys_b : g.keys_a; }
__device__ __forceinline__ uint32_t* keys_of_w(const SortSeg& g, int id) { return id == 1 ? g.keys_b : g.keys_a; }
__device__ __forceinline__ const uint32_t* vals_of(const SortSeg& g, int id) {
    return id == 1 ? g.vals_b : id == 2 ? g.vals_c : g.vals_a;
}
__device__ __forceinline__ uint32_t* vals_of_w(const SortSeg& g, int id) {
    return id == 1 ? g.vals_b : id == 2 ? g.vals_c : g.vals_a;
}

// Every kernel of a pass serves all segments of a batch: blockIdx.y is the segment, blocks past
// a segment's own count return at once (the grid is sized for the largest segment).
template <int IT>
__global__ void __launch_bounds__(256) k_rts_count(const SortBatch b, int pass, int in_b, int shift, int nbits) {
    __shared__ uint32_t s_h[4][RDX];
    __shared__ uint32_t s_mm[2][4];
    const SortSeg& sg = b.s[blockIdx.y];
    const size_t nbi = rts_blocks(sg.n, IT);
    if (blockIdx.x >= nbi) return;                                   // block-uniform
    const PassDesc pd = pass_desc(sg, pass, in_b, shift, nbits, 0);
    if (!pd.active) return;                                          // segment-uniform
    const uint32_t* __restrict__ keys = keys_of(sg, pd.src);
    const int drop = sg.kept && pass == 0;                         // first pass drops, later passes read
    const size_t n = rts_n(sg.n, sg.kept && pass > 0 ? sg.kept : nullptr);
    uint32_t* __restrict__ counts = rts_rows(sg, pass, nbi);
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        s_h[w][tid] = 0;
        s_h[w][tid + 256] = 0;
    }
    __syncthreads();
    const uint32_t mask = (1u << pd.nbits) - 1u;
    const uint64_t lt = lanemask_lt();
    const size_t base = (size_t)blockIdx.x * (256 * IT) + (size_t)wave * (64 * IT);
    uint32_t key[IT];
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const size_t idx = base + (size_t)r * 64 + lane;
        key[r] = idx < n ? keys[idx] : 0u;
    }
    uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const bool valid = base + (size_t)r * 64 + lane < n && !(drop && key[r] == 0xFFFFFFFFu);
        if (valid) {
            kmin = min(kmin, key[r]);
            kmax = max(kmax, key[r]);
        }
        const uint32_t d = ((key[r] - pd.kbase) >> pd.shift) & mask;
        const uint64_t peers = match_digit(d, valid, pd.nbits);
        if (valid && (peers & lt) == 0) s_h[wave][d] += (uint32_t)__popcll(peers);   // one leader per digit
        __builtin_amdgcn_wave_barrier();
    }
    const bool plan = sg.vals_c && pass == 0;                      // segment-uniform
    if (plan) {
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
            kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
        }
        if (lane == 0) { s_mm[0][wave] = kmin; s_mm[1][wave] = kmax; }
    }
    __syncthreads();
    for (int d = tid; d < (1 << pd.nbits); d += 256)
        counts[(size_t)blockIdx.x * RDX + d] = s_h[0][d] + s_h[1][d] + s_h[2][d] + s_h[3][d];
    if (plan && tid < 2) {   // words 256 / 257 of the 8-bit pass's row: the block's kept-key range
        const uint32_t v = tid == 0 ? min(min(s_mm[0][0], s_mm[0][1]), min(s_mm[0][2], s_mm[0][3]))
                                    : max(max(s_mm[1][0], s_mm[1][1]), max(s_mm[1][2], s_mm[1][3]));
        counts[(size_t)blockIdx.x * RDX + 256 + tid] = v;
    }
}

// The scan, one block per (DG-digit group, segment): thread t owns SCAN_ROWS consecutive block
// rows of a chunk and reads each row's DG counts as DG / 4 16-byte loads (all in flight at once),
// so the count table is read once in whole pieces instead of one 4-byte word per (row, digit
// block) -- a per-digit scan kernel touched every line of the table from 256 blocks (33 us per
// depth pass, 58 us per tile pass on 8 views).  Digit groups past 2^nbits only zero their totals.
// For a device-planned segment, block 0 of the first pass also makes the plan from the rows'
// key ranges.
constexpr int SCAN_ROWS = 8;
template <int DG>
__global__ void __launch_bounds__(256) k_rts_scan(const SortBatch b, int pass, int it, int in_b, int nbits_h) {
    constexpr int Q = DG / 4;
    __shared__ uint32_t s_part[4][DG];
    const SortSeg& sg = b.s[blockIdx.y];
    const PassDesc pd = pass_desc(sg, pass, in_b, 0, nbits_h, 0);
    if (!pd.active) return;                                          // segment-uniform
    const int nbits = pd.nbits;
    const int d0 = DG * (int)blockIdx.x, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    uint32_t* __restrict__ totals = rts_totals(sg, pass);
    const int nb = (int)rts_blocks(sg.n, it);
    uint32_t* __restrict__ counts = rts_rows(sg, pass, (size_t)nb);
    if (sg.vals_c && pass == 0 && blockIdx.x == 0) {   // the depth plan: smallest / largest kept key
        uint32_t kmin = 0xFFFFFFFFu, kmax = 0u;
        for (int r = tid; r < nb; r += 256) {
            kmin = min(kmin, counts[(size_t)r * RDX + 256]);
            kmax = max(kmax, counts[(size_t)r * RDX + 257]);
        }
#pragma unroll
        for (int o = 32; o >= 1; o >>= 1) {
            kmin = min(kmin, (uint32_t)__shfl_xor((int)kmin, o));
            kmax = max(kmax, (uint32_t)__shfl_xor((int)kmax, o));
        }
        if (lane == 0) { s_part[0][wave] = kmin; s_part[1][wave] = kmax; }
        __syncthreads();
        if (tid == 0) {
            const uint32_t lo = min(min(s_part[0][0], s_part[0][1]), min(s_part[0][2], s_part[0][3]));
            const uint32_t hi = max(max(s_part[1][0], s_part[1][1]), max(s_part[1][2], s_part[1][3]));
            const uint32_t kbase = lo & ~0xFFu;
            const bool three = lo <= hi && hi - kbase < (1u << 26);
            uint32_t* pl = rts_plan(sg);
            pl[0] = three ? kbase : 0u;
            pl[1] = three ? 1u : 0u;
        }
        __syncthreads();   // s_part reused below
    }
    if (d0 >= (1 << nbits)) {                                        // block-uniform
        if (tid < DG) totals[d0 + tid] = 0u;
        return;
    }
    uint32_t carry[DG];
#pragma unroll
    for (int j = 0; j < DG; ++j) carry[j] = 0u;
    for (int c0 = 0; c0 < nb; c0 += 256 * SCAN_ROWS) {
        const int r0 = c0 + tid * SCAN_ROWS;
        uint4 v[SCAN_ROWS][Q];
#pragma unroll
        for (int r = 0; r < SCAN_ROWS; ++r) {
            const uint4* p = reinterpret_cast<const uint4*>(counts + (size_t)(r0 + r) * RDX + d0);
#pragma unroll
            for (int q = 0; q < Q; ++q) v[r][q] = r0 + r < nb ? p[q] : make_uint4(0u, 0u, 0u, 0u);
        }
        uint32_t sum[DG];
#pragma unroll
        for (int q = 0; q < Q; ++q) {
            sum[4 * q] = 0u; sum[4 * q + 1] = 0u; sum[4 * q + 2] = 0u; sum[4 * q + 3] = 0u;
#pragma unroll
            for (int r = 0; r < SCAN_ROWS; ++r) {
                sum[4 * q] += v[r][q].x; sum[4 * q + 1] += v[r][q].y;
                sum[4 * q + 2] += v[r][q].z; sum[4 * q + 3] += v[r][q].w;
            }
        }
        // exclusive scan of the DG per-thread sums over the block's threads (rows in order)
        uint32_t off[DG], tot[DG];
#pragma unroll
        for (int j = 0; j < DG; ++j) {
            uint32_t inc = sum[j];
#pragma unroll
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t t = __shfl_up(inc, o);
                if (lane >= o) inc += t;
            }
            off[j] = inc - sum[j];
            if (lane == 63) s_part[wave][j] = inc;
        }
        __syncthreads();
#pragma unroll
        for (int j = 0; j < DG; ++j) {
            uint32_t before = 0u, all = 0u;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t x = s_part[w][j];
                before += w < wave ? x : 0u;
                all += x;
            }
            off[j] += before + carry[j];
            tot[j] = all;
        }
#pragma unroll
        for (int r = 0; r < SCAN_ROWS; ++r) {
            if (r0 + r >= nb) break;
            uint4* p = reinterpret_cast<uint4*>(counts + (size_t)(r0 + r) * RDX + d0);
#pragma unroll
            for (int q = 0; q < Q; ++q) {
                const uint4 x = v[r][q];
                p[q] = make_uint4(off[4 * q], off[4 * q + 1], off[4 * q + 2], off[4 * q + 3]);
                off[4 * q] += x.x; off[4 * q + 1] += x.y; off[4 * q + 2] += x.z; off[4 * q + 3] += x.w;
            }
        }
#pragma unroll
        for (int j = 0; j < DG; ++j) carry[j] += tot[j];
        __syncthreads();   // s_part reused by the next chunk
    }
    if (tid < DG) {
        uint32_t t = 0u;
#pragma unroll
        for (int j = 0; j < DG; ++j) t = tid == j ? carry[j] : t;
        totals[d0 + tid] = t;
    }
}

// digits per scan block: LSR_SCAN_DG = 4 / 8 / 16 overrides (diagnostic A/B)
static int scan_dg() {
    static const int dg = [] {
        const char* e = std::getenv("LSR_SCAN_DG");
        const int v = e ? std::atoi(e) : 0;
        return (v == 4 || v == 8 || v == 16) ? v : 16;
    }();
    return dg;
}
static void launch_rts_scan(const SortBatch& bt, int ns, int p, int items, int in_b, int nbits, hipStream_t st) {
    switch (scan_dg()) {   // the grid covers RDX digits (groups past a pass's digits exit)
        case 4: hipLaunchKernelGGL(k_rts_scan<4>, dim3(RDX / 4, ns), dim3(256), 0, st, bt, p, items, in_b, nbits); break;
        case 8: hipLaunchKernelGGL(k_rts_scan<8>, dim3(RDX / 8, ns), dim3(256), 0, st, bt, p, items, in_b, nbits); break;
        default: hipLaunchKernelGGL(k_rts_scan<16>, dim3(RDX / 16, ns), dim3(256), 0, st, bt, p, items, in_b, nbits); break;
    }
}

template <int IT>
__global__ void __launch_bounds__(256) k_rts_scatter(const SortBatch b, int pass, int in_b, int shift, int nbits_h,
                                                     int last_h) {
    __shared__ uint32_t s_key[(256 * IT)];
    __shared__ uint32_t s_val[(256 * IT)];
    __shared__ uint32_t s_wcnt[4][RDX];
    __shared__ uint32_t s_gbase[RDX];
    __shared__ uint32_t s_lbase[RDX];
    __shared__ uint32_t s_wave[4];
    const SortSeg& sg = b.s[blockIdx.y];
    const size_t nbi = rts_blocks(sg.n, IT);
    const uint32_t bid = blockIdx.x;
    if (bid >= nbi) return;                                          // block-uniform
    const PassDesc pd = pass_desc(sg, pass, in_b, shift, nbits_h, last_h);
    if (!pd.active) return;                                          // segment-uniform
    const uint32_t* __restrict__ keys_in = keys_of(sg, pd.src);
    const uint32_t* __restrict__ vals_in = vals_of(sg, pd.src);
    uint32_t* __restrict__ keys_out = keys_of_w(sg, pd.dst);
    uint32_t* __restrict__ vals_out = vals_of_w(sg, pd.dst);
    const int drop = sg.kept && pass == 0;
    uint32_t* kept_out = drop ? sg.kept : nullptr;
    const uint32_t* __restrict__ totals = rts_totals(sg, pass);
    const uint32_t* __restrict__ offs = rts_rows(sg, pass, nbi);
    const SortGather gather = pd.last ? sg.gather : SortGather{nullptr, nullptr, nullptr};
    const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
    const int nd = 1 << pd.nbits;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
        s_wcnt[w][tid] = 0;
        s_wcnt[w][tid + 256] = 0;
    }
    const size_t n = rts_n(sg.n, sg.kept && pass > 0 ? sg.kept : nullptr);
    __syncthreads();
    const uint32_t mask = (uint32_t)nd - 1u;
    const uint64_t lt = lanemask_lt();
    const size_t base = (size_t)bid * (256 * IT) + (size_t)wave * (64 * IT);
    uint32_t key[IT], val[IT], rank[IT];
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const size_t idx = base + (size_t)r * 64 + lane;
        const bool valid = idx < n;
        key[r] = valid ? keys_in[idx] : 0u;
        val[r] = valid ? vals_in[idx] : 0u;
    }
    // block offsets and digit starts of this thread's two digits (2 tid, 2 tid + 1): independent of
    // the ranking, loaded while it runs
    const int da = 2 * tid, db = 2 * tid + 1;
    const uint32_t pre_a = da < nd ? offs[(size_t)bid * RDX + da] : 0u, pre_b = db < nd ? offs[(size_t)bid * RDX + db] : 0u;
    const uint32_t hc_a = da < nd ? totals[da] : 0u, hc_b = db < nd ? totals[db] : 0u;
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const bool valid = base + (size_t)r * 64 + lane < n && !(drop && key[r] == 0xFFFFFFFFu);
        const uint32_t d = ((key[r] - pd.kbase) >> pd.shift) & mask;
        const uint64_t peers = match_digit(d, valid, pd.nbits);
        const uint32_t before = s_wcnt[wave][d];
        const uint32_t pr = (uint32_t)__popcll(peers & lt);
        rank[r] = before + pr;
        __builtin_amdgcn_wave_barrier();
        if (valid && pr == 0) s_wcnt[wave][d] = before + (uint32_t)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
    }
    __syncthreads();
    uint32_t tot_a, tot_b;
    {
        const uint32_t a0 = s_wcnt[0][da], a1 = s_wcnt[1][da], a2 = s_wcnt[2][da], a3 = s_wcnt[3][da];
        const uint32_t b0 = s_wcnt[0][db], b1 = s_wcnt[1][db], b2 = s_wcnt[2][db], b3 = s_wcnt[3][db];
        tot_a = a0 + a1 + a2 + a3;
        tot_b = b0 + b1 + b2 + b3;
        s_wcnt[0][da] = 0; s_wcnt[1][da] = a0; s_wcnt[2][da] = a0 + a1; s_wcnt[3][da] = a0 + a1 + a2;
        s_wcnt[0][db] = 0; s_wcnt[1][db] = b0; s_wcnt[2][db] = b0 + b1; s_wcnt[3][db] = b0 + b1 + b2;
    }
    const uint32_t dstart_a = block_excl_scan256(hc_a + hc_b, s_wave);   // global start of digit 2 tid
    const uint32_t lbase_a = block_excl_scan256(tot_a + tot_b, s_wave);  // local start of digit 2 tid
    s_lbase[da] = lbase_a;
    s_lbase[db] = lbase_a + tot_a;
    s_gbase[da] = dstart_a + pre_a - lbase_a;
    s_gbase[db] = dstart_a + hc_a + pre_b - (lbase_a + tot_a);
    if (tid == 255) {
        s_wave[0] = lbase_a + tot_a + tot_b;                          // keys this block places
        if (kept_out && bid == 0) *kept_out = dstart_a + hc_a + hc_b;  // keys kept over all blocks
    }
    __syncthreads();
    const int ntile = (int)s_wave[0];
#pragma unroll
    for (int r = 0; r < IT; ++r) {
        const bool valid = base + (size_t)r * 64 + lane < n && !(drop && key[r] == 0xFFFFFFFFu);
        if (valid) {
            const uint32_t d = ((key[r] - pd.kbase) >> pd.shift) & mask;
            const uint32_t pos = s_lbase[d] + s_wcnt[wave][d] + rank[r];
            s_key[pos] = key[r];
            s_val[pos] = val[r];
        }
    }
    __syncthreads();
    if (gather.rect) {   // last pass of the depth sort: the counts gather instead of the keys
        // every random rect load of the thread in flight before the first store (a load-store
        // loop waited one memory latency per key: 0.25 ms for the 8 views' last pass)
        uint2 rc[IT];
        uint32_t vv[IT], dd[IT];
#pragma unroll
        for (int r = 0; r < IT; ++r) {
            const int i = tid + 256 * r;
            const bool ok = i < ntile;
            const uint32_t k = s_key[ok ? i : 0], v = s_val[ok ? i : 0];
            vv[r] = v;
            dd[r] = s_gbase[((k - pd.kbase) >> pd.shift) & mask] + (uint32_t)i;
            rc[r] = ok ? gather.rect[v] : make_uint2(0u, 0u);
        }
#pragma unroll
        for (int r = 0; r < IT; ++r) {
            if (tid + 256 * r < ntile) {
                vals_out[dd[r]] = vv[r];
                gather.rect_sorted[dd[r]] = rc[r];
                gather.counts[dd[r]] = rect_count(rc[r]);
            }
        }
        return;
    }
    uint2* __restrict__ ranges = pd.last ? sg.ranges : nullptr;
    for (int i = tid; i < ntile; i += 256) {
        const uint32_t k = s_key[i];
        const uint32_t dst = s_gbase[((k - pd.kbase) >> pd.shift) & mask] + (uint32_t)i;
        keys_out[dst] = k;
        vals_out[dst] = s_val[i];
        if (ranges && k < sg.nranges) {
            // the tile ranges (upstream identifyTileRanges): a key's run inside this block's LDS is
            // contiguous in the output (one digit run), so its first / last element's position bounds
            // the key's range; runs of one key in neighbouring blocks meet through the atomics
            if (i == 0 || s_key[i - 1] != k) atomicMin(&ranges[k].x, dst);
            if (i == ntile - 1 || s_key[i + 1] != k) atomicMax(&ranges[k].y, dst + 1u);
        }
    }
}

static size_t os_blocks(size_t n) { return (n + OS_TILE - 1) / OS_TILE; }

size_t radix_temp_bytes(size_t n) {
    // digit totals [4][RDX] | plan | count rows [4][blocks][RDX] (blocks of OS_TILE keys: the most rows)
    return RTS_ROWS_OFF + align_up(4 * os_blocks(n) * RDX * 4, 256);
}

int radix_sort_batch(const SortSeg* segs, int nseg, int begin_bit, int end_bit, hipStream_t st) {
    SortBatch bt{};
    int ns = 0;
    size_t nmax = 0;
    for (int i = 0; i < nseg; ++i)
        if (segs[i].n > 0) { bt.s[ns++] = segs[i]; nmax = std::max(nmax, segs[i].n); }
    if (ns == 0 || end_bit <= begin_bit) return 0;
    // the device plan (vals_c) is the depth sort's and applies to the whole batch: every launch below
    // serves every segment, so a batch mixing planned and host-planned segments cannot be sorted
    for (int i = 1; i < ns; ++i)
        if ((bt.s[i].vals_c == nullptr) != (bt.s[0].vals_c == nullptr)) return -1;
    if (bt.s[0].vals_c && (begin_bit != 0 || end_bit != 32)) return -1;
    // keys per thread: 8 (2M keys: more, shorter blocks), 12 above 4M keys (the 6M-instance
    // tile sort: longer digit runs per block); swept 8 / 12 / 16 on both sorts
    // the device-planned depth sort takes 12 keys per thread: its 9-bit passes' digit runs are half
    // as long, and longer blocks win them back (depth sort 0.086-0.087 vs 0.088-0.090 ms per view
    // at 8; LSR_DEPTH_ITEMS=8 for A/B)
    static const int depth_items = [] {
        const char* e = std::getenv("LSR_DEPTH_ITEMS");
        return e && std::atoi(e) == 8 ? OS_ITEMS : 12;
    }();
    const int items = nmax > ((size_t)4 << 20) ? 12 : (bt.s[0].vals_c ? depth_items : OS_ITEMS);
    const unsigned nbi = (unsigned)((nmax + 256 * items - 1) / (256 * items));   // <= os_blocks: rows fit
    auto pass = [&](int p, int in_b, int shift, int nbits, int last) {
        if (items == 12)
            hipLaunchKernelGGL(k_rts_count<12>, dim3(nbi, ns), dim3(256), 0, st, bt, p, in_b, shift, nbits);
        else
            hipLaunchKernelGGL(k_rts_count<OS_ITEMS>, dim3(nbi, ns), dim3(256), 0, st, bt, p, in_b, shift, nbits);
        launch_rts_scan(bt, ns, p, items, in_b, nbits, st);
        if (items == 12)
            hipLaunchKernelGGL(k_rts_scatter<12>, dim3(nbi, ns), dim3(256), 0, st, bt, p, in_b, shift, nbits, last);
        else
            hipLaunchKernelGGL(k_rts_scatter<OS_ITEMS>, dim3(nbi, ns), dim3(256), 0, st, bt, p, in_b, shift, nbits,
                               last);
    };
    if (bt.s[0].vals_c) {   // the depth sort's device plan (every segment of the batch has one)
        for (int p = 0; p < 4; ++p) pass(p, 0, 0, 8, 0);
        return 0;           // either plan ends in the (a) buffers
    }
    bool in_b = false;
    // the bits spread evenly over the passes (13 bits: 7 + 6, not 8 + 5): fewer digits in a pass
    // mean longer runs per digit in its scatter, i.e. fuller write segments
    const int npass = (end_bit - begin_bit + 7) / 8;
    for (int shift = begin_bit, nbits = 0, p = 0; shift < end_bit; shift += nbits, ++p) {
        nbits = (end_bit - begin_bit) / npass + (p < (end_bit - begin_bit) % npass ? 1 : 0);
        pass(p, (int)in_b, shift, nbits, shift + nbits >= end_bit);
        in_b = !in_b;
    }
    return in_b ? 1 : 0;
}

bool radix_sort_pairs(uint32_t* keys_a, uint32_t* vals_a, uint32_t* keys_b, uint32_t* vals_b, size_t n,
                      int begin_bit, int end_bit, void* temp, hipStream_t st, uint32_t* kept, const SortGather* gather,
                      uint32_t* vals_c) {
    if (n == 0 || end_bit <= begin_bit) return false;
    SortSeg sg{keys_a, vals_a, keys_b, vals_b, temp, kept, gather ? *gather : SortGather{nullptr, nullptr, nullptr}, n};
    sg.vals_c = (vals_c && kept && gather && begin_bit == 0 && end_bit == 32) ? vals_c : nullptr;
    return radix_sort_batch(&sg, 1, begin_bit, end_bit, st) == 1;   // one segment: never mixed
}

}  // namespace lsr
