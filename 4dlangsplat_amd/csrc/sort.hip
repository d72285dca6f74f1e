// sort.hip -- device-wide exclusive scan and stable LSD radix sort of (u32 key, u32 value) pairs,
// written for wave64: per-wave digit matching by ballots (one 64-bit ballot per key bit), per-wave
// digit counts in LDS, and per-digit running offsets, so every pass is stable.
//
// Used twice per frame by the binning (binning.hip):
//   1. depth order of all P Gaussians: key = view-space depth bits (culled = 0xFFFFFFFF), 4 passes;
//   2. tile order of the K (Gaussian, tile) instances emitted in depth order: key = tile id,
//      ceil(log2(tiles)) bits (2 passes at 5,440 tiles).
// Stable tile sort of depth-ordered instances == the upstream sort of (tile << 32 | depth) keys.
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

constexpr int SCAN_ITEMS = 8;
constexpr int SCAN_TILE = 256 * SCAN_ITEMS;
constexpr int RADIX_ITEMS = 16;
constexpr int RADIX_TILE = 256 * RADIX_ITEMS;

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
    uint32_t* scanned = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(temp) + align_up(nb * 4, 256));
    void* deeper = reinterpret_cast<char*>(temp) + 2 * align_up(nb * 4, 256);
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)nb), dim3(256), 0, st, in, n, partials);
    exclusive_scan_u32(partials, scanned, nb, total, deeper, st);
    hipLaunchKernelGGL(k_scan_down, dim3((unsigned)nb), dim3(256), 0, st, in, out, n, (const uint32_t*)scanned,
                       (uint32_t*)nullptr);
}

// ---- radix sort -------------------------------------------------------------------------------
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

__global__ void __launch_bounds__(256) k_radix_count(const uint32_t* __restrict__ keys, size_t n, int shift,
                                                     int nbits, uint32_t* __restrict__ counts, uint32_t nb) {
    __shared__ uint32_t s_h[256];
    const int tid = threadIdx.x;
    s_h[tid] = 0;
    __syncthreads();
    const uint32_t mask = (1u << nbits) - 1u;
    const uint64_t lt = lanemask_lt();
    const size_t base = (size_t)blockIdx.x * RADIX_TILE;
    for (int r = 0; r < RADIX_ITEMS; ++r) {
        const size_t idx = base + (size_t)r * 256 + tid;
        const bool valid = idx < n;
        const uint32_t d = valid ? (keys[idx] >> shift) & mask : 0u;
        const uint64_t peers = match_digit(d, valid, nbits);
        if (valid && __popcll(peers & lt) == 0) atomicAdd(&s_h[d], (uint32_t)__popcll(peers));
    }
    __syncthreads();
    counts[(size_t)tid * nb + blockIdx.x] = s_h[tid];
}

__global__ void __launch_bounds__(256) k_radix_scatter(const uint32_t* __restrict__ keys_in,
                                                       const uint32_t* __restrict__ vals_in,
                                                       uint32_t* __restrict__ keys_out, uint32_t* __restrict__ vals_out,
                                                       size_t n, int shift, int nbits,
                                                       const uint32_t* __restrict__ offsets, uint32_t nb) {
    __shared__ uint32_t s_run[256];
    __shared__ uint32_t s_cnt[4][256];
    __shared__ uint32_t s_off[4][256];
    const int tid = threadIdx.x, wave = tid >> 6;
    s_run[tid] = offsets[(size_t)tid * nb + blockIdx.x];
#pragma unroll
    for (int w = 0; w < 4; ++w) s_cnt[w][tid] = 0;
    __syncthreads();
    const uint32_t mask = (1u << nbits) - 1u;
    const uint64_t lt = lanemask_lt();
    const size_t base = (size_t)blockIdx.x * RADIX_TILE;
    for (int r = 0; r < RADIX_ITEMS; ++r) {
        const size_t idx = base + (size_t)r * 256 + tid;
        const bool valid = idx < n;
        uint32_t key = 0, val = 0, d = 0;
        if (valid) { key = keys_in[idx]; val = vals_in[idx]; d = (key >> shift) & mask; }
        const uint64_t peers = match_digit(d, valid, nbits);
        const uint32_t rank = (uint32_t)__popcll(peers & lt);
        if (valid && rank == 0) s_cnt[wave][d] = (uint32_t)__popcll(peers);
        __syncthreads();
        {
            uint32_t run = s_run[tid];
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                const uint32_t c = s_cnt[w][tid];
                s_off[w][tid] = run;
                run += c;
                s_cnt[w][tid] = 0;
            }
            s_run[tid] = run;
        }
        __syncthreads();
        if (valid) {
            const uint32_t dst = s_off[wave][d] + rank;
            keys_out[dst] = key;
            vals_out[dst] = val;
        }
    }
}

size_t radix_temp_bytes(size_t n) {
    const size_t nb = (n + RADIX_TILE - 1) / RADIX_TILE;
    const size_t nc = nb * 256;
    return align_up(nc * 4, 256) * 2 + scan_temp_bytes(nc);
}

bool radix_sort_pairs(uint32_t* keys_a, uint32_t* vals_a, uint32_t* keys_b, uint32_t* vals_b, size_t n,
                      int begin_bit, int end_bit, void* temp, hipStream_t st) {
    if (n == 0 || end_bit <= begin_bit) return false;
    const size_t nb = (n + RADIX_TILE - 1) / RADIX_TILE;
    const size_t nc = nb * 256;
    uint32_t* counts = reinterpret_cast<uint32_t*>(temp);
    uint32_t* offs = reinterpret_cast<uint32_t*>(reinterpret_cast<char*>(temp) + align_up(nc * 4, 256));
    void* scan_tmp = reinterpret_cast<char*>(temp) + 2 * align_up(nc * 4, 256);
    bool in_b = false;
    for (int shift = begin_bit; shift < end_bit; shift += 8) {
        const int nbits = (end_bit - shift) < 8 ? (end_bit - shift) : 8;
        const uint32_t* kin = in_b ? keys_b : keys_a;
        const uint32_t* vin = in_b ? vals_b : vals_a;
        uint32_t* kout = in_b ? keys_a : keys_b;
        uint32_t* vout = in_b ? vals_a : vals_b;
        hipLaunchKernelGGL(k_radix_count, dim3((unsigned)nb), dim3(256), 0, st, kin, n, shift, nbits, counts, (uint32_t)nb);
        exclusive_scan_u32(counts, offs, nc, (uint32_t*)nullptr, scan_tmp, st);
        hipLaunchKernelGGL(k_radix_scatter, dim3((unsigned)nb), dim3(256), 0, st, kin, vin, kout, vout, n, shift, nbits,
                           (const uint32_t*)offs, (uint32_t)nb);
        in_b = !in_b;
    }
    return in_b;
}

}  // namespace lsr
