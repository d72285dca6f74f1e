// binning.hip -- (Gaussian, tile) instance emission in depth order and per-tile ranges.
//
// Upstream emits one 64-bit key (tile << 32 | depth bits) per instance and
// radix-sorts all of them on 32 + log2(tiles) bits.  Here the depth order is established once on
// the P Gaussians (sort.hip, 32-bit keys), instances are emitted in that order, and a stable sort
// on the tile id alone (13 bits at 5,440 tiles) finishes the job: the per-tile lists come out in
// the same (depth, index) order, with about a third of the sort traffic.
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

__global__ void __launch_bounds__(256) k_iota(int n, uint32_t* __restrict__ out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = (uint32_t)i;
}
void launch_iota(int n, uint32_t* out, hipStream_t st) {
    if (n > 0) hipLaunchKernelGGL(k_iota, dim3((n + 255) / 256), dim3(256), 0, st, n, out);
}

__global__ void __launch_bounds__(256) k_gather_tile_counts(int P, const uint32_t* __restrict__ order,
                                                            const uint32_t* __restrict__ tiles,
                                                            uint32_t* __restrict__ counts) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= P) return;
    counts[r] = tiles[order[r]];
}

void launch_gather_tile_counts(int P, const uint32_t* order, const uint32_t* tiles, uint32_t* counts, hipStream_t st) {
    if (P == 0) return;
    hipLaunchKernelGGL(k_gather_tile_counts, dim3((P + 255) / 256), dim3(256), 0, st, P, order, tiles, counts);
}

// One lane per depth rank: the tiles of its rectangle in row-major order, keys = tile id,
// values = Gaussian id.  inst_offset_by_id[g] = first instance slot of Gaussian g (the backward
// writes per-instance gradient records there, contiguous per Gaussian).
__global__ void __launch_bounds__(256) k_emit(int P, const uint32_t* __restrict__ order,
                                              const uint32_t* __restrict__ offsets,
                                              const uint32_t* __restrict__ tiles, const float2* __restrict__ xy,
                                              const int* __restrict__ radii, int gx, int gy,
                                              uint32_t* __restrict__ keys, uint32_t* __restrict__ vals,
                                              uint32_t* __restrict__ inst_offset_by_id) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= P) return;
    const uint32_t g = order[r];
    if (tiles[g] == 0) return;
    uint32_t off = offsets[r];
    if (inst_offset_by_id) inst_offset_by_id[g] = off;
    int2 rmin, rmax;
    tile_rect(xy[g], radii[g], gx, gy, rmin, rmax);
    for (int y = rmin.y; y < rmax.y; ++y)
        for (int x = rmin.x; x < rmax.x; ++x) {
            keys[off] = (uint32_t)(y * gx + x);
            vals[off] = g;
            ++off;
        }
}

void launch_emit_instances(int P, const uint32_t* order, const uint32_t* offsets, const uint32_t* tiles,
                           const float2* xy, const int* radii, int grid_x, int grid_y, uint32_t* keys,
                           uint32_t* vals, uint32_t* inst_offset_by_id, hipStream_t st) {
    if (P == 0) return;
    hipLaunchKernelGGL(k_emit, dim3((P + 255) / 256), dim3(256), 0, st, P, order, offsets, tiles, xy, radii,
                       grid_x, grid_y, keys, vals, inst_offset_by_id);
}

__global__ void __launch_bounds__(256) k_tile_ranges(size_t K, const uint32_t* __restrict__ keys,
                                                     uint2* __restrict__ ranges) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= K) return;
    const uint32_t t = keys[i];
    if (i == 0 || keys[i - 1] != t) ranges[t].x = (uint32_t)i;
    if (i == K - 1 || keys[i + 1] != t) ranges[t].y = (uint32_t)(i + 1);
}

void launch_tile_ranges(size_t K, const uint32_t* keys, uint2* ranges, hipStream_t st) {
    if (K == 0) return;
    hipLaunchKernelGGL(k_tile_ranges, dim3((unsigned)((K + 255) / 256)), dim3(256), 0, st, K, keys, ranges);
}

}  // namespace lsr
