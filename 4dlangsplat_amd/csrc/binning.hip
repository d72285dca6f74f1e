// binning.hip -- (Gaussian, tile) instance emission in depth order.  The per-tile ranges are made
// by the tile sort's last scatter pass (sort.hip).
//
// Upstream emits one 64-bit key (tile << 32 | depth bits) per instance and
// radix-sorts all of them on 32 + log2(tiles) bits.  Here the depth order is established once on
// the P Gaussians (sort.hip, 32-bit keys), instances are emitted in that order, and a stable sort
// on the tile id alone (13 bits at 5,440 tiles) finishes the job: the per-tile lists come out in
// the same (depth, index) order, with about a third of the sort traffic.
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

// Instance emission, one wave per 64 consecutive depth ranks.  Their instances occupy one
// contiguous slot range [offsets[r0], offsets[r0+63] + counts[r0+63]), so the wave walks that
// range with consecutive lanes on consecutive slots (fully coalesced key/value stores); a lane
// finds the rank owning its slot by binary search over the 64 start offsets in LDS.  Slot order
// inside a Gaussian is its rectangle in row-major order (as upstream's duplicateWithKeys).
// Each instance also gets the 8x8 quadrants of its tile that the splat may reach (a conservative
// test, emit_quad_mask) that the compositors' per-quadrant waves used to evaluate while scanning
// every list entry (quad_may_touch); once per instance here, so their scans read only the point
// list (no centre / conic gathers).  An instance reaching no quadrant would be skipped at every
// pixel of its tile: it gets key 0xFFFFFFFF, which the tile sort's first pass drops.
__global__ void __launch_bounds__(256) k_emit(const EmitBatch eb) {
    __shared__ uint32_t s_off[4][64];
    __shared__ uint2 s_rc[4][64];
    __shared__ uint32_t s_id[4][64];
    __shared__ EmitSplat s_sp[4][64];
    const EmitView& ev = eb.v[blockIdx.y];   // one view of the batch per grid row
    const int P = eb.P, gx = eb.grid_x, W = eb.W, H = eb.H;
    const uint32_t* __restrict__ order = ev.order;
    const uint32_t* __restrict__ offsets = ev.offsets;
    const uint32_t* __restrict__ counts = ev.counts;
    const uint2* __restrict__ rect_sorted = ev.rect_sorted;
    const float2* __restrict__ xy = ev.xy;
    const float4* __restrict__ conic_o = ev.conic_o;
    uint32_t* __restrict__ keys = ev.keys;
    uint32_t* __restrict__ vals = ev.vals;
    clear_words(ev.clear);   // tile ranges, per-tile bounds, tile-sort workspace (used after this kernel)
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int base = (blockIdx.x * 4 + w) * 64;
    if (base >= P) return;                                   // wave-uniform
    const int r = base + lane;
    const bool ok = r < P;
    const uint32_t cnt = ok ? counts[r] : 0u;
    const uint32_t off = ok ? offsets[r] : 0u;
    const int last = min(P - 1 - base, 63);
    const uint32_t end = __shfl(off + cnt, last);
    const uint32_t start = __shfl(off, 0);
    s_off[w][lane] = ok ? off : end;                         // past-the-end lanes never own a slot
    s_rc[w][lane] = ok ? rect_sorted[r] : make_uint2(0u, 0u);
    const uint32_t id = ok ? order[r] : 0u;
    s_id[w][lane] = id;
    // splats of rectangles beyond 2 x 2 tiles (no precomputed quadrant map): gathered here
    const uint2 rc_own = ok ? rect_sorted[r] : make_uint2(0u, 0u);
    uint32_t ox0, oy0, ox1, oy1;
    rect_unpack(rc_own, ox0, oy0, ox1, oy1);
    const bool big = ok && cnt > 0 && (ox1 - ox0 > 2 || oy1 - oy0 > 2);
    if (big) s_sp[w][lane] = emit_splat(xy[id], conic_o[id]);
    __builtin_amdgcn_wave_barrier();
    for (uint32_t j = start + lane; j < end; j += 64) {
        int k = 0;                                           // last rank with s_off <= j
#pragma unroll
        for (int step = 32; step >= 1; step >>= 1)
            if (s_off[w][k + step] <= j) k += step;
        const uint2 rc = s_rc[w][k];
        uint32_t x0, y0, x1, y1;
        rect_unpack(rc, x0, y0, x1, y1);
        const uint32_t wd = x1 - x0;
        const uint32_t loc = j - s_off[w][k];
        uint32_t dx, dy, quads;
        if (rect_small(x0, y0, x1, y1)) {   // the preprocess's map: the loc-th reachable tile
            const uint32_t map = rect_quad_map(rc);
            uint32_t m = rect_tile_mask(map);
            for (uint32_t i = 0; i < loc; ++i) m &= m - 1u;
            const uint32_t pos = (uint32_t)__builtin_ctz(m);
            dx = pos & 1u;
            dy = pos >> 1;
            const uint32_t sh = 8 * dy + 2 * dx;
            quads = ((map >> sh) & 3u) | (((map >> (sh + 4)) & 3u) << 2);
        } else {
            dy = loc / wd;
            dx = loc - dy * wd;
            quads = emit_quad_mask(s_sp[w][k], (int)(x0 + dx) * LSR_TILE_X, (int)(y0 + dy) * LSR_TILE_Y, W, H);
        }
        const uint32_t tx = x0 + dx, ty = y0 + dy;
        keys[j] = quads ? ty * (uint32_t)gx + tx : 0xFFFFFFFFu;   // dropped by the tile sort's first pass
        vals[j] = s_id[w][k] | (quads << PL_QUAD_SHIFT);
    }
}

void launch_emit_instances(const EmitBatch& eb, int nv, hipStream_t st) {
    if (eb.P == 0 || nv <= 0) return;
    hipLaunchKernelGGL(k_emit, dim3((eb.P + 255) / 256, nv), dim3(256), 0, st, eb);
}

// inst_off[g] = first instance slot of Gaussian g: only the deterministic backward needs it (its
// per-(Gaussian, tile) records are addressed by it), so it is scattered there, not in the forward.
__global__ void __launch_bounds__(256) k_scatter_inst_off(int P, const uint32_t* __restrict__ order,
                                                          const uint32_t* __restrict__ offsets,
                                                          const uint32_t* __restrict__ counts,
                                                          uint32_t* __restrict__ inst_off) {
    const int r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < P && counts[r] > 0) inst_off[order[r]] = offsets[r];
}

void launch_scatter_inst_off(int P, const uint32_t* order, const uint32_t* offsets, const uint32_t* counts,
                             uint32_t* inst_off, hipStream_t st) {
    if (P == 0) return;
    hipLaunchKernelGGL(k_scatter_inst_off, dim3((P + 255) / 256), dim3(256), 0, st, P, order, offsets, counts,
                       inst_off);
}

}  // namespace lsr
