// render_fwd.hip -- the compositor forward's entry point.
//
// Upstream renderCUDA restated: alpha <= 0.99, skip alpha < 1/255, stop when T (1 - alpha) < 1e-4,
// RGB += T bg, language channels without background, depth = sum z alpha T; per tile the largest
// n_contrib of its pixels (the backward's replay bound).  Every channel count runs on the
// compacted per-quadrant waves: render_fwd_wave.hip (VALU sums, C <= 16 or > 32) and
// render_fwd_mfma_wave.hip (17..32 channels, sums on matrix cores).  Round 1's one-workgroup-per-
// tile kernels were removed in round 3 (DESIGN.md 7.1 records their numbers).
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

void launch_render_fwd(const RenderFwdArgs& a, hipStream_t st) { launch_render_fwd_views(&a, 1, st); }

void launch_render_fwd_views(const RenderFwdArgs* a, int n, hipStream_t st) {
    RenderFwdArgs f[LSR_MAX_VIEWS];
    for (int v = 0; v < n; ++v) {
        f[v] = a[v];
        f[v].tile_order = nullptr;   // the forward takes no cost order: its scratch is not written
    }
    launch_render_fwd_wave_views(f, n, st);
}

}  // namespace lsr
