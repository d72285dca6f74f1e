/*
 * lsr.h -- C ABI of liblsr.so, the MI355X-native (gfx950, HIP) 4D language-feature Gaussian
 * rasterizer.  Drop-in for the native half of diff_gaussian_rasterization as used by 4D-LangSplat.
 *
 * Reference interface this replaces (the un-vendored submodule zrporz/4d-langsplat-rasterization,
 * /root/reference/.gitmodules:4-6; source absent, so the binding is cited at its call sites):
 *   - GaussianRasterizationSettings(...)            gaussian_renderer/__init__.py:49-63,
 *                                                    scene/dataset_readers.py:502-515
 *   - GaussianRasterizer(raster_settings)(means3D, means2D, shs, colors_precomp,
 *       language_feature_precomp, opacities, scales, rotations, cov3D_precomp)
 *       -> (color [3,H,W], language_feature [C,H,W], radii int32 [P], depth [1,H,W])
 *                                                    gaussian_renderer/__init__.py:79,219-228
 *   - _C.rasterize_gaussians            -> lsr_forward_preprocess + lsr_forward_render
 *   - _C.rasterize_gaussians_backward   -> lsr_backward
 *   - _C.mark_visible                   -> lsr_mark_visible
 *   The upstream byte buffers (geomBuffer / binningBuffer / imgBuffer, sized through resize
 *   callbacks) become caller-owned workspaces sized by the *_bytes queries below.
 *
 * Conventions
 *   - Every pointer is a DEVICE pointer to contiguous memory: float32 except radii (int32) and
 *     present (uint8).  Matrices are the torch world_view_transform / full_proj_transform
 *     (flat 16 floats, row-vector convention: row 0 of the transform is m[0], m[4], m[8], m[12]).
 *   - The library allocates nothing; the caller owns every input, output and workspace buffer.
 *   - Every launch goes on `stream` (a hipStream_t).  The only host synchronisation is the read
 *     of num_rendered at the end of lsr_forward_preprocess (as upstream).
 *   - Return value: 0 = success, otherwise an LSR_E* code; lsr_last_error() describes the last
 *     failure of the calling thread.
 *   - C (language channels) is a runtime value.  include_feature = 0 skips the language
 *     channels (their output is written as zeros), as the 'base' training stages do.
 */
#ifndef LSR_H_
#define LSR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LSR_API_VERSION 4   /* 3: lsr_fwd_in.language_feature_split, lsr_language_split;
                               4: lsr_require_api; the sort status words are gone (lsr_fwd_out
                                  .host_sort_status, lsr_forward_status, lsr_test_inject_sort_fault:
                                  the radix sorts have no look-back that could time out) */

#define LSR_OK 0
#define LSR_EINVAL 1     /* bad argument (null pointer, exactly-one-of violation, size) */
#define LSR_EHIP 2       /* HIP runtime / launch error */
#define LSR_ECAPACITY 3  /* workspace too small */

typedef void *lsr_stream_t; /* hipStream_t */

typedef struct lsr_settings {
    int32_t image_height;
    int32_t image_width;
    float tanfovx;
    float tanfovy;
    const float *bg;          /* [3] */
    float scale_modifier;
    const float *viewmatrix;  /* [16] world_view_transform */
    const float *projmatrix;  /* [16] full_proj_transform */
    int32_t sh_degree;        /* active SH degree, 0..3 */
    const float *campos;      /* [3] camera centre */
    int32_t prefiltered;
    int32_t debug;            /* 1: synchronise and check after every kernel */
    int32_t include_feature;
} lsr_settings;

typedef struct lsr_fwd_in {
    int32_t P;                        /* Gaussians */
    int32_t M;                        /* SH coefficients per Gaussian (shs.shape[1]); 0 if shs == NULL */
    int32_t C;                        /* language-feature channels (0 allowed) */
    const float *means3D;             /* [P,3] */
    const float *shs;                 /* [P,M,3]  exactly one of shs / colors_precomp */
    const float *colors_precomp;      /* [P,3] */
    const float *language_feature;    /* [P,C]  (may be NULL when C == 0) */
    const float *opacities;           /* [P]    activated */
    const float *scales;              /* [P,3]  activated; with rotations, or cov3D_precomp */
    const float *rotations;           /* [P,4]  activated (normalised) */
    const float *cov3D_precomp;       /* [P,6] */
    const uint16_t *language_feature_split; /* optional, C == 32 only: [P,64] bf16 bit patterns, per
                                         Gaussian the 32 channels' bf16(x) then bf16(x - bf16(x)),
                                         as lsr_language_split writes them (the compositors' matrix-
                                         core operands, made once for all views of a batch instead
                                         of per entry in every quadrant wave: same bits, same
                                         results).  NULL: split in the compositors. */
} lsr_fwd_in;

typedef struct lsr_fwd_out {
    float *out_color;                 /* [3,H,W] */
    float *out_language_feature;      /* [C,H,W] (may be NULL when C == 0) */
    int32_t *radii;                   /* [P] */
    float *out_depth;                 /* [1,H,W] */
} lsr_fwd_out;

typedef struct lsr_bwd_in {
    const float *dL_dout_color;              /* [3,H,W] */
    const float *dL_dout_language_feature;   /* [C,H,W] or NULL (treated as zero) */
    const float *dL_dout_depth;              /* [1,H,W] or NULL (treated as zero) */
    int32_t deterministic;                   /* 1: fixed-order reduction, bitwise reproducible
                                                gradients (slower); 0: float atomics, as upstream */
} lsr_bwd_in;

typedef struct lsr_bwd_out {                 /* any pointer may be NULL if that gradient is unused */
    float *dL_dmeans3D;               /* [P,3] */
    float *dL_dmeans2D;               /* [P,3] NDC units (x 0.5 W, 0.5 H), z = 0 */
    float *dL_dcolors;                /* [P,3] */
    float *dL_dlanguage_feature;      /* [P,C] */
    float *dL_dopacity;               /* [P]   */
    float *dL_dcov3D;                 /* [P,6] */
    float *dL_dsh;                    /* [P,M,3] */
    float *dL_dscales;                /* [P,3] */
    float *dL_drotations;             /* [P,4] */
} lsr_bwd_out;

int lsr_version(void);
const char *lsr_last_error(void);
/* Call once before any other entry point with LSR_API_VERSION from the lsr.h the caller was built
 * against: the structs above are read with THIS header's layout, so a caller built against another
 * version is refused (LSR_EINVAL, every entry point) instead of having trailing fields misread. */
int lsr_require_api(int32_t caller_version);

/* Workspace sizes in bytes (upstream geomBuffer / binningBuffer / imgBuffer + backward scratch). */
int64_t lsr_geom_bytes(int32_t P);
int64_t lsr_binning_bytes(int64_t num_rendered);
int64_t lsr_img_bytes(int32_t image_width, int32_t image_height);
int64_t lsr_backward_bytes(int32_t P, int64_t num_rendered, int32_t C, int32_t deterministic);

/* Forward, phase 1: per-Gaussian preprocess (cull, EWA projection, SH colour, tile count) and
 * the depth ordering of the visible set.  Writes out->radii.  Returns num_rendered, the number of
 * (Gaussian, tile) instances; the caller then sizes `binning`.  Synchronises `stream`. */
int lsr_forward_preprocess(const lsr_settings *s, const lsr_fwd_in *in, lsr_fwd_out *out, void *geom,
                           int64_t *num_rendered, lsr_stream_t stream);

/* lsr_forward_preprocess without the host synchronisation: the same launches, then an
 * asynchronous copy of two words to `host_count` (page-locked host memory): [0] num_rendered,
 * [1] reserved (0).  Valid once the stream
 * has passed this point (an event recorded after the call).  Lets a caller enqueue the next
 * view's preprocess ahead of the current view's compositing on ONE stream and read the count
 * later, so the device never idles on the host between views. */
int lsr_forward_preprocess_async(const lsr_settings *s, const lsr_fwd_in *in, lsr_fwd_out *out, void *geom,
                                 uint32_t *host_count, lsr_stream_t stream);

/* lsr_forward_preprocess_async for n_views >= 1 cameras of the same Gaussians `in` (one training
 * batch), batched: ONE preprocess launch per 8 views reads each Gaussian's inputs (and builds its
 * 3D covariance) once for all of them, and the depth sorts and instance scans of those views run
 * as one set of launches (every kernel serves all the views).  s[v], out[v], geom[v] are view v's
 * (workspaces as for lsr_forward_preprocess_async); `host_counts` (page-locked, 2 * n_views words)
 * receives [2v] num_rendered of view v ([2v + 1] reserved, 0), valid once the
 * stream has passed this point.  The views must share the image size, sh_degree and
 * scale_modifier.  Results equal lsr_forward_preprocess_async per view.  The pointer arrays are
 * HOST arrays. */
int lsr_forward_preprocess_views_async(int32_t n_views, const lsr_settings *const *s, const lsr_fwd_in *in,
                                       lsr_fwd_out *const *out, void *const *geom, uint32_t *host_counts,
                                       lsr_stream_t stream);

/* lsr_forward_preprocess_views_async in two parts, so that the depth ordering of some views can
 * run on a second stream (behind an event the caller records after this call) while the first
 * views bin and composite: the preprocess of all n_views views (one launch per 8), then the depth
 * ordering and instance counts of the first n_ordered (0 <= n_ordered <= n_views) on `stream`,
 * their counts in host_counts[2v] as above.  The other views are then ordered by
 * lsr_forward_depth_order_views_async (given their s / geom arrays).  Same results as
 * lsr_forward_preprocess_views_async. */
int lsr_forward_preprocess_views_split_async(int32_t n_views, int32_t n_ordered, const lsr_settings *const *s,
                                             const lsr_fwd_in *in, lsr_fwd_out *const *out, void *const *geom,
                                             uint32_t *host_counts, lsr_stream_t stream);
/* The preprocess of lsr_forward_preprocess_views_split_async(n_ordered = 0) for the Gaussians
 * [row0, row1) only (row0 a multiple of 256): a caller whose inputs arrive in row chunks (the sharded
 * optimizer's all-gather) preprocesses each chunk as it lands, then orders the views with
 * lsr_forward_depth_order_views_async once every row [0, P) was preprocessed. */
int lsr_forward_preprocess_views_rows_async(int32_t n_views, int32_t row0, int32_t row1, const lsr_settings *const *s,
                                            const lsr_fwd_in *in, lsr_fwd_out *const *out, void *const *geom,
                                            lsr_stream_t stream);
/* Depth ordering + instance counts of n_views views whose preprocess already ran (geom[v] as that
 * call left it): one set of sort and scan launches per 8 views; host_counts as above. */
int lsr_forward_depth_order_views_async(int32_t n_views, const lsr_settings *const *s, const lsr_fwd_in *in,
                                        void *const *geom, uint32_t *host_counts, lsr_stream_t stream);

/* Forward, phase 2: tile binning and compositing of RGB + C language channels + depth.
 * `geom` is the buffer phase 1 filled; `binning` holds >= lsr_binning_bytes(num_rendered) bytes. */
int lsr_forward_render(const lsr_settings *s, const lsr_fwd_in *in, lsr_fwd_out *out, void *geom,
                       void *binning, void *img, int64_t num_rendered, lsr_stream_t stream);

/* lsr_forward_render in two halves, so that the binning of one view can run on a side stream
 * while another view composites (lsr_forward_render == binning then composite on one stream).
 * Binning: instance emission, stable tile sort, per-tile ranges (fills `binning`, and the tile
 * ranges in `img`).  Composite: front-to-back compositing of the binned lists (fills `out` and the
 * rest of `img`).  Neither synchronises the host. */
int lsr_forward_binning(const lsr_settings *s, const lsr_fwd_in *in, void *geom, void *binning, void *img,
                        int64_t num_rendered, lsr_stream_t stream);
int lsr_forward_composite(const lsr_settings *s, const lsr_fwd_in *in, lsr_fwd_out *out, const void *geom,
                          const void *binning, void *img, int64_t num_rendered, lsr_stream_t stream);
/* lsr_forward_binning of n_views >= 1 views of the same Gaussians (phase 1 done, by either entry
 * point): the emissions, tile sorts and tile ranges of all of them as one set of launches per 8
 * views.  geom[v], binning[v], img[v], num_rendered[v] are view v's; the views must share the
 * image size.  Results equal lsr_forward_binning per view.  HOST pointer arrays. */
int lsr_forward_binning_views(int32_t n_views, const lsr_settings *const *s, const lsr_fwd_in *in,
                              void *const *geom, void *const *binning, void *const *img,
                              const int64_t *num_rendered, lsr_stream_t stream);

/* Tile-bucket binning: the same per-tile lists (same entries, same (depth, id) order) without the
 * depth sort of the Gaussians or a sort of all instances.  Phase 1 is
 * lsr_forward_preprocess_views_tb_async (the preprocess of rows [row0, row1) of n_views views; the
 * per-Gaussian instance counts are kept in id order) over every row, then
 * lsr_forward_instance_scan_views_async (their exclusive scans; num_rendered into host_counts as
 * for lsr_forward_depth_order_views_async); phase 2 is lsr_forward_binning_views_tb (instances
 * bucketed by tile, each bucket sorted in LDS) with binning[v] of >= lsr_binning_bytes_tb bytes, then
 * lsr_forward_composite_views / lsr_backward as usual.  A geom workspace prepared by one binning
 * must be binned by the same one.  At most 12288 tiles (LSR_EINVAL otherwise).  Replaces the same
 * upstream stages as the sort path (rasterizer_impl.cu's InclusiveSum, duplicateWithKeys,
 * SortPairs and identifyTileRanges). */
int64_t lsr_binning_bytes_tb(int64_t num_rendered, int32_t P, int32_t image_width, int32_t image_height);
int lsr_forward_preprocess_views_tb_async(int32_t n_views, int32_t row0, int32_t row1, const lsr_settings *const *s,
                                          const lsr_fwd_in *in, lsr_fwd_out *const *out, void *const *geom,
                                          lsr_stream_t stream);
int lsr_forward_instance_scan_views_async(int32_t n_views, const lsr_settings *const *s, const lsr_fwd_in *in,
                                          void *const *geom, uint32_t *host_counts, lsr_stream_t stream);
int lsr_forward_binning_views_tb(int32_t n_views, const lsr_settings *const *s, const lsr_fwd_in *in,
                                 void *const *geom, void *const *binning, void *const *img,
                                 const int64_t *num_rendered, lsr_stream_t stream);
/* lsr_forward_composite of n_views >= 1 binned views of the same Gaussians in ONE compositor
 * launch per 8 views (grid row = view: a view's last waves run beside the next view's first ones
 * instead of the chip draining between per-view launches).  out[v], geom[v], binning[v], img[v],
 * num_rendered[v] are view v's; the views must share the image size and include_feature.  Results
 * equal lsr_forward_composite per view.  HOST pointer arrays. */
int lsr_forward_composite_views(int32_t n_views, const lsr_settings *const *s, const lsr_fwd_in *in,
                                lsr_fwd_out *const *out, const void *const *geom, const void *const *binning,
                                void *const *img, const int64_t *num_rendered, lsr_stream_t stream);

/* Backward through compositing and preprocess.  accumulate != 0 adds into the outputs instead of
 * overwriting them (multi-view gradient accumulation).  `scratch` holds >= lsr_backward_bytes. */
int lsr_backward(const lsr_settings *s, const lsr_fwd_in *in, const lsr_bwd_in *gin, lsr_bwd_out *gout,
                 const void *geom, const void *binning, const void *img, void *scratch, int64_t num_rendered,
                 int32_t accumulate, lsr_stream_t stream);

/* Backward of n_views >= 1 views of the same Gaussians `in` (one training batch), summed:
 * gout (+)= sum_v dL_v/d(inputs) (accumulate != 0 adds to gout; otherwise gout is overwritten).
 * This is what train.py's loss.backward() does over its per-view renders
 * (/root/reference/train.py:242-268,339), in one call: every view's compositor backward runs on
 * `stream`, then ONE preprocess backward per 8 views reads each Gaussian's rows and writes its
 * gradient rows once instead of once per view.  Float-atomic reduction only (every gin[v] must
 * have deterministic == 0; lsr_backward per view gives the deterministic mode).  All views must
 * share scale_modifier.  s[v], gin[v], geom[v], binning[v], img[v], num_rendered[v] are view v's
 * forward state; the per-Gaussian screen-space sums live in geom (its accumulator rows were zeroed
 * by the forward), so each forward is backpropagated by this call ONCE.  The pointer arrays are
 * HOST arrays of device pointers. */
int lsr_backward_views(int32_t n_views, const lsr_settings *const *s, const lsr_fwd_in *in,
                       const lsr_bwd_in *const *gin, lsr_bwd_out *gout, void *const *geom,
                       const void *const *binning, const void *const *img, const int64_t *num_rendered,
                       int32_t accumulate, lsr_stream_t stream);

/* lsr_backward_views in two halves, so that a view's compositor backward can run as soon as its
 * upstream gradients exist (and overlap the next view's preprocess on another stream), while the
 * preprocess backward still runs once per batch:
 *  - lsr_backward_composite: compositor backward of ONE view; its per-Gaussian screen-space sums
 *    are added to accumulator rows in `geom` (zeroed by lsr_forward_preprocess), so it runs EXACTLY
 *    ONCE per forward: a second call on the same forward state doubles every screen-space sum the
 *    preprocess backward consumes (the Python wrapper raises on reuse).  Its language gradients are
 *    ADDED to dL_dlanguage [P,C] (zero it first; NULL skips them).  Float atomics only.
 *  - lsr_backward_preprocess_views: the preprocess backward of n_views views whose composite
 *    backward ran: gout (+)= sum_v (every output except dL_dlanguage_feature, which the composite
 *    calls already filled). */
int lsr_backward_composite(const lsr_settings *s, const lsr_fwd_in *in, const lsr_bwd_in *gin, float *dL_dlanguage,
                           void *geom, const void *binning, const void *img, int64_t num_rendered,
                           lsr_stream_t stream);
/* lsr_backward_composite of n_views >= 1 views in one compositor launch per 8 views (and one
 * launch for their tile orders); same image size and include_feature; the same once-per-forward
 * rule per view.  Equals lsr_backward_composite per view up to the order of float atomics. */
int lsr_backward_composite_views(int32_t n_views, const lsr_settings *const *s, const lsr_fwd_in *in,
                                 const lsr_bwd_in *const *gin, float *dL_dlanguage, void *const *geom,
                                 const void *const *binning, const void *const *img,
                                 const int64_t *num_rendered, lsr_stream_t stream);
int lsr_backward_preprocess_views(int32_t n_views, const lsr_settings *const *s, const lsr_fwd_in *in,
                                  lsr_bwd_out *gout, const void *const *geom, int32_t accumulate,
                                  lsr_stream_t stream);
/* lsr_backward_preprocess_views over the Gaussian rows [row_begin, row_begin + row_count) only
 * (row_begin a multiple of 256); every gout pointer addresses row row_begin of its array.  Lets a
 * data-parallel caller start the all-reduce of finished rows while the next rows are computed. */
int lsr_backward_preprocess_views_rows(int32_t n_views, const lsr_settings *const *s, const lsr_fwd_in *in,
                                       lsr_bwd_out *gout, const void *const *geom, int32_t accumulate,
                                       int32_t row_begin, int32_t row_count, lsr_stream_t stream);

/* language_feature [P,C] fp32 -> out [P,2C] bf16 bit patterns (hi channels then lo channels) for
 * lsr_fwd_in.language_feature_split.  C must be 32.  No reference counterpart (an MI355X operand
 * layout); on the caller's stream. */
int lsr_language_split(int32_t P, int32_t C, const float *language_feature, uint16_t *out, lsr_stream_t stream);

/* out[i] = max(out[i] if accumulate, radii_v[i] over the n_views views): the radii MAX of a training
 * batch's views (/root/reference/train.py:270, torch.stack(radii_list).max(dim=0)), one pass over
 * host array `radii` of 16-byte aligned device pointers.  No reference counterpart in the rasterizer
 * (the reference reduces with PyTorch). */
int lsr_radii_max(int32_t P, int32_t n_views, const int32_t *const *radii, int32_t *out, int32_t accumulate,
                  lsr_stream_t stream);

/* markVisible: present[i] = (view-space z of means3D[i]) > 0.2 */
int lsr_mark_visible(int32_t P, const float *means3D, const float *viewmatrix, const float *projmatrix,
                     uint8_t *present, lsr_stream_t stream);

/* Per-phase GPU timing (profiling aid): when enabled, every phase below is bracketed by hipEvents
 * recorded on the caller's stream.  lsr_profile_read waits for the recorded events, adds their
 * durations to per-phase totals (milliseconds) and launch counts, and returns LSR_NUM_PHASES. */
#define LSR_PHASE_PREPROCESS 0
#define LSR_PHASE_DEPTH_SORT 1
#define LSR_PHASE_INSTANCE_SCAN 2
#define LSR_PHASE_EMIT 3
#define LSR_PHASE_TILE_SORT 4
#define LSR_PHASE_TILE_RANGES 5
#define LSR_PHASE_RENDER_FWD 6
#define LSR_PHASE_RENDER_BWD 7
#define LSR_PHASE_PREPROCESS_BWD 8
#define LSR_PHASE_PREPROCESS_BWD_VIEWS 9   /* lsr_backward_views: one launch per <= 8 views */
#define LSR_NUM_PHASES 10
int lsr_profile_enable(int32_t on);   /* resets the totals */
/* Which phases are timed while profiling is on: bit (1 << LSR_PHASE_*); default all.  Each timed
 * phase adds two event records to its stream. */
int lsr_profile_phases(uint32_t mask);
int lsr_profile_read(double *ms_total, int64_t *launches, int32_t n);

#ifdef __cplusplus
}
#endif
#endif /* LSR_H_ */
