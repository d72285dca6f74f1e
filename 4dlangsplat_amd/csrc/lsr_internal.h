// lsr_internal.h -- kernel argument blocks and launcher declarations shared by the HIP sources.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lsr {

// Pitch (floats) of the per-Gaussian screen-space gradient accumulators of the atomic backward
// ([P, ACC_PITCH], fields 0..9 used: rgb 0-2, depth 3, mean2D 4-5, conic 6-8, opacity 9): 64-byte
// records, so the atomics of one entry are one 64-byte memory-side request.
constexpr int ACC_PITCH = 16;

// Word ranges a kernel zeroes on the side (grid-stride), for the kernels that follow it in stream
// order: replaces separate hipMemsetAsync launches (each a dispatch that waits for a free CU).
struct ClearList {
    uint32_t* p[4];
    uint32_t n[4];
    uint32_t even[4];   // value of the even-indexed words (odd ones are zeroed); 0 = plain clear
};

constexpr int LSR_MAX_VIEWS = 8;   // views per launch; more are processed in chunks
__device__ __forceinline__ void clear_words(const ClearList& c) {
    const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x, stride = gridDim.x * blockDim.x;
#pragma unroll
    for (int k = 0; k < 4; ++k)
        for (uint32_t i = t; i < c.n[k]; i += stride) c.p[k][i] = (i & 1u) ? 0u : c.even[k];
}

// Packed binning rectangle [x0, x1) x [y0, y1) in tiles (12 bits each: <= 4096 tiles per axis)
// plus, for rectangles of at most 2 x 2 tiles, the 16-bit map of the quadrants the splat may
// reach (bit (2 (ty - y0) + band) * 4 + 2 (tx - x0) + column; emit_quad_mask), computed by the
// preprocess while the splat is in registers so the binning needs no centre / conic gather for
// them.  .x = x0 | y0 << 12 | map[0:8] << 24, .y = x1 | y1 << 12 | map[8:16] << 24.
__host__ __device__ __forceinline__ uint2 rect_pack(uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1, uint32_t map) {
    return make_uint2(x0 | y0 << 12 | (map & 0xFFu) << 24, x1 | y1 << 12 | (map >> 8) << 24);
}
__host__ __device__ __forceinline__ void rect_unpack(uint2 r, uint32_t& x0, uint32_t& y0, uint32_t& x1, uint32_t& y1) {
    x0 = r.x & 0xFFFu; y0 = (r.x >> 12) & 0xFFFu; x1 = r.y & 0xFFFu; y1 = (r.y >> 12) & 0xFFFu;
}
__host__ __device__ __forceinline__ uint32_t rect_quad_map(uint2 r) { return (r.x >> 24) | (r.y >> 24) << 8; }
// Rectangles of at most 2 x 2 tiles carry their quadrant map: only their tiles with a reachable
// quadrant get an instance.  Bit 2 dy + dx of the mask: tile (x0 + dx, y0 + dy) has one.
__host__ __device__ __forceinline__ bool rect_small(uint32_t x0, uint32_t y0, uint32_t x1, uint32_t y1) {
    return x1 - x0 <= 2 && y1 - y0 <= 2;
}
__host__ __device__ __forceinline__ uint32_t rect_tile_mask(uint32_t map) {
    return ((map & 0x33u) ? 1u : 0u) | ((map & 0xCCu) ? 2u : 0u) | ((map & 0x3300u) ? 4u : 0u) |
           ((map & 0xCC00u) ? 8u : 0u);
}
// Instances a rectangle emits: its reachable tiles when small, else all its tiles.
__host__ __device__ __forceinline__ uint32_t rect_count(uint2 r) {
    uint32_t x0, y0, x1, y1;
    rect_unpack(r, x0, y0, x1, y1);
    if ((x1 - x0) * (y1 - y0) > 0 && rect_small(x0, y0, x1, y1)) return __builtin_popcount(rect_tile_mask(rect_quad_map(r)));
    return (x1 - x0) * (y1 - y0);
}
// Index of tile (tx, ty) among the rectangle's emitted instances (row-major order).
__host__ __device__ __forceinline__ uint32_t rect_local_index(uint2 r, uint32_t tx, uint32_t ty) {
    uint32_t x0, y0, x1, y1;
    rect_unpack(r, x0, y0, x1, y1);
    if (rect_small(x0, y0, x1, y1))
        return __builtin_popcount(rect_tile_mask(rect_quad_map(r)) & ((1u << (2 * (ty - y0) + (tx - x0))) - 1u));
    return (ty - y0) * (x1 - x0) + (tx - x0);
}

// One camera of a preprocess launch and its outputs.
struct PreprocessView {
    float tanfovx, tanfovy, focal_x, focal_y;
    const float* view;
    const float* proj;
    const float* campos;
    int* radii;
    int* radius;      // internal copy of radii (the backward recomputes tile rectangles)
    uint32_t* tiles;
    uint2* rect;      // tile rectangle + small-rectangle quadrant map (rect_pack); 0 when culled
    uint32_t* key;
    float2* xy;
    float4* conic_o;
    float4* rgbd;
    uint8_t* clamped;
    uint32_t* order;  // if set: order[i] = i (the depth sort's initial values)
    uint32_t* rank_counts;   // if set: zeroed (per depth rank instance counts; the sort's last
                             // pass fills the visible ranks, the culled ones stay 0)
    float4* acc;      // if set: [P, ACC_PITCH / 4] backward accumulators, zeroed for visible rows
    ClearList clear;  // zeroed on the side (sort workspace, counters)
};
// Preprocess of nv <= LSR_MAX_VIEWS cameras over the same Gaussians: with nv > 1 a Gaussian's
// inputs are read (and its cov3D built) once for all of them.
struct PreprocessArgs {
    int P, M, deg, W, H, grid_x, grid_y, nv;
    int row0;   // the launch covers Gaussians [row0, P) (a row chunk; a multiple of 256), usually 0
    int counts_tiles;   // 1: rank_counts[i] = tiles[i] (the tile-bucket binning's index-order counts)
    float scale_modifier;
    const float* means3D;
    const float* scales;
    const float* rotations;
    const float* opacities;
    const float* shs;
    const float* colors_precomp;
    const float* cov3D_precomp;
    PreprocessView v[LSR_MAX_VIEWS];
};

struct PreprocessBwdArgs {
    int P, M, deg;
    float tanfovx, tanfovy, focal_x, focal_y, scale_modifier;
    const float* means3D;
    const float* scales;
    const float* rotations;
    const float* shs;
    const float* cov3D_precomp;
    const float* view;
    const float* proj;
    const float* campos;
    const uint32_t* tiles;    // tiles touched (0 = culled; same as radii == 0)
    const uint8_t* clamped;
    // per-(Gaussian, tile) records of the compositor backward (render_bwd.hip), contiguous per
    // Gaussian from inst_off[g]; flags[e] = 1 where the record was written
    const float* rec;
    const uint8_t* flags;
    const uint32_t* inst_off;
    int recq;
    int deterministic;
    const float* acc_small;   // atomic mode: [P, ACC_PITCH] summed records
    // outputs (nullable)
    float* dopacity;
    float* dmeans3D;
    float* dmeans2D;
    float* dcolors;
    float* dcov3D;
    float* dsh;
    float* dscales;
    float* drots;
};

// Preprocess backward of several views of the same Gaussians in one pass (lsr_backward_views):
// per Gaussian, the view-independent rows (mean, scale, rotation, SH) are read once, each view's
// screen-space sums (acc_small of its compositor backward) are pushed through that view's camera,
// and the summed gradient rows are written (or accumulated) once.
struct ViewCam {
    const float* view;
    const float* proj;
    const float* campos;
    float tanfovx, tanfovy, focal_x, focal_y;
    int deg;
    const uint32_t* tiles;    // tiles touched in this view (0 = culled)
    const uint8_t* clamped;
    const float* acc_small;   // [P, ACC_PITCH] the view's summed records
};
struct PreprocessBwdViewsArgs {
    int P, M, nv;
    float scale_modifier;
    const float* means3D;
    const float* scales;
    const float* rotations;
    const float* shs;
    const float* cov3D_precomp;
    ViewCam cam[LSR_MAX_VIEWS];
    float* dopacity;
    float* dmeans3D;
    float* dmeans2D;
    float* dcolors;
    float* dcov3D;
    float* dsh;
    float* dscales;
    float* drots;
};
void launch_preprocess_bwd_views(const PreprocessBwdViewsArgs& a, bool accumulate, hipStream_t st);

void launch_language_split(int P, const float* lang, uint16_t* out, hipStream_t st);
void launch_radii_max(int P, int n, const int* const* radii, int* out, bool accumulate, hipStream_t st);

struct RenderFwdArgs {
    int W, H, grid_x, grid_y, C, include_feature;
    uint2* ranges;                // read; an empty tile's preset (~0, 0) is rewritten to (0, 0)
    const uint32_t* point_list;
    const float2* xy;
    const float4* conic_o;
    const float4* rgbd;
    const float* lang;
    const uint16_t* lang_split;   // [P][64] bf16 hi | lo (lsr_language_split; C == 32) or null
    const float* bg;
    float* final_T;
    uint32_t* n_contrib;
    uint32_t* tile_max_contrib;   // per tile: max n_contrib over its pixels (bounds the backward replay)
    uint32_t* tile_order;         // [tiles] scratch: longest-list-first launch order (null: tile order)
    float* out_color;
    float* out_lang;
    float* out_depth;
};

struct RenderBwdArgs {
    int W, H, grid_x, grid_y, C, include_feature;
    const uint2* ranges;
    const uint32_t* point_list;
    const float2* xy;
    const float4* conic_o;
    const float4* rgbd;
    const uint2* rect;        // binning rectangles (deterministic records are indexed within them)
    const uint32_t* inst_off;
    const float* lang;
    const uint16_t* lang_split;   // [P][64] bf16 hi | lo (lsr_language_split; C == 32) or null
    const float* bg;
    const float* final_T;
    const uint32_t* n_contrib;
    const uint32_t* tile_max_contrib;
    uint32_t* tile_order;     // [tiles] scratch: the wave backward's longest-first tile order
    const float* dL_dcolor;   // [3,H,W]
    const float* dL_dlang;    // [C,H,W] or null
    const float* dL_ddepth;   // [H,W] or null
    // outputs: one record of recq floats per (Gaussian, tile) instance that has a contributing pixel
    //   [0..2] dL/dcolor, [3] dL/ddepth, [4..5] dL/dmean2D (NDC), [6..8] dL/dconic (x, y, w),
    //   [9] dL/dopacity, [10..11] 0, [12..12+C) dL/dlanguage
    float* rec;
    uint8_t* flags;
    int recq;
    int deterministic;
    // default (atomic) mode: per-Gaussian accumulators
    float* acc_small;         // [P, ACC_PITCH], record layout [0..9]
    float* acc_lang;          // [P,C] (the caller's dL/dlanguage buffer), may be null
};

// The compacted-wave compositors take up to LSR_MAX_VIEWS views of one image size per launch
// (grid row = view; blocks dispatch row by row, so a view's tail waves overlap the next view's
// first ones instead of draining the chip between launches).  A single view is a batch of one.
struct RenderFwdBatch { RenderFwdArgs v[LSR_MAX_VIEWS]; };
struct RenderBwdBatch { RenderBwdArgs v[LSR_MAX_VIEWS]; };
void launch_render_fwd_views(const RenderFwdArgs* a, int n, hipStream_t st);
// non-deterministic views with C <= 32 only (the wave backward); tile orders built in one launch
void launch_render_bwd_wave_views(const RenderBwdArgs* a, int n, hipStream_t st);

// record width for C language channels (multiple of 4 floats)
inline int lang_pad(int C) { return C == 0 ? 0 : C <= 4 ? 4 : C <= 8 ? 8 : C <= 16 ? 16 : C <= 32 ? 32 : 64; }
inline int record_floats(int C) { return 12 + lang_pad(C); }

// deformation field (deform.hip; include/lsr_deform.h)
constexpr int DEF_MAX_LAYERS = 4;     // feature_out Linear layers
constexpr int DEF_HEADS = 6;          // pos, scales, rotations, opacity, shs, coff
constexpr int DEF_W2ROWS = 64;        // output rows of every head's last layer, zero padded
constexpr int DEF_LANG_MODE_PASS = 0, DEF_LANG_MODE_RESIDUAL = 1, DEF_LANG_MODE_NORESNET = 2,
              DEF_LANG_MODE_DISCRETE = 3;
struct DeformArgs {
    int P;
    int n_scales, nlayers;
    uint32_t heads;                   // bit h: head h computed
    int apply_rotation, lang_mode, lang_dim, centers, lang_in;   // lang_in: input lang channels
    const float* means3D;
    const float* time;
    const float* aabb;                // [2][3] device: xyz_max, xyz_min
    const float* planes;              // packed channel-last planes
    int64_t poff[24];                 // float offset of plane 6 s + ci
    int pw[24], ph[24];               // its width / height
    const __bf16 *wf_h[DEF_MAX_LAYERS], *wf_l[DEF_MAX_LAYERS];   // layer k: [128][K_k], K_0 = 16 n_scales
    const __bf16 *w1_h[DEF_HEADS], *w1_l[DEF_HEADS];             // [128][128]
    const __bf16 *w2_h[DEF_HEADS], *w2_l[DEF_HEADS];             // [DEF_W2ROWS][128]
    const float* b_feat[DEF_MAX_LAYERS];
    const float* b1[DEF_HEADS];
    const float* b2[DEF_HEADS];
    const float* in[5];               // means3D, scales, rotations, opacity, shs
    const float* lang;                // [P, lang_in]
    float* out[5];
    float* out_lang;                  // DISCRETE: [P, lang_dim]
    float* out_coff;                  // DISCRETE: [P, centers] or null
};
void launch_deform_fwd(const DeformArgs& a, hipStream_t st);
void launch_pack_plane(const float* src, float* dst, int H, int W, hipStream_t st);
// lsr_deform_prepare's packing jobs in one launch per PACK_MAX_JOBS (k_pack_batch)
enum PackKind { PACK_PLANE = 0, PACK_WEIGHT = 1, PACK_WEIGHT_T = 2 };
struct PackJob {
    int kind, a, b, c, d;             // PLANE: a = H * W; WEIGHT: rows, rows_pad, cols, cols_pad; T: rows, cols, k_pad, cols_pad
    uint32_t first_block;             // set by launch_pack_batch
    const float* src;
    void* hi;                         // PLANE: the float destination
    __bf16* lo;
};
constexpr int PACK_MAX_JOBS = 64;
struct PackBatch { PackJob j[PACK_MAX_JOBS]; int n; };
void launch_pack_batch(PackJob* jobs, int n, hipStream_t st);
void launch_pack_weight(const float* src, __bf16* hi, __bf16* lo, int rows, int rows_pad, int cols, int cols_pad,
                        hipStream_t st);
// transposed packing: src fp32 [rows][cols] -> hi / lo [cols_pad][k_pad] with dst[c][r] = src[r][c],
// zero for r >= rows or c >= cols
void launch_pack_weight_t(const float* src, __bf16* hi, __bf16* lo, int rows, int cols, int k_pad, int cols_pad,
                          hipStream_t st);

// deformation backward (deform.hip): phase A per 64 Gaussians (recompute, data gradients, plane
// scatter, saved activations), phase B the weight gradients as split-K A^T B products
struct DeformBwdArgs {
    DeformArgs f;                     // planes, packed weights, biases, means3D, time, aabb, lang, in[2]
    const __bf16 *wft_h[DEF_MAX_LAYERS], *wft_l[DEF_MAX_LAYERS];   // layer k transposed: [K_k pad 32][128]
    const __bf16 *w1t_h[DEF_HEADS], *w1t_l[DEF_HEADS];             // [128 in][128 out]
    const __bf16 *w2t_h[DEF_HEADS], *w2t_l[DEF_HEADS];             // [128 in][64 out, zero padded]
    const float* up[5];               // gradients of the five outputs (null: head off)
    const float* up_lang;             // DISCRETE: [P, lang_dim] or null
    const float* up_coff;             // DISCRETE: [P, centers] or null
    float* d_means3D;
    float* d_rotations;               // apply_rotation: [P, 4]
    float* d_lang;                    // DISCRETE: [P, lang_in]
    float* dplanes;                   // packed channel-last gradient planes (same offsets as f.planes),
    int64_t plane_stride;             //   `replicas` copies plane_stride floats apart (block b adds
    int replicas;                     //   into copy b % replicas; the unpack sums them)
    // time planes (xt, yt, zt) of waves whose Gaussians all have time[0] (the render path's one time
    // per view): every tap lies in the rows y0, y1 of time[0] with weights 1 - fy, fy, so the wave adds
    // dv (1 - fx), dv fx into one x-row [W][16] per plane (at trow + toff[pi], copy b % trow_reps),
    // and the unpack adds (1 - fy) and fy times its sum into the two rows.  Null: off.
    float* trow;
    int64_t toff[24];
    int64_t trow_stride;
    int trow_reps;
    float* sX;                        // saved [P, 16 n_scales] features
    float* sA[DEF_MAX_LAYERS];        // saved [P,128] relu(H_k)
    float* sdH[DEF_MAX_LAYERS];       // saved [P,128] gradients of H_k
    float* sG_rot;                    // apply_rotation: [P,4] gradient of the rotation head's output
    float* sG_coff;                   // DISCRETE: [P, centers] gradient of coff
    float* daabb;                     // [2][3] gradient of the HexPlane box (accumulated), or null;
                                      //   phase A adds into DEF_AABB_SLOTS partial rows of daabb_part
                                      //   (block b: row b % slots, 64 B apart), the unpack sums them
    float* daabb_part;
};
constexpr int DEF_AABB_SLOTS = 64;
void launch_deform_bwd_a(const DeformBwdArgs& a, hipStream_t st);
// Weight gradients of the computed heads by recompute (deform.hip k_head_wgrad): per head and block
// of rows, from the saved last trunk activation A and the head's output gradient G,
// Z1 = A W1^T + b1, dZ1 = (G W2) [Z1 > 0]; dW1 += dZ1^T A, db1 += sum dZ1, dW2 += G^T relu(Z1),
// db2 += sum G.  One launch for every head (grid row = job).
struct HeadWgradJob {
    const float* G;                   // [P][nout]
    const __bf16 *w1_h, *w1_l;        // forward pack [128][128]
    const float* b1;
    const __bf16 *w2t_h, *w2t_l;      // backward pack [128][64] (W2 transposed, K padded to 64)
    const __bf16 *w2_h, *w2_l;        // forward pack [64 pad][128] (the VALU path of nout <= 4)
    float *dW1, *db1, *dW2, *db2;     // accumulated
    int nout;
};
constexpr int DEF_WGRAD_MAX_JOBS = DEF_HEADS;
struct HeadWgradArgs {
    HeadWgradJob job[DEF_WGRAD_MAX_JOBS];
    const float* A;                   // [P][128] the trunk's last activation (phase A saved it)
    int P, rows_per_block;            // rows_per_block: set per launch by launch_head_wgrad
};
void launch_head_wgrad(const HeadWgradArgs& a, int njobs, hipStream_t st);
struct AtbJob {                        // C[M][N] += sum_g L[g][m] R[g][n]; bias[m] += sum_g L[g][m]
    const float* L;
    const float* R;
    float* C;
    float* bias;
    int M, N;
};
constexpr int LSR_ATB_MAX_JOBS = 20;
struct AtbArgs {
    AtbJob job[LSR_ATB_MAX_JOBS];
    int P;
    int rows_per_block;
};
void launch_atb(const AtbArgs& a, int njobs, hipStream_t st);
// Every gradient plane of a call in one launch: plane j's packed replicas at src + off[j] (floats)
// summed and added into dst[j] ([16][H][W]); with daabb set, the last block also adds the
// DEF_AABB_SLOTS partial rows of daabb_part into daabb.
constexpr int DEF_UNPACK_MAX = 24;   // 6 planes x LSR_DEFORM_MAX_SCALES
struct UnpackBatch {
    const float* src;
    int64_t off[DEF_UNPACK_MAX];
    float* dst[DEF_UNPACK_MAX];
    int H[DEF_UNPACK_MAX], W[DEF_UNPACK_MAX];
    int block0[DEF_UNPACK_MAX + 1];   // first block of plane j; block0[n] = the planes' blocks
    int n, replicas;
    int64_t stride;
    const float* daabb_part;
    float* daabb;
    // DeformBwdArgs.trow: plane j's x-row copies at trow + toff[j] (toff[j] < 0: none), folded into
    // its rows of time time0[0]
    const float* trow;
    int64_t toff[DEF_UNPACK_MAX];
    int64_t trow_stride;
    int trow_reps;
    const float* time0;
};
void launch_unpack_planes(const UnpackBatch& u, hipStream_t st);

// lang_deform (RESIDUAL / NORESNET): relu([lang, poc_fre(t)]) -> Linear, ReLU, Linear, ReLU, Linear,
// (+ lang), normalised.  Separate kernels: the MLP reads only the language rows and the time.
struct LangDeformArgs {
    int P, lang_dim, time_pe, kin, residual;   // kin = lang_dim + 1 + 2 time_pe
    const float* lang;                // [P, lang_dim]
    const float* time;
    const __bf16 *w_h[3], *w_l[3];    // [128][kpad], [128][128], [32][128] (rows past lang_dim zero)
    const float* b[3];
    float* out_lang;
    // backward only
    const __bf16 *wt_h[3], *wt_l[3];  // transposed: [kpad 32][128], [128][128], [128][32]
    const float* up_lang;             // [P, lang_dim] or null
    float* d_lang;                    // [P, lang_dim]
    float *sU0, *sU1, *sU2;           // saved [P, kin], [P,128], [P,128]
    float *sdv, *sdZ2, *sdZ1;         // saved [P, lang_dim], [P,128], [P,128]
};
void launch_lang_deform_fwd(const LangDeformArgs& a, hipStream_t st);
void launch_lang_deform_bwd(const LangDeformArgs& a, hipStream_t st);

void launch_preprocess(const PreprocessArgs& a, hipStream_t st);
void launch_preprocess_bwd(const PreprocessBwdArgs& a, bool accumulate, hipStream_t st);
void launch_reduce_lang(int P, int C, int cpad, int recq, const float* rec, const uint8_t* flags,
                        const uint32_t* inst_off, const uint32_t* tiles, float* dlang, bool accumulate, hipStream_t st);
void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t st);

// device-wide primitives (sort.hip)
size_t scan_temp_bytes(size_t n);
// exclusive scan of n u32 values; writes the total to *total (device) if non-null
void exclusive_scan_u32(const uint32_t* in, uint32_t* out, size_t n, uint32_t* total, void* temp, hipStream_t st);
// Exclusive scans of a batch of independent segments (in, out, n; total and the scan workspace
// scan_temp_bytes(n) as for exclusive_scan_u32): two launches for all segments of 2K..8M values.
constexpr int SCAN_SEG_TILES = 4096;
struct ScanSeg {
    const uint32_t* in;
    uint32_t* out;
    uint32_t* total;
    uint32_t* partials;   // the segment's scan workspace
    size_t n;
    // optional: host-mapped pinned word the scan writes the total to itself (no copy launch)
    uint32_t* host_total = nullptr;
};
struct ScanBatch { ScanSeg s[LSR_MAX_VIEWS]; };
// Returns the segments (bit i = segs[i]) whose host_total the scan wrote; the caller copies the
// others' totals itself (single-tile segments and those beyond 8M values take another path).
uint32_t exclusive_scan_batch(const ScanSeg* segs, int nseg, hipStream_t st);
size_t radix_temp_bytes(size_t n);
// stable LSD sort of (key, value) pairs on bits [begin_bit, end_bit); returns true when the result
// is in (keys_b, vals_b).  Every word of temp it reads it has written (no zeroing needed).
// kept (device word, may be null): the first pass drops every key equal to 0xFFFFFFFF and writes
// the number of kept keys here; the later passes sort only those, so the output holds the kept
// pairs in [0, *kept) (the rest of the buffers is left as it was).
// gather (may be null): the last pass also writes, per output position, rect_sorted = rect[value]
// and counts = rect_count of it, and not the keys.
struct SortGather {
    const uint2* rect;
    uint32_t* counts;
    uint2* rect_sorted;
};
// One sort of a batch: its own arrays, workspace (radix_temp_bytes(n)), optional kept count (the
// first pass drops 0xFFFFFFFF keys and counts the rest there) and last-pass gather.
struct SortSeg {
    uint32_t *keys_a, *vals_a, *keys_b, *vals_b;
    void* temp;
    uint32_t* kept;
    SortGather gather;
    size_t n;
    // tile sort: the per-key [start, end) ranges, made by the last pass's scatter (atomicMin /
    // atomicMax at the key runs' ends; entries preset to (0xFFFFFFFF, 0), keys >= nranges skipped)
    uint2* ranges;
    uint32_t nranges;
    // depth sort (with kept and gather): [n] scratch for the values of the device-planned middle
    // pass (sort.hip); set, the batch's passes are planned on the device (every segment sets it)
    uint32_t* vals_c;
};
struct SortBatch { SortSeg s[LSR_MAX_VIEWS]; };
// Sorts up to LSR_MAX_VIEWS independent segments with one launch per kernel of each pass (every
// segment the same key bits); returns whether the results are in the (b) buffers.
// 0: the result is in the (a) buffers, 1: in (b); -1: a batch mixing device-planned (vals_c) and
// host-planned segments, or a planned sort over other than bits [0, 32) (nothing launched)
int radix_sort_batch(const SortSeg* segs, int nseg, int begin_bit, int end_bit, hipStream_t st);
bool radix_sort_pairs(uint32_t* keys_a, uint32_t* vals_a, uint32_t* keys_b, uint32_t* vals_b, size_t n,
                      int begin_bit, int end_bit, void* temp, hipStream_t st, uint32_t* kept = nullptr,
                      const SortGather* gather = nullptr, uint32_t* vals_c = nullptr);

// binning (binning.hip)
// Point-list values: Gaussian id in the low 28 bits, in the top 4 the quadrants (bit 28 + q,
// q = (y >= 8) * 2 + (x >= 8) inside the 16x16 tile) the splat may reach (quad_may_touch); an
// instance reaching none gets key 0xFFFFFFFF, dropped by the tile sort's first pass.
constexpr uint32_t PL_ID_MASK = 0x0FFFFFFFu;
constexpr int PL_QUAD_SHIFT = 28;
// Instance emission of nv <= LSR_MAX_VIEWS views (one grid row per view; same P and tile grid).
struct EmitView {
    const uint32_t* order;       // depth-ranked ids
    const uint32_t* offsets;     // first instance slot per depth rank
    const uint32_t* counts;      // instances per depth rank
    const uint2* rect_sorted;    // rectangles per depth rank
    const float2* xy;
    const float4* conic_o;
    uint32_t* keys;
    uint32_t* vals;
    ClearList clear;
};
struct EmitBatch {
    int P, grid_x, grid_y, W, H;
    EmitView v[LSR_MAX_VIEWS];
};
void launch_emit_instances(const EmitBatch& eb, int nv, hipStream_t st);
void launch_scatter_inst_off(int P, const uint32_t* order, const uint32_t* offsets, const uint32_t* counts,
                             uint32_t* inst_off, hipStream_t st);
// Tile-bucket binning (tilebin.hip): the instances of Gaussians in index order go straight to their
// tile's bucket; each bucket is sorted by (depth, id) in LDS.  One grid row per view.
struct TbView {
    const uint32_t* counts;    // [P] instances per Gaussian (index order)
    const uint32_t* offsets;   // [P] their exclusive scan
    const uint2* rect;         // [P] binning rectangles by id
    const float2* xy;
    const float4* conic_o;
    const uint32_t* depth;     // [P] depth key bits by id
    uint32_t* table;           // [tb_blocks(P), ntiles] per-block tile counts, then their column scans
    uint32_t* tile_total;      // [ntiles]
    uint32_t* tile_start;      // [ntiles] (may alias tile_max: the sort zeroes it after the scatter)
    uint2* ranges;             // [ntiles] (empty tiles: (0, 0))
    uint64_t* keys;            // [K] depth bits << 32 | id << 4 | quadrant bits, bucketed by tile
    uint64_t* tmp;             // [K] merge workspace of buckets longer than one LDS sort
    uint32_t* words;           // [K] the point list (id | quadrant bits << PL_QUAD_SHIFT)
    uint32_t* tile_max;        // [ntiles] zeroed
};
struct TbBatch {
    int P, grid_x, grid_y, W, H, ntiles;
    TbView v[LSR_MAX_VIEWS];
};
int tb_blocks(int P);   // rows of TbView::table
hipError_t launch_tile_bucket_binning(const TbBatch& tb, int nv, hipStream_t st);   // attribute errors returned

// compositing (render_fwd_wave.hip / render_bwd.hip)
void launch_render_bwd(const RenderBwdArgs& a, hipStream_t st);
void launch_render_fwd_wave_views(const RenderFwdArgs* a, int n, hipStream_t st);
void launch_render_fwd_wave_mfma_views(const RenderFwdArgs* a, int n, hipStream_t st);   // 17..32 channels

}  // namespace lsr
