/*
 * lsr_deform.h -- C ABI of the MI355X-native 4D deformation field (HexPlane + MLP heads), part of
 * liblsr.so.  Produces the rasterizer's per-frame inputs.
 *
 * Reference behaviour replaced:
 *   deform_network.forward_dynamic            scene/deformation.py:232-248, poc_fre :261-267
 *   Deformation.create_net / query_time       scene/deformation.py:45-86 (feature_out: max(defor_depth,
 *                                             1) Linear layers, ReLU between them)
 *   Deformation.forward_dynamic               scene/deformation.py:103-182: the residual heads
 *                                             (each can be off: no_dx / no_ds / no_dr / no_do /
 *                                             no_dshs), apply_rotation (batch_quaternion_multiply,
 *                                             utils/graphics_utils.py:109-132), and the language
 *                                             modes below
 *   HexPlaneField.forward / get_density       scene/hexplane.py:160-185
 *   interpolate_ms_features, grid_sample_wrapper (bilinear, align_corners=True, border)
 *                                             scene/hexplane.py:21-106
 * Outputs, per Gaussian (raw values, before activation):
 *   means3D + d_pos,  scales + d_scales,  rotations + d_rot (or normalize(rotations (x) d_rot)),
 *   opacity + d_opacity,  shs + d_shs,  language (mode), coff (discrete mode)
 * Language modes (the reference's no_dlang flag and env vars use_discrete_lang_f / no_resnet):
 *   PASS      the first lang_dim channels of the input                      (:169-170)
 *   RESIDUAL  normalize(lang + lang_deform(relu([lang, poc_fre(t, time_pe)])))  (:172-180)
 *   NORESNET  normalize(lang_deform(...))                                    (:176-177)
 *   DISCRETE  the input holds `centers` centres of lang_dim channels; each is normalised, combined
 *             with coff = discrete_coff_generator(hidden), and the sum normalised   (:156-163)
 * Not supported (rejected): no_grid, grid_pe > 0, static_mlp, empty_voxel, use_tribute_dlang (off
 * in every reference config), channels != 16, width != 128.
 *
 * Conventions: device pointers, float32, contiguous, torch layouts (planes [1, C, res[c1],
 * res[c0]] for the coordinate pair (c0, c1) in the order xy, xz, xt, yz, yt, zt; Linear weights
 * [out, in]).  All launches on `stream`.  Return 0 or an LSR_E* code (lsr.h); lsr_last_error().
 */
#ifndef LSR_DEFORM_H_
#define LSR_DEFORM_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define LSR_DEFORM_API_VERSION 3   /* 2: depth, head mask, apply_rotation, language modes, coff; 3: aabb gradient */
#define LSR_DEFORM_HEADS 6         /* pos 3, scales 3, rotations 4, opacity 1, shs 48, coff (centers) */
#define LSR_DEFORM_MAX_SCALES 4
#define LSR_DEFORM_MAX_DEPTH 4     /* feature_out Linear layers */
#define LSR_DEFORM_LANG_PASS 0
#define LSR_DEFORM_LANG_RESIDUAL 1
#define LSR_DEFORM_LANG_NORESNET 2
#define LSR_DEFORM_LANG_DISCRETE 3

typedef struct lsr_deform_net {
    int32_t n_scales;                   /* multires levels (Neu3D: 2, HyperNeRF: 3) */
    int32_t channels;                   /* plane channels per scale (output_coordinate_dim); 16 */
    int32_t width;                      /* MLP width (net_width); 128 */
    int32_t res[4];                     /* base plane resolution x, y, z, t */
    int32_t multires[LSR_DEFORM_MAX_SCALES];   /* spatial multiplier of each scale (time unscaled) */
    int32_t depth;                      /* defor_depth: feature_out has max(depth, 1) Linear layers */
    uint32_t heads;                     /* bit h: head h computed (bits 0-4 = !no_dx, !no_ds, !no_dr,
                                           !no_do, !no_dshs; bit 5 set iff lang_mode == DISCRETE) */
    int32_t apply_rotation;             /* rotations = normalize(rotations (x) d_rot) */
    int32_t lang_mode;                  /* LSR_DEFORM_LANG_* */
    int32_t lang_dim;                   /* language channels out (language_feature_hiddendim), <= 32 */
    int32_t centers;                    /* DISCRETE: centres (centers_num), <= 8; else 0 */
    int32_t time_pe;                    /* timebase_pe: lang_deform input 2 time_pe + 1 + lang_dim <= 64 */
    const float *aabb;                  /* [2][3]: xyz_max, xyz_min (HexPlaneField.aabb order) */
    const float *planes[LSR_DEFORM_MAX_SCALES][6];
    const float *w_feat[LSR_DEFORM_MAX_DEPTH], *b_feat[LSR_DEFORM_MAX_DEPTH];   /* feature_out.{2k} */
    const float *w1[LSR_DEFORM_HEADS], *b1[LSR_DEFORM_HEADS];   /* {head}.1: [width, width] */
    const float *w2[LSR_DEFORM_HEADS], *b2[LSR_DEFORM_HEADS];   /* {head}.3: [out, width] */
    const float *w_lang[3], *b_lang[3]; /* lang_deform.{1,3,5} (RESIDUAL / NORESNET) */
} lsr_deform_net;

/* Call once before any other lsr_deform_* entry point with LSR_DEFORM_API_VERSION from the
 * lsr_deform.h the caller was built against: lsr_deform_net / lsr_deform_grads are read with THIS
 * header's layout (version 3 added lsr_deform_grads.aabb), so a caller of another version is refused
 * (LSR_EINVAL, every entry point) instead of having its structs misread. */
int lsr_deform_require_api(int32_t caller_version);

/* Workspace holding the packed planes (channel-last) and weights (bf16 hi/lo).  -1: bad net. */
int64_t lsr_deform_workspace_bytes(const lsr_deform_net *net);
/* Pack the parameters into the workspace; call again after every parameter update. */
int lsr_deform_prepare(const lsr_deform_net *net, void *workspace, void *stream);
/* Deform P Gaussians at times time[P].  lang: [P, lang_dim * centers] in DISCRETE mode, else
 * [P, lang_dim] (may be NULL in PASS mode).  The output of a head that is off is not written (the
 * value is the input; its pointer may be NULL); out_lang is written unless PASS (the value is then
 * the input's first lang_dim channels), out_coff in DISCRETE mode (may be NULL).  Outputs alias
 * nothing of the inputs. */
int lsr_deform_forward(const lsr_deform_net *net, const void *workspace, int32_t P, const float *means3D,
                       const float *scales, const float *rotations, const float *opacity, const float *shs,
                       const float *lang, const float *time, float *out_means3D, float *out_scales,
                       float *out_rotations, float *out_opacity, float *out_shs, float *out_lang,
                       float *out_coff, void *stream);

/* Parameter gradients of the field, torch layouts (planes [C, H, W] as the planes themselves).
 * Pointers of parameters the net does not use are ignored. */
typedef struct lsr_deform_grads {
    float *planes[LSR_DEFORM_MAX_SCALES][6];
    float *w_feat[LSR_DEFORM_MAX_DEPTH], *b_feat[LSR_DEFORM_MAX_DEPTH];
    float *w1[LSR_DEFORM_HEADS], *b1[LSR_DEFORM_HEADS];
    float *w2[LSR_DEFORM_HEADS], *b2[LSR_DEFORM_HEADS];
    float *w_lang[3], *b_lang[3];
    /* [2][3] gradient of HexPlaneField.aabb (xyz_max, xyz_min), accumulated; NULL: not computed.  The
     * reference trains the box whenever the whole field has requires_grad (the base stages and
     * joint_train: scene/gaussian_model.py:258,291 requires_grad_(True) reaches the aabb Parameter
     * that set_aabb made with requires_grad=False, and get_grid_parameters hands "grid.aabb" to Adam). */
    float *aabb;
} lsr_deform_grads;

/* Scratch of lsr_deform_backward for P Gaussians (saved activations). */
int64_t lsr_deform_backward_scratch_bytes(const lsr_deform_net *net, int32_t P);

/* Backward of lsr_deform_forward (what autograd does through deform_network.forward_dynamic and
 * HexPlaneField, scene/deformation.py:103-182, scene/hexplane.py:21-106), given the gradients of
 * its outputs d_out_* (same shapes as the outputs; NULL for a head that is off, d_out_lang /
 * d_out_coff NULL = zero):
 *   d_means3D = d_out_means3D + the gradient through the HexPlane sample coordinates (written);
 *   d_rotations (apply_rotation only; written) = the quaternion product's gradient, else the
 *     rotation input gradient is d_out_rotations (identity residual) and is not written;
 *   d_lang [P, lang_in] (written unless PASS, whose input gradient is d_out_lang itself);
 *   the scales / opacity / SH input gradients equal d_out_* (identity residuals): not written;
 *   every parameter gradient in `grads` is ACCUMULATED (+=), as torch accumulates .grad.
 * `workspace` is the prepared forward workspace (its packing must match the current parameters).
 * Float atomics (plane scatter, weight-gradient partials): not bitwise reproducible. */
int lsr_deform_backward(const lsr_deform_net *net, const void *workspace, int32_t P, const float *means3D,
                        const float *rotations, const float *lang, const float *time, const float *d_out_means3D,
                        const float *d_out_scales, const float *d_out_rotations, const float *d_out_opacity,
                        const float *d_out_shs, const float *d_out_lang, const float *d_out_coff, float *d_means3D,
                        float *d_rotations, float *d_lang, const lsr_deform_grads *grads, void *scratch,
                        void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LSR_DEFORM_H_ */
