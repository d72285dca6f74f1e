/*
 * lsr_deform.h -- C ABI of the MI355X-native 4D deformation field (HexPlane + MLP heads), part of
 * liblsr.so.  Produces the rasterizer's per-frame inputs.
 *
 * Reference behaviour replaced (Neu3D structure, arguments/neu3d/default.py):
 *   deform_network.forward_dynamic            scene/deformation.py:232-248
 *   Deformation.forward_dynamic / query_time  scene/deformation.py:76-182 (defor_depth 0: one
 *                                             Linear feature_out; language pass-through)
 *   HexPlaneField.forward / get_density       scene/hexplane.py:160-185
 *   interpolate_ms_features, grid_sample_wrapper (bilinear, align_corners=True, border)
 *                                             scene/hexplane.py:21-106
 * Outputs, per Gaussian:  means3D + d_pos,  scales + d_scales,  rotations + d_rot,
 *                         opacity + d_opacity,  shs + d_shs      (raw values, before activation)
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

#define LSR_DEFORM_HEADS 5      /* pos 3, scales 3, rotations 4, opacity 1, shs 48 */
#define LSR_DEFORM_MAX_SCALES 4

typedef struct lsr_deform_net {
    int32_t n_scales;                   /* multires levels (Neu3D: 2) */
    int32_t channels;                   /* plane channels per scale (output_coordinate_dim); 16 */
    int32_t width;                      /* MLP width (net_width); 128 */
    int32_t res[4];                     /* base plane resolution x, y, z, t */
    int32_t multires[LSR_DEFORM_MAX_SCALES];   /* spatial multiplier of each scale (time unscaled) */
    const float *aabb;                  /* [2][3]: xyz_max, xyz_min (HexPlaneField.aabb order) */
    const float *planes[LSR_DEFORM_MAX_SCALES][6];
    const float *w_feat, *b_feat;       /* feature_out.0: [width, n_scales * channels], [width] */
    const float *w1[LSR_DEFORM_HEADS], *b1[LSR_DEFORM_HEADS];   /* {head}.1: [width, width], [width] */
    const float *w2[LSR_DEFORM_HEADS], *b2[LSR_DEFORM_HEADS];   /* {head}.3: [out, width], [out] */
} lsr_deform_net;

/* Workspace holding the packed planes (channel-last) and weights (bf16 hi/lo). */
int64_t lsr_deform_workspace_bytes(const lsr_deform_net *net);
/* Pack the parameters into the workspace; call again after every parameter update. */
int lsr_deform_prepare(const lsr_deform_net *net, void *workspace, void *stream);
/* Deform P Gaussians at times time[P].  Outputs may alias nothing of the inputs. */
int lsr_deform_forward(const lsr_deform_net *net, const void *workspace, int32_t P, const float *means3D,
                       const float *scales, const float *rotations, const float *opacity, const float *shs,
                       const float *time, float *out_means3D, float *out_scales, float *out_rotations,
                       float *out_opacity, float *out_shs, void *stream);

/* Parameter gradients of the field, torch layouts (planes [C, H, W] as the planes themselves). */
typedef struct lsr_deform_grads {
    float *planes[LSR_DEFORM_MAX_SCALES][6];
    float *w_feat, *b_feat;
    float *w1[LSR_DEFORM_HEADS], *b1[LSR_DEFORM_HEADS];
    float *w2[LSR_DEFORM_HEADS], *b2[LSR_DEFORM_HEADS];
} lsr_deform_grads;

/* Scratch of lsr_deform_backward for P Gaussians (saved activations: 6272 bytes per Gaussian). */
int64_t lsr_deform_backward_scratch_bytes(const lsr_deform_net *net, int32_t P);

/* Backward of lsr_deform_forward (what autograd does through deform_network.forward_dynamic and
 * HexPlaneField, scene/deformation.py:103-182, scene/hexplane.py:21-106), given the gradients of
 * its five outputs d_out_* (same shapes as the outputs):
 *   d_means3D = d_out_means3D + the gradient through the HexPlane sample coordinates (overwritten);
 *   the scales / rotations / opacity / SH input gradients equal d_out_* (identity residuals), so
 *   they are not written here;
 *   every parameter gradient in `grads` is ACCUMULATED (+=), as torch accumulates .grad.
 * `workspace` is the prepared forward workspace (its packing must match the current parameters).
 * Float atomics (plane scatter, weight-gradient partials): not bitwise reproducible. */
int lsr_deform_backward(const lsr_deform_net *net, const void *workspace, int32_t P, const float *means3D,
                        const float *time, const float *d_out_means3D, const float *d_out_scales,
                        const float *d_out_rotations, const float *d_out_opacity, const float *d_out_shs,
                        float *d_means3D, const lsr_deform_grads *grads, void *scratch, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LSR_DEFORM_H_ */
