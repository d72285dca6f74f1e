/*
 * lsr_train.h -- C ABI of the MI355X-native training-step glue, part of liblsr.so (SURVEY.md 8f
 * row 4): the optimizer step over the Gaussian SoA, the densification statistics, and the
 * densify / prune / opacity-reset row surgery of scene/gaussian_model.py.
 *
 * Reference interfaces these replace:
 *   - torch.optim.Adam(groups, lr=0.0, eps=1e-15).step()   scene/gaussian_model.py:301, train.py:420
 *       -> lsr_adam_step (one launch over every parameter group)
 *   - max_radii2D[vis] = max(max_radii2D[vis], radii[vis]);
 *     add_densification_stats(viewspace_grad, vis)        train.py:388-389, gaussian_model.py:746-748
 *       -> lsr_densify_stats
 *   - densify = densify_and_clone + densify_and_split      gaussian_model.py:726-731, 607-627, 575-605
 *       -> lsr_densify_plan (+ lsr_gather_rows, lsr_split_fixup)
 *   - prune                                                gaussian_model.py:714-723, 487-508
 *       -> lsr_prune_plan (+ lsr_gather_rows)
 *   - reset_opacity                                        gaussian_model.py:391-394, 446-459
 *       -> lsr_reset_opacity
 *   - exp / normalize / sigmoid of the render path          gaussian_renderer/__init__.py:191-193
 *       -> lsr_activate, lsr_activate_backward
 *   - the base stages' L1 image loss                         train.py:272-276
 *       -> lsr_l1_loss_views, lsr_l1_loss_views_backward
 *
 * Conventions as lsr.h: device pointers, float32 unless stated, contiguous rows; the library
 * allocates nothing (plans take a workspace of lsr_train_workspace_bytes(P)); every launch on
 * `stream`; no host synchronisation (the plans leave their row counts in device memory, the
 * caller reads them to size the new tensors, as upstream's boolean indexing does).
 * Return 0 or an LSR_E* code (lsr.h); lsr_last_error().
 */
#ifndef LSR_TRAIN_H_
#define LSR_TRAIN_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

#define LSR_ADAM_MAX_GROUPS 16

/* One parameter group of torch.optim.Adam (one tensor each, as gaussian_model.py:238-288). */
typedef struct lsr_adam_group {
    float *param;
    const float *grad;     /* NULL: the group is skipped (torch skips params whose .grad is None) */
    float *exp_avg;
    float *exp_avg_sq;
    int64_t n;             /* floats */
    double lr;
    int64_t step;          /* the group's step count including this update (1 on the first) */
} lsr_adam_group;

/* torch.optim.Adam (amsgrad = False, weight_decay = 0, maximize = False), per element:
 *   m = lerp(m, g, 1 - beta1);  v = v * beta2 + (1 - beta2) * g * g
 *   p -= lr / (1 - beta1^step) * m / (sqrt(v) / sqrt(1 - beta2^step) + eps)
 * with the bias corrections and step size computed in double on the host (as torch does with
 * Python floats) and the element arithmetic in float32.  All groups in one launch. */
int lsr_adam_step(const lsr_adam_group *groups, int32_t n_groups, double beta1, double beta2, double eps,
                  void *stream);

/* Densification statistics of one training iteration, for the Gaussians with radii[i] > 0
 * (radii = max over the iteration's views, train.py:266):
 *   max_radii2D[i] = max(max_radii2D[i], radii[i])
 *   xyz_gradient_accum[i] += |(g[i,0], g[i,1])|   (g = viewspace_point_tensor grad summed over views)
 *   denom[i] += 1
 * means2D_grad rows are grad_stride floats apart (3 for the [P,3] screen-space tensor). */
int lsr_densify_stats(int32_t P, const int32_t *radii, const float *means2D_grad, int32_t grad_stride,
                      float *max_radii2D, float *xyz_gradient_accum, float *denom, void *stream);

int64_t lsr_train_workspace_bytes(int32_t P);

/* Row map of densify (clone, then split into n_copies; the reference's N = 2):
 *   g[i] = xyz_gradient_accum[i] / denom[i]  (NaN -> 0)
 *   s[i] = max_k exp(scaling[i,k])            (raw log-scales, [P,3])
 *   clone[i] = |g[i]| >= grad_threshold and s[i] <= percent_dense * extent
 *   split[i] =  g[i]  >= grad_threshold and s[i] >  percent_dense * extent
 * Output row j of the densified model takes source row index[j]:
 *   [ rows not split, in order | cloned rows, in order | split rows, copy 0 | ... | copy n_copies-1 ]
 * which is the order the reference's cat-then-prune produces.  index holds at least
 * (n_copies + 1) * P int32; counts (device int64[3]) = {rows not split, cloned, split}. */
int lsr_densify_plan(int32_t P, const float *xyz_gradient_accum, const float *denom, const float *scaling,
                     float grad_threshold, float percent_dense, float extent, int32_t n_copies, int32_t *index,
                     int64_t *counts, void *workspace, void *stream);

/* Row map of prune: prune[i] = sigmoid(opacity[i]) < min_opacity, or, when max_screen_size > 0,
 * max_radii2D[i] > max_screen_size or max_k exp(scaling[i,k]) > 0.1 * extent.
 * index[0 .. counts[0]) = the kept rows in order; counts (device int64[1]). */
int lsr_prune_plan(int32_t P, const float *opacity, const float *max_radii2D, const float *scaling,
                   float min_opacity, float max_screen_size, float extent, int32_t *index, int64_t *counts,
                   void *workspace, void *stream);

/* One tensor of the row surgery: dst row j = src row index[j] for j < zero_from, and zeros for
 * j >= zero_from (the optimizer moments of appended rows).  row_bytes is any positive size. */
typedef struct lsr_row_tensor {
    const void *src;
    void *dst;
    int64_t row_bytes;
    int64_t zero_from;
} lsr_row_tensor;
#define LSR_GATHER_MAX_TENSORS 32
/* Every tensor in one launch (n_tensors <= LSR_GATHER_MAX_TENSORS); src and dst must not overlap. */
int lsr_gather_rows(int32_t n_tensors, const lsr_row_tensor *t, const int32_t *index, int64_t n_rows, void *stream);

/* The new rows of a split (gaussian_model.py:587-593), rows base .. base + n_new of the gathered
 * model (copy c of split row k is row base + c * n_split + k, n_new = n_copies * n_split):
 *   xyz[j]     = R(rotation[index[j]]) (exp(scaling[index[j]]) * sample[j - base]) + xyz[index[j]]
 *   scaling[j] = log(exp(scaling[index[j]]) / (0.8 n_copies))
 * R = build_rotation of the normalised quaternion (utils/general_utils.py:84-110); samples are
 * standard-normal [n_new, 3] draws (the reference's torch.normal(0, std) = std * z). */
int lsr_split_fixup(int64_t n_new, int64_t base, int32_t n_copies, const int32_t *index, const float *xyz_src,
                    const float *scaling_src, const float *rotation_src, const float *samples, float *xyz_dst,
                    float *scaling_dst, void *stream);

/* opacity = inverse_sigmoid(min(sigmoid(opacity), 0.01)); its Adam moments zeroed (exp_avg and
 * exp_avg_sq may be NULL). */
int lsr_reset_opacity(int32_t P, float *opacity, float *exp_avg, float *exp_avg_sq, void *stream);

/* render_views' V views of P Gaussians (gaussian_scene.py), every tensor in one launch (t[k].src /
 * dst / row_bytes, rows of whole floats; zero_from unused):
 *   lsr_repeat_rows:    dst row j = src row j mod n_rows, j < n_blocks * n_rows  (torch.Tensor.repeat)
 *   lsr_sum_row_blocks: dst row j = sum over b < n_blocks of src row b * n_rows + j, in b order (its
 *                       backward; torch sums two blocks the same way) */
int lsr_repeat_rows(int32_t n_tensors, const lsr_row_tensor *t, int64_t n_rows, int32_t n_blocks, void *stream);
int lsr_sum_row_blocks(int32_t n_tensors, const lsr_row_tensor *t, int64_t n_rows, int32_t n_blocks, void *stream);

/* The base stages' image loss (train.py:272-276: l1_loss(cat(images), cat(gts)[:, :3]) = mean |x - y|)
 * over V <= 8 views without stacking them: images[v] [n] floats (one [3,H,W] render), the view's
 * gt at gt + v * gt_view_stride (its first n floats: gts[v, :3]).  loss: one device float,
 * sum * (1 / (V n)), the partial sums added in a fixed order (deterministic; not PyTorch's order);
 * workspace >= lsr_l1_workspace_bytes(V).  The backward writes d_images[v] = sign(x - y) * (d_loss * (1 / (V n))),
 * PyTorch's abs / mean backward bit for bit. */
int64_t lsr_l1_workspace_bytes(int32_t V);
int lsr_l1_loss_views(int32_t V, int64_t n, const float *const *images, const float *gt, int64_t gt_view_stride,
                      float *loss, void *workspace, void *stream);
int lsr_l1_loss_views_backward(int32_t V, int64_t n, const float *const *images, const float *gt,
                               int64_t gt_view_stride, const float *d_loss, float *const *d_images, void *stream);

/* The render path's activations over P rows in one launch (gaussian_renderer/__init__.py:191-193,
 * gaussian_model.py:38-46; replaces torch.exp / torch.nn.functional.normalize / torch.sigmoid and
 * their autograd backward there, GaussianScene.render_views):
 *   scales = exp(raw_scales) [P,3];  rotations = raw / max(|raw|, 1e-12) [P,4];  opacity = sigmoid(raw) [P]
 * Any raw input may be NULL (that output is skipped); rotation rows 16-byte aligned. */
int lsr_activate(int32_t P, const float *raw_scales, const float *raw_rotations, const float *raw_opacity,
                 float *scales, float *rotations, float *opacity, void *stream);
/* Their backward from the forward's outputs (scales, opacity) and the raw rotations:
 *   d_raw_scales = d_scales * scales;  d_raw_opacity = d_opacity * opacity * (1 - opacity);
 *   d_raw_rotations = (d - y (y . d)) / |raw| with y = raw / |raw| (d / 1e-12 when |raw| <= 1e-12).
 * A NULL upstream gradient counts as zero; a NULL output gradient is not computed. */
int lsr_activate_backward(int32_t P, const float *scales, const float *raw_rotations, const float *opacity,
                          const float *d_scales, const float *d_rotations, const float *d_opacity,
                          float *d_raw_scales, float *d_raw_rotations, float *d_raw_opacity, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LSR_TRAIN_H_ */
