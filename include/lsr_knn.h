/*
 * lsr_knn.h -- C ABI of the MI355X-native mean nearest-neighbour distance, part of liblsr.so
 * (SURVEY.md 8f row 3).  Replaces simple_knn._C.distCUDA2, the un-vendored submodule
 * submodules/simple-knn (/root/reference/.gitmodules:1-3), called once at scene initialisation:
 *   dist2 = torch.clamp_min(distCUDA2(points), 1e-7)      scene/gaussian_model.py:22,203-204
 *   scales = log(sqrt(dist2)) repeated over 3 axes        scene/gaussian_model.py:204
 *
 * mean_dist[i] = (d1 + d2 + d3) / 3 with d1 <= d2 <= d3 the three smallest squared Euclidean
 * distances from point i to the OTHER points (a duplicate point counts, at distance 0).  Exact:
 * points are ordered along a 30-bit Morton curve, bounded in boxes of 1024, and every box that
 * can hold a closer point than the current third is scanned.  With fewer than 4 points the
 * missing distances are FLT_MAX (as upstream), so the mean overflows to +inf.
 *
 * Conventions: device pointers, float32, contiguous; points [P, 3]; mean_dist [P].  `workspace`
 * holds >= lsr_knn_workspace_bytes(P) bytes.  All launches on `stream`; no host synchronisation.
 * Return 0 or an LSR_E* code (lsr.h); lsr_last_error().
 */
#ifndef LSR_KNN_H_
#define LSR_KNN_H_
#include <stdint.h>
#ifdef __cplusplus
extern "C" {
#endif

int64_t lsr_knn_workspace_bytes(int32_t P);
int lsr_knn_mean_dist(int32_t P, const float *points, float *mean_dist, void *workspace, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* LSR_KNN_H_ */
