// knn.hip -- mean squared distance to the 3 nearest other points (include/lsr_knn.h), the
// initial-scale estimate of scene/gaussian_model.py:203-204 (upstream simple_knn distCUDA2,
// un-vendored).
//
//   1. bounding box (block partials, one final block);
//   2. 30-bit Morton code per point (10 bits per axis of the box) and a stable radix sort of
//      (code, index) pairs (sort.hip);
//   3. the points gathered into Morton order as float4 (16-byte loads from here on);
//   4. boxes of 1024 consecutive Morton points: their bounds;
//   5. one lane per point: the 6 Morton neighbours give an upper bound `reject` on the third
//      distance; every box whose distance to the point is within both `reject` and the current
//      third best is scanned point by point.  The box bounds are staged in LDS (all lanes read the
//      same box: broadcast), so a lane's work is its box tests plus the few boxes it scans.
// The pruning is conservative, so the result is the exact 3-NN mean (float32 distances
// dx*dx + dy*dy + dz*dz, the three smallest in ascending order, (d1 + d2 + d3) / 3).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <string>

#include "../../include/lsr.h"
#include "../../include/lsr_knn.h"
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {
int fail(int code, const std::string& msg);   // lsr_api.hip (thread-local lsr_last_error)
}

namespace {

constexpr int KNN_BOX = 1024;       // Morton-ordered points per box
constexpr int KNN_RED_BLOCKS = 512; // bounding-box partials
constexpr int KNN_BOX_CHUNK = 1024; // box bounds staged in LDS per round (24 KB)

struct Bounds {
    float mnx, mny, mnz, mxx, mxy, mxz;
};

size_t al256(size_t x) { return (x + 255) / 256 * 256; }

struct KnnWs {
    Bounds* partial;      // [KNN_RED_BLOCKS]
    Bounds* bbox;         // [1]
    uint32_t *code_a, *code_b, *idx_a, *idx_b;
    void* sort_tmp;
    float4* sp;           // points in Morton order
    Bounds* boxes;        // [ceil(P / KNN_BOX)]
    size_t bytes;
};

KnnWs carve(void* base, size_t P) {
    char* b = static_cast<char*>(base);
    KnnWs w{};
    size_t o = 0;
    auto take = [&](size_t n) { char* p = b ? b + o : nullptr; o += al256(n); return p; };
    w.partial = reinterpret_cast<Bounds*>(take(sizeof(Bounds) * KNN_RED_BLOCKS));
    w.bbox = reinterpret_cast<Bounds*>(take(sizeof(Bounds)));
    w.code_a = reinterpret_cast<uint32_t*>(take(4 * P));
    w.code_b = reinterpret_cast<uint32_t*>(take(4 * P));
    w.idx_a = reinterpret_cast<uint32_t*>(take(4 * P));
    w.idx_b = reinterpret_cast<uint32_t*>(take(4 * P));
    w.sort_tmp = take(lsr::radix_temp_bytes(P));
    w.sp = reinterpret_cast<float4*>(take(sizeof(float4) * P));
    w.boxes = reinterpret_cast<Bounds*>(take(sizeof(Bounds) * ((P + KNN_BOX - 1) / KNN_BOX)));
    w.bytes = o;
    return w;
}

__device__ __forceinline__ void wave_minmax(float (&v)[6]) {
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1)
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            const float t = __shfl_xor(v[k], o);
            v[k] = k < 3 ? fminf(v[k], t) : fmaxf(v[k], t);
        }
}

// block (256 threads) min/max of v into out (thread 0 writes)
__device__ __forceinline__ void block_minmax(float (&v)[6], Bounds* out) {
    __shared__ float s[4][6];
    wave_minmax(v);
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0)
#pragma unroll
        for (int k = 0; k < 6; ++k) s[w][k] = v[k];
    __syncthreads();
    if (threadIdx.x == 0) {
        float r[6];
#pragma unroll
        for (int k = 0; k < 6; ++k) {
            r[k] = s[0][k];
            for (int j = 1; j < 4; ++j) r[k] = k < 3 ? fminf(r[k], s[j][k]) : fmaxf(r[k], s[j][k]);
        }
        *out = Bounds{r[0], r[1], r[2], r[3], r[4], r[5]};
    }
}

__global__ void __launch_bounds__(256) k_bbox_partial(int P, const float* __restrict__ pts, Bounds* __restrict__ partial) {
    float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = blockIdx.x * 256 + threadIdx.x; i < P; i += gridDim.x * 256) {
        const float x = pts[3 * i], y = pts[3 * i + 1], z = pts[3 * i + 2];
        v[0] = fminf(v[0], x); v[1] = fminf(v[1], y); v[2] = fminf(v[2], z);
        v[3] = fmaxf(v[3], x); v[4] = fmaxf(v[4], y); v[5] = fmaxf(v[5], z);
    }
    block_minmax(v, partial + blockIdx.x);
}

__global__ void __launch_bounds__(256) k_bbox_final(int n, const Bounds* __restrict__ partial, Bounds* __restrict__ bbox) {
    float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    for (int i = threadIdx.x; i < n; i += 256) {
        const Bounds b = partial[i];
        v[0] = fminf(v[0], b.mnx); v[1] = fminf(v[1], b.mny); v[2] = fminf(v[2], b.mnz);
        v[3] = fmaxf(v[3], b.mxx); v[4] = fmaxf(v[4], b.mxy); v[5] = fmaxf(v[5], b.mxz);
    }
    block_minmax(v, bbox);
}

__device__ __forceinline__ uint32_t spread3(uint32_t x) {   // 10 bits -> every third bit
    x = (x | (x << 16)) & 0x030000FFu;
    x = (x | (x << 8)) & 0x0300F00Fu;
    x = (x | (x << 4)) & 0x030C30C3u;
    x = (x | (x << 2)) & 0x09249249u;
    return x;
}

__device__ __forceinline__ uint32_t quant10(float c, float mn, float mx) {
    const float t = (c - mn) / (mx - mn) * 1023.0f;   // NaN / out of range (flat axis) -> clamped
    return t >= 0.0f ? (uint32_t)fminf(t, 1023.0f) : 0u;
}

__global__ void __launch_bounds__(256) k_morton(int P, const float* __restrict__ pts, const Bounds* __restrict__ bbox,
                                               uint32_t* __restrict__ code, uint32_t* __restrict__ idx) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const Bounds b = *bbox;
    const uint32_t x = quant10(pts[3 * i], b.mnx, b.mxx), y = quant10(pts[3 * i + 1], b.mny, b.mxy),
                   z = quant10(pts[3 * i + 2], b.mnz, b.mxz);
    code[i] = spread3(x) | (spread3(y) << 1) | (spread3(z) << 2);
    idx[i] = (uint32_t)i;
}

__global__ void __launch_bounds__(256) k_gather_sorted(int P, const float* __restrict__ pts, const uint32_t* __restrict__ idx,
                                                      float4* __restrict__ sp) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    const uint32_t j = idx[i];
    sp[i] = make_float4(pts[3 * j], pts[3 * j + 1], pts[3 * j + 2], 0.0f);
}

__global__ void __launch_bounds__(256) k_box_bounds(int P, const float4* __restrict__ sp, Bounds* __restrict__ boxes) {
    float v[6] = {FLT_MAX, FLT_MAX, FLT_MAX, -FLT_MAX, -FLT_MAX, -FLT_MAX};
    const int end = min(P, (int)(blockIdx.x + 1) * KNN_BOX);
    for (int i = blockIdx.x * KNN_BOX + threadIdx.x; i < end; i += 256) {
        const float4 p = sp[i];
        v[0] = fminf(v[0], p.x); v[1] = fminf(v[1], p.y); v[2] = fminf(v[2], p.z);
        v[3] = fmaxf(v[3], p.x); v[4] = fmaxf(v[4], p.y); v[5] = fmaxf(v[5], p.z);
    }
    block_minmax(v, boxes + blockIdx.x);
}

__device__ __forceinline__ void update3(float (&best)[3], float4 ref, float4 q) {
    const float dx = q.x - ref.x, dy = q.y - ref.y, dz = q.z - ref.z;
    float d = dx * dx + dy * dy + dz * dz;
#pragma unroll
    for (int k = 0; k < 3; ++k)
        if (best[k] > d) { const float t = best[k]; best[k] = d; d = t; }
}

__device__ __forceinline__ float box_dist(const Bounds& b, float4 p) {
    float dx = 0.0f, dy = 0.0f, dz = 0.0f;
    if (p.x < b.mnx || p.x > b.mxx) dx = fminf(fabsf(p.x - b.mnx), fabsf(p.x - b.mxx));
    if (p.y < b.mny || p.y > b.mxy) dy = fminf(fabsf(p.y - b.mny), fabsf(p.y - b.mxy));
    if (p.z < b.mnz || p.z > b.mxz) dz = fminf(fabsf(p.z - b.mnz), fabsf(p.z - b.mxz));
    return dx * dx + dy * dy + dz * dz;
}

__global__ void __launch_bounds__(256) k_mean_dist(int P, int nbox, const float4* __restrict__ sp,
                                                  const uint32_t* __restrict__ idx, const Bounds* __restrict__ boxes,
                                                  float* __restrict__ out) {
    __shared__ Bounds s_box[KNN_BOX_CHUNK];
    const int i = blockIdx.x * 256 + threadIdx.x;
    const bool valid = i < P;
    const float4 p = valid ? sp[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float best[3] = {FLT_MAX, FLT_MAX, FLT_MAX};
    if (valid)
        for (int j = max(0, i - 3); j <= min(P - 1, i + 3); ++j)
            if (j != i) update3(best, p, sp[j]);
    const float reject = best[2];
    best[0] = best[1] = best[2] = FLT_MAX;
    for (int b0 = 0; b0 < nbox; b0 += KNN_BOX_CHUNK) {
        const int nb = min(KNN_BOX_CHUNK, nbox - b0);
        __syncthreads();
        for (int t = threadIdx.x; t < nb; t += 256) s_box[t] = boxes[b0 + t];
        __syncthreads();
        if (!valid) continue;
        for (int t = 0; t < nb; ++t) {
            const float d = box_dist(s_box[t], p);
            if (d > reject || d > best[2]) continue;
            const int b = b0 + t, end = min(P, (b + 1) * KNN_BOX);
            for (int j = b * KNN_BOX; j < end; ++j)
                if (j != i) update3(best, p, sp[j]);
        }
    }
    if (valid) out[idx[i]] = (best[0] + best[1] + best[2]) / 3.0f;
}

}  // namespace

extern "C" {

int64_t lsr_knn_workspace_bytes(int32_t P) { return (int64_t)carve(nullptr, (size_t)(P > 0 ? P : 1)).bytes; }

int lsr_knn_mean_dist(int32_t P, const float* points, float* mean_dist, void* workspace, void* stream) {
    if (P < 0) return lsr::fail(LSR_EINVAL, "P must be >= 0");
    if (P == 0) return LSR_OK;
    if (!points || !mean_dist || !workspace) return lsr::fail(LSR_EINVAL, "points, mean_dist and workspace are required");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    KnnWs w = carve(workspace, (size_t)P);
    const int nblk = (P + 255) / 256, nred = std::min(KNN_RED_BLOCKS, nblk);
    const int nbox = (P + KNN_BOX - 1) / KNN_BOX;
    hipLaunchKernelGGL(k_bbox_partial, dim3(nred), dim3(256), 0, st, P, points, w.partial);
    hipLaunchKernelGGL(k_bbox_final, dim3(1), dim3(256), 0, st, nred, (const Bounds*)w.partial, w.bbox);
    hipLaunchKernelGGL(k_morton, dim3(nblk), dim3(256), 0, st, P, points, (const Bounds*)w.bbox, w.code_a, w.idx_a);
    const bool in_b = lsr::radix_sort_pairs(w.code_a, w.idx_a, w.code_b, w.idx_b, (size_t)P, 0, 30, w.sort_tmp, st);
    const uint32_t* idx = in_b ? w.idx_b : w.idx_a;
    hipLaunchKernelGGL(k_gather_sorted, dim3(nblk), dim3(256), 0, st, P, points, idx, w.sp);
    hipLaunchKernelGGL(k_box_bounds, dim3(nbox), dim3(256), 0, st, P, (const float4*)w.sp, w.boxes);
    hipLaunchKernelGGL(k_mean_dist, dim3(nblk), dim3(256), 0, st, P, nbox, (const float4*)w.sp, idx,
                       (const Bounds*)w.boxes, mean_dist);
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return lsr::fail(LSR_EHIP, std::string("knn: ") + hipGetErrorString(e));
    return LSR_OK;
}

}  // extern "C"
