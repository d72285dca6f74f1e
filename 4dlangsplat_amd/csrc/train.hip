// train.hip -- training-step glue over the Gaussian SoA (include/lsr_train.h):
// fused multi-group Adam, densification statistics, the densify / prune row maps, the multi-tensor
// row gather, the split's new positions and scales, and the opacity reset.
//
// All of it is HBM-bound elementwise or row-copy work: one launch covers every tensor (the
// reference issues one torch op per tensor and per group), loads and stores are 16 bytes wide
// where the rows allow, and the row maps come from the device scan in sort.hip.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <string>

#include "../../include/lsr.h"
#include "../../include/lsr_train.h"
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {
int fail(int code, const std::string& msg);   // lsr_api.hip (thread-local lsr_last_error)
}

namespace {

size_t al256(size_t x) { return (x + 255) / 256 * 256; }

// ---------------------------------------------------------------------------------------------
// Adam.  Blocks own chunks of ADAM_CHUNK floats of one group; group g owns chunks
// [chunk0[g], chunk0[g + 1]).
constexpr int ADAM_THREADS = 256;
constexpr int ADAM_CHUNK = ADAM_THREADS * 16;

struct AdamGroupDev {
    float* p;
    const float* g;
    float* m;
    float* v;
    int64_t n;
    float w1, b2, w2, bc2s, ss, eps;   // 1-beta1, beta2, 1-beta2, sqrt(1-beta2^t), -lr/(1-beta1^t), eps
    int vec;                            // all four pointers 16-byte aligned
};
struct AdamArgs {
    AdamGroupDev grp[LSR_ADAM_MAX_GROUPS];
    int64_t chunk0[LSR_ADAM_MAX_GROUPS + 1];
    int ng;
};

// torch's foreach Adam element update (lerp, mul, addcmul, sqrt, div, add, addcdiv), in float32
// with no contraction (the build uses -ffp-contract=off)
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamGroupDev& c) {
    m = m + c.w1 * (g - m);
    v = v * c.b2;
    v = v + c.w2 * (g * g);
    const float den = sqrtf(v) / c.bc2s + c.eps;
    p = p + c.ss * (m / den);
}

__global__ void __launch_bounds__(ADAM_THREADS) k_adam(AdamArgs a) {
    const int64_t b = blockIdx.x;
    int gi = 0;
    for (int k = 1; k < a.ng; ++k) gi = b >= a.chunk0[k] ? k : gi;   // block-uniform
    const AdamGroupDev& c = a.grp[gi];
    const int64_t lo = (b - a.chunk0[gi]) * ADAM_CHUNK, hi = min(c.n, lo + ADAM_CHUNK);
    if (c.vec && hi - lo == ADAM_CHUNK) {
        float4* p4 = reinterpret_cast<float4*>(c.p + lo);
        const float4* g4 = reinterpret_cast<const float4*>(c.g + lo);
        float4* m4 = reinterpret_cast<float4*>(c.m + lo);
        float4* v4 = reinterpret_cast<float4*>(c.v + lo);
        float4 P[4], G[4], M[4], V[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int i = r * ADAM_THREADS + threadIdx.x;
            P[r] = p4[i]; G[r] = g4[i]; M[r] = m4[i]; V[r] = v4[i];
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            adam_elem(P[r].x, G[r].x, M[r].x, V[r].x, c);
            adam_elem(P[r].y, G[r].y, M[r].y, V[r].y, c);
            adam_elem(P[r].z, G[r].z, M[r].z, V[r].z, c);
            adam_elem(P[r].w, G[r].w, M[r].w, V[r].w, c);
            const int i = r * ADAM_THREADS + threadIdx.x;
            p4[i] = P[r]; m4[i] = M[r]; v4[i] = V[r];
        }
    } else {
        for (int64_t i = lo + threadIdx.x; i < hi; i += ADAM_THREADS) {
            float p = c.p[i], m = c.m[i], v = c.v[i];
            adam_elem(p, c.g[i], m, v, c);
            c.p[i] = p; c.m[i] = m; c.v[i] = v;
        }
    }
}

// ---------------------------------------------------------------------------------------------
__global__ void k_densify_stats(int P, const int* radii, const float* grad, int stride, float* max_r,
                                float* accum, float* denom) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const int r = radii[i];
    if (r <= 0) return;
    max_r[i] = fmaxf(max_r[i], (float)r);
    const float gx = grad[(size_t)i * stride], gy = grad[(size_t)i * stride + 1];
    accum[i] += sqrtf(gx * gx + gy * gy);
    denom[i] += 1.0f;
}

__device__ __forceinline__ float max_scale(const float* scaling, int i) {
    return fmaxf(fmaxf(expf(scaling[3 * i]), expf(scaling[3 * i + 1])), expf(scaling[3 * i + 2]));
}

__global__ void k_densify_flags(int P, const float* accum, const float* denom, const float* scaling, float thr,
                                float limit, uint32_t* fclone, uint32_t* fsplit) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    float g = accum[i] / denom[i];
    if (g != g) g = 0.0f;
    const float s = max_scale(scaling, i);
    fclone[i] = (fabsf(g) >= thr && s <= limit) ? 1u : 0u;
    fsplit[i] = (g >= thr && s > limit) ? 1u : 0u;
}

// totals: [0] cloned, [1] split (exclusive_scan_u32 totals)
__global__ void k_densify_index(int P, int copies, const uint32_t* fclone, const uint32_t* fsplit,
                                const uint32_t* oclone, const uint32_t* osplit, const uint32_t* totals, int* index,
                                int64_t* counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t nclone = totals[0], nsplit = totals[1];
    const uint32_t kept = (uint32_t)P - nsplit;
    if (i == 0) {
        counts[0] = kept; counts[1] = nclone; counts[2] = nsplit;
    }
    if (i >= P) return;
    if (fsplit[i]) {
        const size_t base = (size_t)kept + nclone + osplit[i];
        for (int c = 0; c < copies; ++c) index[base + (size_t)c * nsplit] = i;
    } else {
        index[i - osplit[i]] = i;
    }
    if (fclone[i]) index[kept + oclone[i]] = i;
}

__global__ void k_prune_flags(int P, const float* opacity, const float* max_r, const float* scaling, float min_op,
                              float max_screen, float big_ws, uint32_t* keep) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float o = 1.0f / (1.0f + expf(-opacity[i]));
    bool prune = o < min_op;
    if (max_screen > 0.0f) prune = prune || max_r[i] > max_screen || max_scale(scaling, i) > big_ws;
    keep[i] = prune ? 0u : 1u;
}

__global__ void k_prune_index(int P, const uint32_t* keep, const uint32_t* off, const uint32_t* total, int* index,
                              int64_t* counts) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i == 0) counts[0] = total[0];
    if (i < P && keep[i]) index[off[i]] = i;
}

// ---------------------------------------------------------------------------------------------
// Row gather: blockIdx.y = tensor; units of 16, 4 or 1 bytes (the widest that divides the row and
// both base addresses).
struct GatherTensor {
    const char* src;
    char* dst;
    int64_t row_units, zero_from;
    int unit;
};
struct GatherArgs {
    GatherTensor t[LSR_GATHER_MAX_TENSORS];
    int64_t n_rows;
};

template <typename U>
__device__ void gather_units(const GatherTensor& t, const int* index, int64_t n_rows) {
    const U* src = reinterpret_cast<const U*>(t.src);
    U* dst = reinterpret_cast<U*>(t.dst);
    const int64_t total = n_rows * t.row_units;
    const int64_t stride = (int64_t)gridDim.x * blockDim.x;
    for (int64_t u = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; u < total; u += stride) {
        const int64_t j = u / t.row_units, k = u - j * t.row_units;
        U val;
        if (j < t.zero_from) val = src[(int64_t)index[j] * t.row_units + k];
        else val = U{};
        dst[u] = val;
    }
}

__global__ void __launch_bounds__(256) k_gather_rows(GatherArgs a, const int* index) {
    const GatherTensor& t = a.t[blockIdx.y];
    if (t.unit == 16) gather_units<uint4>(t, index, a.n_rows);
    else if (t.unit == 4) gather_units<uint32_t>(t, index, a.n_rows);
    else gather_units<uint8_t>(t, index, a.n_rows);
}

__global__ void k_split_fixup(int64_t n_new, int64_t base, float div, const int* index, const float* xyz_src,
                              const float* sc_src, const float* rot_src, const float* samples, float* xyz_dst,
                              float* sc_dst) {
    const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n_new) return;
    const int64_t j = base + k;
    const int i = index[j];
    // build_rotation (utils/general_utils.py:84-110): normalised quaternion (r, x, y, z)
    const float q0 = rot_src[4 * i], q1 = rot_src[4 * i + 1], q2 = rot_src[4 * i + 2], q3 = rot_src[4 * i + 3];
    const float nrm = sqrtf(q0 * q0 + q1 * q1 + q2 * q2 + q3 * q3);
    const float r = q0 / nrm, x = q1 / nrm, y = q2 / nrm, z = q3 / nrm;
    const float R[9] = {1.0f - 2.0f * (y * y + z * z), 2.0f * (x * y - r * z), 2.0f * (x * z + r * y),
                        2.0f * (x * y + r * z), 1.0f - 2.0f * (x * x + z * z), 2.0f * (y * z - r * x),
                        2.0f * (x * z - r * y), 2.0f * (y * z + r * x), 1.0f - 2.0f * (x * x + y * y)};
    float s[3], smp[3];
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float sd = expf(sc_src[3 * i + a]);
        smp[a] = sd * samples[3 * k + a];             // torch.normal(0, std) = std * z
        s[a] = logf(sd / div);                         // log(get_scaling / (0.8 N))
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) {
        const float d = R[3 * a] * smp[0] + R[3 * a + 1] * smp[1] + R[3 * a + 2] * smp[2];
        xyz_dst[3 * j + a] = d + xyz_src[3 * i + a];
        sc_dst[3 * j + a] = s[a];
    }
}

__global__ void k_reset_opacity(int P, float* opacity, float* m, float* v) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float o = fminf(1.0f / (1.0f + expf(-opacity[i])), 0.01f);
    opacity[i] = logf(o / (1.0f - o));
    if (m) m[i] = 0.0f;
    if (v) v[i] = 0.0f;
}

// The render path's activations (gaussian_renderer/__init__.py:191-193 with gaussian_model.py:38-46:
// torch.exp, torch.nn.functional.normalize (x / max(|x|, 1e-12)), torch.sigmoid), one thread per row
// of all three, in PyTorch's order of operations: bit for bit its results (checked on 4M random rows:
// its norm sums the squares pairwise, (x0^2 + x1^2) + (x2^2 + x3^2); exp and 1 / (1 + exp(-x)) as here).
__global__ void __launch_bounds__(256) k_activate(int P, const float* __restrict__ rs, const float* __restrict__ rr,
                                                  const float* __restrict__ ro, float* __restrict__ s,
                                                  float* __restrict__ r, float* __restrict__ o) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    if (rs) {
#pragma unroll
        for (int c = 0; c < 3; ++c) s[3 * i + c] = expf(rs[3 * i + c]);
    }
    if (rr) {
        const float4 q = reinterpret_cast<const float4*>(rr)[i];
        const float n = fmaxf(sqrtf((q.x * q.x + q.y * q.y) + (q.z * q.z + q.w * q.w)), 1e-12f);
        reinterpret_cast<float4*>(r)[i] = make_float4(q.x / n, q.y / n, q.z / n, q.w / n);
    }
    if (ro) o[i] = 1.0f / (1.0f + expf(-ro[i]));
}
// Their backward (the autograd formulas of the three ops): d exp = d s, d normalize = (d - y (y . d)) / |x|
// for |x| > 1e-12 (d / 1e-12 below, where the clamp is constant), d sigmoid = d o (1 - o).
__global__ void __launch_bounds__(256) k_activate_bwd(int P, const float* __restrict__ s, const float* __restrict__ rr,
                                                      const float* __restrict__ o, const float* __restrict__ ds,
                                                      const float* __restrict__ dr, const float* __restrict__ dop,
                                                      float* __restrict__ dsr, float* __restrict__ drr,
                                                      float* __restrict__ dor) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= P) return;
    if (dsr) {
#pragma unroll
        for (int c = 0; c < 3; ++c) dsr[3 * i + c] = ds ? ds[3 * i + c] * s[3 * i + c] : 0.0f;
    }
    if (drr) {
        const float4 q = reinterpret_cast<const float4*>(rr)[i];
        const float4 d = dr ? reinterpret_cast<const float4*>(dr)[i] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const float len = sqrtf((q.x * q.x + q.y * q.y) + (q.z * q.z + q.w * q.w));
        float4 g;
        if (len > 1e-12f) {
            const float4 y = make_float4(q.x / len, q.y / len, q.z / len, q.w / len);
            const float yd = y.x * d.x + y.y * d.y + y.z * d.z + y.w * d.w;
            g = make_float4((d.x - y.x * yd) / len, (d.y - y.y * yd) / len, (d.z - y.z * yd) / len,
                            (d.w - y.w * yd) / len);
        } else {
            g = make_float4(d.x / 1e-12f, d.y / 1e-12f, d.z / 1e-12f, d.w / 1e-12f);
        }
        reinterpret_cast<float4*>(drr)[i] = g;
    }
    if (dor) dor[i] = dop ? dop[i] * o[i] * (1.0f - o[i]) : 0.0f;
}

// render_views' V views of P Gaussians (gaussian_scene.py): a tensor's rows repeated V times
// (torch.Tensor.repeat(V, 1, ...)) and, backward, the V row blocks summed, every tensor of the call
// in one launch (grid row = tensor); rows of whole floats, flat element index e.
struct RowBlocksArgs {
    const float* src[LSR_GATHER_MAX_TENSORS];
    float* dst[LSR_GATHER_MAX_TENSORS];
    int64_t n[LSR_GATHER_MAX_TENSORS];   // floats of one block (n_rows * row floats)
    int nb;                              // blocks (views)
};
__global__ void __launch_bounds__(256) k_repeat_rows(RowBlocksArgs a) {
    const float* __restrict__ src = a.src[blockIdx.y];
    float* __restrict__ dst = a.dst[blockIdx.y];
    const int64_t n = a.n[blockIdx.y];
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
        const float v = src[e];
        for (int b = 0; b < a.nb; ++b) dst[(int64_t)b * n + e] = v;
    }
}
__global__ void __launch_bounds__(256) k_sum_row_blocks(RowBlocksArgs a) {
    const float* __restrict__ src = a.src[blockIdx.y];
    float* __restrict__ dst = a.dst[blockIdx.y];
    const int64_t n = a.n[blockIdx.y];
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < n; e += (int64_t)gridDim.x * 256) {
        float v = src[e];
        for (int b = 1; b < a.nb; ++b) v += src[(int64_t)b * n + e];
        dst[e] = v;
    }
}

// The base stages' loss (train.py:272-276, utils/loss_utils.py l1_loss): mean |image_v - gt_v| over the
// views' [3, H, W] images without stacking them; the per-block partial sums are added in a fixed
// order by one block (deterministic), and the backward is PyTorch's abs / mean backward,
// sign(x) * (g * (1 / N)), bit for bit.
constexpr int L1_MAX_VIEWS = 8, L1_BLOCKS = 256;
struct L1Args {
    const float* img[L1_MAX_VIEWS];
    float* grad[L1_MAX_VIEWS];
    const float* gt;
    int64_t gt_stride, n;     // floats between the views' gt blocks; floats per view
    int64_t total;            // V n
    const float* d_loss;
    float* partial;           // [V][L1_BLOCKS]
    float* loss;
};
__global__ void __launch_bounds__(256) k_l1_partial(L1Args a) {
    __shared__ float s_w[4];
    const float* __restrict__ x = a.img[blockIdx.y];
    const float* __restrict__ y = a.gt + blockIdx.y * a.gt_stride;
    float acc = 0.0f;
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < a.n; e += (int64_t)gridDim.x * 256) acc += fabsf(x[e] - y[e]);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) a.partial[blockIdx.y * gridDim.x + blockIdx.x] = (s_w[0] + s_w[1]) + (s_w[2] + s_w[3]);
}
__global__ void __launch_bounds__(256) k_l1_final(L1Args a, int nparts) {
    __shared__ float s_w[4];
    float acc = 0.0f;
    for (int i = threadIdx.x; i < nparts; i += 256) acc += a.partial[i];
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc += __shfl_xor(acc, off);
    if ((threadIdx.x & 63) == 0) s_w[threadIdx.x >> 6] = acc;
    __syncthreads();
    if (threadIdx.x == 0) a.loss[0] = ((s_w[0] + s_w[1]) + (s_w[2] + s_w[3])) * (1.0f / (float)a.total);
}
__global__ void __launch_bounds__(256) k_l1_grad(L1Args a) {
    const float* __restrict__ x = a.img[blockIdx.y];
    const float* __restrict__ y = a.gt + blockIdx.y * a.gt_stride;
    float* __restrict__ d = a.grad[blockIdx.y];
    // mean's backward, g / N, as PyTorch's division by a host scalar runs it (times the float reciprocal),
    // then abs's: * sign
    const float s = a.d_loss[0] * (1.0f / (float)a.total);
    for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < a.n; e += (int64_t)gridDim.x * 256) {
        const float v = x[e] - y[e];
        d[e] = s * (v > 0.0f ? 1.0f : (v < 0.0f ? -1.0f : 0.0f));
    }
}

struct TrainWs {
    uint32_t *f0, *f1, *o0, *o1, *totals;
    void* scan_tmp;
    size_t bytes;
};
TrainWs carve(void* base, size_t P) {
    char* b = static_cast<char*>(base);
    TrainWs w{};
    size_t o = 0;
    auto take = [&](size_t n) { char* p = b ? b + o : nullptr; o += al256(n); return p; };
    w.f0 = reinterpret_cast<uint32_t*>(take(4 * P));
    w.f1 = reinterpret_cast<uint32_t*>(take(4 * P));
    w.o0 = reinterpret_cast<uint32_t*>(take(4 * P));
    w.o1 = reinterpret_cast<uint32_t*>(take(4 * P));
    w.totals = reinterpret_cast<uint32_t*>(take(16));
    w.scan_tmp = take(lsr::scan_temp_bytes(P));
    w.bytes = o;
    return w;
}

int launched(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return lsr::fail(LSR_EHIP, std::string(what) + ": " + hipGetErrorString(e));
    return LSR_OK;
}

bool al16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

}  // namespace

extern "C" {

int lsr_adam_step(const lsr_adam_group* groups, int32_t n_groups, double beta1, double beta2, double eps,
                  void* stream) {
    if (n_groups < 0 || n_groups > LSR_ADAM_MAX_GROUPS || (n_groups > 0 && !groups))
        return lsr::fail(LSR_EINVAL, "lsr_adam_step: 0 <= n_groups <= LSR_ADAM_MAX_GROUPS");
    AdamArgs a{};
    int64_t chunks = 0;
    for (int k = 0; k < n_groups; ++k) {
        const lsr_adam_group& g = groups[k];
        if (g.n < 0 || g.step < 1) return lsr::fail(LSR_EINVAL, "lsr_adam_step: n >= 0 and step >= 1 required");
        if (!g.grad || g.n == 0) continue;
        if (!g.param || !g.exp_avg || !g.exp_avg_sq) return lsr::fail(LSR_EINVAL, "lsr_adam_step: null tensor");
        AdamGroupDev& d = a.grp[a.ng];
        d.p = g.param; d.g = g.grad; d.m = g.exp_avg; d.v = g.exp_avg_sq; d.n = g.n;
        // torch/optim/adam.py: bias corrections and step size in Python floats (double)
        const double bc1 = 1.0 - std::pow(beta1, (double)g.step), bc2 = 1.0 - std::pow(beta2, (double)g.step);
        d.w1 = (float)(1.0 - beta1); d.b2 = (float)beta2; d.w2 = (float)(1.0 - beta2);
        d.bc2s = (float)std::sqrt(bc2); d.ss = (float)(-(g.lr / bc1)); d.eps = (float)eps;
        d.vec = al16(g.param) && al16(g.grad) && al16(g.exp_avg) && al16(g.exp_avg_sq);
        a.chunk0[a.ng] = chunks;
        chunks += (g.n + ADAM_CHUNK - 1) / ADAM_CHUNK;
        ++a.ng;
    }
    a.chunk0[a.ng] = chunks;
    if (chunks == 0) return LSR_OK;
    hipLaunchKernelGGL(k_adam, dim3((unsigned)chunks), dim3(ADAM_THREADS), 0, reinterpret_cast<hipStream_t>(stream), a);
    return launched("adam");
}

int lsr_densify_stats(int32_t P, const int32_t* radii, const float* means2D_grad, int32_t grad_stride,
                      float* max_radii2D, float* xyz_gradient_accum, float* denom, void* stream) {
    if (P < 0 || grad_stride < 2) return lsr::fail(LSR_EINVAL, "lsr_densify_stats: P >= 0, grad_stride >= 2");
    if (P == 0) return LSR_OK;
    if (!radii || !means2D_grad || !max_radii2D || !xyz_gradient_accum || !denom)
        return lsr::fail(LSR_EINVAL, "lsr_densify_stats: null tensor");
    hipLaunchKernelGGL(k_densify_stats, dim3((P + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), P,
                       radii, means2D_grad, grad_stride, max_radii2D, xyz_gradient_accum, denom);
    return launched("densify stats");
}

int64_t lsr_train_workspace_bytes(int32_t P) { return (int64_t)carve(nullptr, (size_t)(P > 0 ? P : 1)).bytes; }

int lsr_densify_plan(int32_t P, const float* xyz_gradient_accum, const float* denom, const float* scaling,
                     float grad_threshold, float percent_dense, float extent, int32_t n_copies, int32_t* index,
                     int64_t* counts, void* workspace, void* stream) {
    if (P < 0 || n_copies < 1) return lsr::fail(LSR_EINVAL, "lsr_densify_plan: P >= 0, n_copies >= 1");
    if (!counts) return lsr::fail(LSR_EINVAL, "lsr_densify_plan: counts required");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (P == 0) {
        if (hipMemsetAsync(counts, 0, 3 * sizeof(int64_t), st) != hipSuccess) return launched("densify plan");
        return LSR_OK;
    }
    if (!xyz_gradient_accum || !denom || !scaling || !index || !workspace)
        return lsr::fail(LSR_EINVAL, "lsr_densify_plan: null tensor");
    TrainWs w = carve(workspace, (size_t)P);
    const dim3 grid((P + 255) / 256);
    hipLaunchKernelGGL(k_densify_flags, grid, dim3(256), 0, st, P, xyz_gradient_accum, denom, scaling, grad_threshold,
                       percent_dense * extent, w.f0, w.f1);
    lsr::exclusive_scan_u32(w.f0, w.o0, (size_t)P, w.totals, w.scan_tmp, st);
    lsr::exclusive_scan_u32(w.f1, w.o1, (size_t)P, w.totals + 1, w.scan_tmp, st);
    hipLaunchKernelGGL(k_densify_index, grid, dim3(256), 0, st, P, n_copies, (const uint32_t*)w.f0,
                       (const uint32_t*)w.f1, (const uint32_t*)w.o0, (const uint32_t*)w.o1, (const uint32_t*)w.totals,
                       index, counts);
    return launched("densify plan");
}

int lsr_prune_plan(int32_t P, const float* opacity, const float* max_radii2D, const float* scaling,
                   float min_opacity, float max_screen_size, float extent, int32_t* index, int64_t* counts,
                   void* workspace, void* stream) {
    if (P < 0) return lsr::fail(LSR_EINVAL, "lsr_prune_plan: P >= 0");
    if (!counts) return lsr::fail(LSR_EINVAL, "lsr_prune_plan: counts required");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    if (P == 0) {
        if (hipMemsetAsync(counts, 0, sizeof(int64_t), st) != hipSuccess) return launched("prune plan");
        return LSR_OK;
    }
    if (!opacity || !scaling || !index || !workspace || (max_screen_size > 0.0f && !max_radii2D))
        return lsr::fail(LSR_EINVAL, "lsr_prune_plan: null tensor");
    TrainWs w = carve(workspace, (size_t)P);
    const dim3 grid((P + 255) / 256);
    hipLaunchKernelGGL(k_prune_flags, grid, dim3(256), 0, st, P, opacity, max_radii2D, scaling, min_opacity,
                       max_screen_size, 0.1f * extent, w.f0);
    lsr::exclusive_scan_u32(w.f0, w.o0, (size_t)P, w.totals, w.scan_tmp, st);
    hipLaunchKernelGGL(k_prune_index, grid, dim3(256), 0, st, P, (const uint32_t*)w.f0, (const uint32_t*)w.o0,
                       (const uint32_t*)w.totals, index, counts);
    return launched("prune plan");
}

int lsr_gather_rows(int32_t n_tensors, const lsr_row_tensor* t, const int32_t* index, int64_t n_rows, void* stream) {
    if (n_tensors < 0 || n_tensors > LSR_GATHER_MAX_TENSORS || n_rows < 0 || (n_tensors > 0 && !t))
        return lsr::fail(LSR_EINVAL, "lsr_gather_rows: 0 <= n_tensors <= LSR_GATHER_MAX_TENSORS, n_rows >= 0");
    if (n_tensors == 0 || n_rows == 0) return LSR_OK;
    GatherArgs a{};
    a.n_rows = n_rows;
    int64_t most = 0;
    bool needs_index = false;
    for (int k = 0; k < n_tensors; ++k) {
        const lsr_row_tensor& r = t[k];
        if (r.row_bytes <= 0 || !r.dst || (r.zero_from > 0 && !r.src))
            return lsr::fail(LSR_EINVAL, "lsr_gather_rows: row_bytes > 0, dst (and src unless all rows are zero)");
        const uintptr_t bits = reinterpret_cast<uintptr_t>(r.src) | reinterpret_cast<uintptr_t>(r.dst) |
                               (uintptr_t)r.row_bytes;
        const int unit = (bits & 15u) == 0 ? 16 : (bits & 3u) == 0 ? 4 : 1;
        a.t[k].src = static_cast<const char*>(r.src);
        a.t[k].dst = static_cast<char*>(r.dst);
        a.t[k].unit = unit;
        a.t[k].row_units = r.row_bytes / unit;
        a.t[k].zero_from = r.zero_from;
        needs_index = needs_index || r.zero_from > 0;
        most = std::max(most, n_rows * a.t[k].row_units);
    }
    if (needs_index && !index) return lsr::fail(LSR_EINVAL, "lsr_gather_rows: index required");
    const unsigned bx = (unsigned)std::min<int64_t>((most + 255) / 256, 2048);
    hipLaunchKernelGGL(k_gather_rows, dim3(bx, n_tensors), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a,
                       index);
    return launched("gather rows");
}

int lsr_split_fixup(int64_t n_new, int64_t base, int32_t n_copies, const int32_t* index, const float* xyz_src,
                    const float* scaling_src, const float* rotation_src, const float* samples, float* xyz_dst,
                    float* scaling_dst, void* stream) {
    if (n_new < 0 || base < 0 || n_copies < 1) return lsr::fail(LSR_EINVAL, "lsr_split_fixup: bad sizes");
    if (n_new == 0) return LSR_OK;
    if (!index || !xyz_src || !scaling_src || !rotation_src || !samples || !xyz_dst || !scaling_dst)
        return lsr::fail(LSR_EINVAL, "lsr_split_fixup: null tensor");
    // get_scaling / (0.8 * N): the divisor is a Python float, applied in float32
    const float div = (float)(0.8 * (double)n_copies);
    hipLaunchKernelGGL(k_split_fixup, dim3((unsigned)((n_new + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), n_new, base, div, index, xyz_src, scaling_src,
                       rotation_src, samples, xyz_dst, scaling_dst);
    return launched("split fixup");
}

int lsr_reset_opacity(int32_t P, float* opacity, float* exp_avg, float* exp_avg_sq, void* stream) {
    if (P < 0) return lsr::fail(LSR_EINVAL, "lsr_reset_opacity: P >= 0");
    if (P == 0) return LSR_OK;
    if (!opacity) return lsr::fail(LSR_EINVAL, "lsr_reset_opacity: opacity required");
    hipLaunchKernelGGL(k_reset_opacity, dim3((P + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), P,
                       opacity, exp_avg, exp_avg_sq);
    return launched("reset opacity");
}

static int row_blocks(const char* what, bool sum, int32_t n_tensors, const lsr_row_tensor* t, int64_t n_rows,
                      int32_t n_blocks, void* stream) {
    if (n_tensors < 0 || n_tensors > LSR_GATHER_MAX_TENSORS || n_rows < 0 || n_blocks < 1 || (n_tensors > 0 && !t))
        return lsr::fail(LSR_EINVAL, std::string(what) + ": 0 <= n_tensors <= LSR_GATHER_MAX_TENSORS, n_rows >= 0, "
                                                       "n_blocks >= 1");
    if (n_tensors == 0 || n_rows == 0) return LSR_OK;
    RowBlocksArgs a{};
    a.nb = n_blocks;
    int64_t most = 0;
    for (int k = 0; k < n_tensors; ++k) {
        if (!t[k].src || !t[k].dst || t[k].row_bytes <= 0 || t[k].row_bytes % 4)
            return lsr::fail(LSR_EINVAL, std::string(what) + ": src, dst and rows of whole floats required");
        a.src[k] = static_cast<const float*>(t[k].src);
        a.dst[k] = static_cast<float*>(t[k].dst);
        a.n[k] = n_rows * (t[k].row_bytes / 4);
        most = std::max(most, a.n[k]);
    }
    const dim3 grid((unsigned)std::min<int64_t>((most + 255) / 256, 4096), n_tensors);
    if (sum) hipLaunchKernelGGL(k_sum_row_blocks, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
    else hipLaunchKernelGGL(k_repeat_rows, grid, dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
    return launched(what);
}

int lsr_repeat_rows(int32_t n_tensors, const lsr_row_tensor* t, int64_t n_rows, int32_t n_blocks, void* stream) {
    return row_blocks("lsr_repeat_rows", false, n_tensors, t, n_rows, n_blocks, stream);
}

int lsr_sum_row_blocks(int32_t n_tensors, const lsr_row_tensor* t, int64_t n_rows, int32_t n_blocks, void* stream) {
    return row_blocks("lsr_sum_row_blocks", true, n_tensors, t, n_rows, n_blocks, stream);
}

int64_t lsr_l1_workspace_bytes(int32_t V) { return (int64_t)(V > 0 ? V : 1) * L1_BLOCKS * (int64_t)sizeof(float); }

static int l1_args(const char* what, int32_t V, int64_t n, const float* const* images, const float* gt,
                   int64_t gt_view_stride, L1Args& a) {
    if (V < 1 || V > L1_MAX_VIEWS || n < 0 || !images || !gt || gt_view_stride < n)
        return lsr::fail(LSR_EINVAL, std::string(what) + ": 1 <= V <= 8, n >= 0, gt_view_stride >= n, images and gt");
    a = L1Args{};
    for (int v = 0; v < V; ++v) {
        if (!images[v]) return lsr::fail(LSR_EINVAL, std::string(what) + ": null image");
        a.img[v] = images[v];
    }
    a.gt = gt;
    a.gt_stride = gt_view_stride;
    a.n = n;
    a.total = (int64_t)V * n;
    return LSR_OK;
}

int lsr_l1_loss_views(int32_t V, int64_t n, const float* const* images, const float* gt, int64_t gt_view_stride,
                      float* loss, void* workspace, void* stream) {
    L1Args a;
    if (int rc = l1_args("lsr_l1_loss_views", V, n, images, gt, gt_view_stride, a)) return rc;
    if (!loss || !workspace) return lsr::fail(LSR_EINVAL, "lsr_l1_loss_views: loss and workspace required");
    a.partial = static_cast<float*>(workspace);
    a.loss = loss;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    hipLaunchKernelGGL(k_l1_partial, dim3(L1_BLOCKS, V), dim3(256), 0, st, a);
    hipLaunchKernelGGL(k_l1_final, dim3(1), dim3(256), 0, st, a, V * L1_BLOCKS);
    return launched("l1 loss");
}

int lsr_l1_loss_views_backward(int32_t V, int64_t n, const float* const* images, const float* gt,
                               int64_t gt_view_stride, const float* d_loss, float* const* d_images, void* stream) {
    L1Args a;
    if (int rc = l1_args("lsr_l1_loss_views_backward", V, n, images, gt, gt_view_stride, a)) return rc;
    if (!d_loss || !d_images) return lsr::fail(LSR_EINVAL, "lsr_l1_loss_views_backward: d_loss and d_images required");
    for (int v = 0; v < V; ++v) {
        if (!d_images[v]) return lsr::fail(LSR_EINVAL, "lsr_l1_loss_views_backward: null gradient image");
        a.grad[v] = d_images[v];
    }
    a.d_loss = d_loss;
    const unsigned bx = (unsigned)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 1024));
    hipLaunchKernelGGL(k_l1_grad, dim3(bx, V), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), a);
    return launched("l1 loss backward");
}

int lsr_activate(int32_t P, const float* raw_scales, const float* raw_rotations, const float* raw_opacity,
                 float* scales, float* rotations, float* opacity, void* stream) {
    if (P < 0) return lsr::fail(LSR_EINVAL, "lsr_activate: P >= 0");
    if ((raw_scales && !scales) || (raw_rotations && !rotations) || (raw_opacity && !opacity))
        return lsr::fail(LSR_EINVAL, "lsr_activate: every given input needs its output");
    if (raw_rotations && (!al16(raw_rotations) || !al16(rotations)))
        return lsr::fail(LSR_EINVAL, "lsr_activate: rotation rows must be 16-byte aligned");
    if (P == 0) return LSR_OK;
    hipLaunchKernelGGL(k_activate, dim3((P + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), P,
                       raw_scales, raw_rotations, raw_opacity, scales, rotations, opacity);
    return launched("activate");
}

int lsr_activate_backward(int32_t P, const float* scales, const float* raw_rotations, const float* opacity,
                          const float* d_scales, const float* d_rotations, const float* d_opacity,
                          float* d_raw_scales, float* d_raw_rotations, float* d_raw_opacity, void* stream) {
    if (P < 0) return lsr::fail(LSR_EINVAL, "lsr_activate_backward: P >= 0");
    if ((d_raw_scales && !scales) || (d_raw_rotations && !raw_rotations) || (d_raw_opacity && !opacity))
        return lsr::fail(LSR_EINVAL, "lsr_activate_backward: every requested gradient needs its forward values");
    if (d_raw_rotations && (!al16(raw_rotations) || !al16(d_raw_rotations) || (d_rotations && !al16(d_rotations))))
        return lsr::fail(LSR_EINVAL, "lsr_activate_backward: rotation rows must be 16-byte aligned");
    if (P == 0) return LSR_OK;
    hipLaunchKernelGGL(k_activate_bwd, dim3((P + 255) / 256), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), P,
                       scales, raw_rotations, opacity, d_scales, d_rotations, d_opacity, d_raw_scales, d_raw_rotations,
                       d_raw_opacity);
    return launched("activate backward");
}

}  // extern "C"
