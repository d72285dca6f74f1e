// deform_api.hip -- C ABI of the deformation field (include/lsr_deform.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/lsr.h"
#include "../../include/lsr_deform.h"
#include "lsr_internal.h"

namespace lsr {
int fail(int code, const std::string& msg);   // lsr_api.hip (thread-local lsr_last_error)
}

namespace {

constexpr int kCombos[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};
constexpr int kHeadOut[5] = {3, 3, 4, 1, 48};
constexpr int kW2Rows = 64;

size_t align256(size_t x) { return (x + 255) / 256 * 256; }

// plane 6 s + ci: width (along coordinate c0) and height (along c1)
void plane_dims(const lsr_deform_net* n, int s, int ci, int& W, int& H) {
    auto res = [&](int c) { return c < 3 ? n->res[c] * n->multires[s] : n->res[3]; };
    W = res(kCombos[ci][0]);
    H = res(kCombos[ci][1]);
}

struct Layout {
    size_t plane_off[12];   // bytes
    size_t planes_end;      // bytes of the packed planes
    size_t wf, w1, w2;      // bytes: hi arrays, lo right after each
    size_t wft, w1t, w2t;   // transposed packs for the backward: [32][128], [5][128][128], [5][128][64]
    size_t total;
};

Layout layout(const lsr_deform_net* n) {
    Layout L{};
    size_t o = 0;
    for (int s = 0; s < n->n_scales; ++s)
        for (int ci = 0; ci < 6; ++ci) {
            int W, H;
            plane_dims(n, s, ci, W, H);
            L.plane_off[6 * s + ci] = o;
            o += align256((size_t)W * H * 16 * sizeof(float));
        }
    L.planes_end = o;
    const size_t bf = sizeof(__bf16);
    L.wf = o; o += align256((size_t)128 * 32 * bf) * 2;
    L.w1 = o; o += align256((size_t)5 * 128 * 128 * bf) * 2;
    L.w2 = o; o += align256((size_t)5 * kW2Rows * 128 * bf) * 2;
    L.wft = o; o += align256((size_t)32 * 128 * bf) * 2;
    L.w1t = o; o += align256((size_t)5 * 128 * 128 * bf) * 2;
    L.w2t = o; o += align256((size_t)5 * 128 * 64 * bf) * 2;
    L.total = o;
    return L;
}

int check(const lsr_deform_net* n) {
    if (!n) return lsr::fail(LSR_EINVAL, "null deformation net");
    if (n->n_scales != 2 || n->channels != 16 || n->width != 128)
        return lsr::fail(LSR_EINVAL, "this build supports the Neu3D structure: 2 scales x 16 channels, width 128");
    for (int c = 0; c < 4; ++c)
        if (n->res[c] < 2) return lsr::fail(LSR_EINVAL, "plane resolutions must be >= 2");
    for (int s = 0; s < n->n_scales; ++s) {
        if (n->multires[s] < 1) return lsr::fail(LSR_EINVAL, "multires must be >= 1");
        for (int ci = 0; ci < 6; ++ci)
            if (!n->planes[s][ci]) return lsr::fail(LSR_EINVAL, "missing plane");
    }
    if (!n->aabb || !n->w_feat || !n->b_feat) return lsr::fail(LSR_EINVAL, "missing aabb / feature_out");
    for (int h = 0; h < LSR_DEFORM_HEADS; ++h)
        if (!n->w1[h] || !n->b1[h] || !n->w2[h] || !n->b2[h]) return lsr::fail(LSR_EINVAL, "missing head weights");
    return LSR_OK;
}

}  // namespace

extern "C" int64_t lsr_deform_workspace_bytes(const lsr_deform_net* net) {
    if (check(net)) return -1;
    return (int64_t)layout(net).total;
}

extern "C" int lsr_deform_prepare(const lsr_deform_net* net, void* workspace, void* stream) {
    int rc = check(net);
    if (rc) return rc;
    if (!workspace) return lsr::fail(LSR_EINVAL, "workspace is required");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const Layout L = layout(net);
    char* ws = reinterpret_cast<char*>(workspace);
    for (int s = 0; s < net->n_scales; ++s)
        for (int ci = 0; ci < 6; ++ci) {
            int W, H;
            plane_dims(net, s, ci, W, H);
            lsr::launch_pack_plane(net->planes[s][ci], reinterpret_cast<float*>(ws + L.plane_off[6 * s + ci]), H, W, st);
        }
    auto hi_lo = [&](size_t off, size_t count, __bf16*& hi, __bf16*& lo) {
        hi = reinterpret_cast<__bf16*>(ws + off);
        lo = reinterpret_cast<__bf16*>(ws + off + align256(count * sizeof(__bf16)));
    };
    __bf16 *h, *l;
    hi_lo(L.wf, 128 * 32, h, l);
    lsr::launch_pack_weight(net->w_feat, h, l, 128, 128, 32, st);
    hi_lo(L.w1, 5 * 128 * 128, h, l);
    for (int hd = 0; hd < 5; ++hd)
        lsr::launch_pack_weight(net->w1[hd], h + (size_t)hd * 128 * 128, l + (size_t)hd * 128 * 128, 128, 128, 128, st);
    hi_lo(L.w2, 5 * kW2Rows * 128, h, l);
    for (int hd = 0; hd < 5; ++hd)
        lsr::launch_pack_weight(net->w2[hd], h + (size_t)hd * kW2Rows * 128, l + (size_t)hd * kW2Rows * 128,
                                kHeadOut[hd], kW2Rows, 128, st);
    // transposed packs (B operands of the backward's data gradients)
    hi_lo(L.wft, 32 * 128, h, l);
    lsr::launch_pack_weight_t(net->w_feat, h, l, 128, 32, 128, st);
    hi_lo(L.w1t, 5 * 128 * 128, h, l);
    for (int hd = 0; hd < 5; ++hd)
        lsr::launch_pack_weight_t(net->w1[hd], h + (size_t)hd * 128 * 128, l + (size_t)hd * 128 * 128, 128, 128, 128, st);
    hi_lo(L.w2t, 5 * 128 * 64, h, l);
    for (int hd = 0; hd < 5; ++hd)
        lsr::launch_pack_weight_t(net->w2[hd], h + (size_t)hd * 128 * 64, l + (size_t)hd * 128 * 64, kHeadOut[hd], 128,
                                  64, st);
    if (hipGetLastError() != hipSuccess) return lsr::fail(LSR_EHIP, "deformation packing launch failed");
    return LSR_OK;
}

namespace {

// forward kernel arguments common to the forward and the backward (planes, packed weights, biases)
lsr::DeformArgs forward_args(const lsr_deform_net* net, const void* workspace, int32_t P) {
    const Layout L = layout(net);
    const char* ws = reinterpret_cast<const char*>(workspace);
    lsr::DeformArgs a{};
    a.P = P;
    a.aabb = net->aabb;
    a.planes = reinterpret_cast<const float*>(ws);
    for (int s = 0; s < 2; ++s)
        for (int ci = 0; ci < 6; ++ci) {
            int W, H;
            plane_dims(net, s, ci, W, H);
            a.poff[6 * s + ci] = (int64_t)(L.plane_off[6 * s + ci] / sizeof(float));
            a.pw[6 * s + ci] = W;
            a.ph[6 * s + ci] = H;
        }
    auto hi_lo = [&](size_t off, size_t count, const __bf16*& hi, const __bf16*& lo) {
        hi = reinterpret_cast<const __bf16*>(ws + off);
        lo = reinterpret_cast<const __bf16*>(ws + off + align256(count * sizeof(__bf16)));
    };
    hi_lo(L.wf, 128 * 32, a.wf_h, a.wf_l);
    hi_lo(L.w1, 5 * 128 * 128, a.w1_h, a.w1_l);
    hi_lo(L.w2, 5 * kW2Rows * 128, a.w2_h, a.w2_l);
    a.b_feat = net->b_feat;
    for (int hd = 0; hd < 5; ++hd) {
        a.b1[hd] = net->b1[hd];
        a.b2[hd] = net->b2[hd];
    }
    return a;
}

// backward scratch: saved activations, then kGradReplicas copies of the packed gradient planes
constexpr int kGradReplicas = 16;
struct BwdScratch {
    size_t X, A0, dH0, A1, dZ1, dplanes, total;
};
BwdScratch bwd_scratch(const lsr_deform_net* net, size_t P) {
    BwdScratch s{};
    size_t o = 0;
    const size_t f = sizeof(float);
    s.X = o; o += align256(P * 32 * f);
    s.A0 = o; o += align256(P * 128 * f);
    s.dH0 = o; o += align256(P * 128 * f);
    s.A1 = o; o += align256(5 * P * 128 * f);
    s.dZ1 = o; o += align256(5 * P * 128 * f);
    s.dplanes = o; o += kGradReplicas * layout(net).planes_end;
    s.total = o;
    return s;
}

}  // namespace

extern "C" int lsr_deform_forward(const lsr_deform_net* net, const void* workspace, int32_t P, const float* means3D,
                                  const float* scales, const float* rotations, const float* opacity,
                                  const float* shs, const float* time, float* out_means3D, float* out_scales,
                                  float* out_rotations, float* out_opacity, float* out_shs, void* stream) {
    int rc = check(net);
    if (rc) return rc;
    if (P < 0) return lsr::fail(LSR_EINVAL, "P must be >= 0");
    if (P == 0) return LSR_OK;
    if (!workspace || !means3D || !scales || !rotations || !opacity || !shs || !time || !out_means3D ||
        !out_scales || !out_rotations || !out_opacity || !out_shs)
        return lsr::fail(LSR_EINVAL, "all inputs, outputs and the workspace are required");
    lsr::DeformArgs a = forward_args(net, workspace, P);
    a.means3D = means3D;
    a.time = time;
    a.in[0] = means3D; a.in[1] = scales; a.in[2] = rotations; a.in[3] = opacity; a.in[4] = shs;
    a.out[0] = out_means3D; a.out[1] = out_scales; a.out[2] = out_rotations; a.out[3] = out_opacity; a.out[4] = out_shs;
    lsr::launch_deform_fwd(a, reinterpret_cast<hipStream_t>(stream));
    if (hipGetLastError() != hipSuccess) return lsr::fail(LSR_EHIP, "deformation forward launch failed");
    return LSR_OK;
}

extern "C" int64_t lsr_deform_backward_scratch_bytes(const lsr_deform_net* net, int32_t P) {
    if (check(net) || P < 0) return -1;
    return (int64_t)bwd_scratch(net, (size_t)(P > 0 ? P : 1)).total;
}

extern "C" int lsr_deform_backward(const lsr_deform_net* net, const void* workspace, int32_t P, const float* means3D,
                                   const float* time, const float* d_out_means3D, const float* d_out_scales,
                                   const float* d_out_rotations, const float* d_out_opacity, const float* d_out_shs,
                                   float* d_means3D, const lsr_deform_grads* grads, void* scratch, void* stream) {
    int rc = check(net);
    if (rc) return rc;
    if (P < 0) return lsr::fail(LSR_EINVAL, "P must be >= 0");
    if (P == 0) return LSR_OK;
    if (!workspace || !means3D || !time || !d_out_means3D || !d_out_scales || !d_out_rotations || !d_out_opacity ||
        !d_out_shs || !d_means3D || !grads || !scratch)
        return lsr::fail(LSR_EINVAL, "inputs, upstream gradients, d_means3D, grads and scratch are required");
    if (!grads->w_feat || !grads->b_feat) return lsr::fail(LSR_EINVAL, "missing feature_out gradients");
    for (int h = 0; h < LSR_DEFORM_HEADS; ++h)
        if (!grads->w1[h] || !grads->b1[h] || !grads->w2[h] || !grads->b2[h])
            return lsr::fail(LSR_EINVAL, "missing head gradients");
    for (int s = 0; s < net->n_scales; ++s)
        for (int ci = 0; ci < 6; ++ci)
            if (!grads->planes[s][ci]) return lsr::fail(LSR_EINVAL, "missing plane gradient");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const Layout L = layout(net);
    const BwdScratch S = bwd_scratch(net, (size_t)P);
    char* sc = reinterpret_cast<char*>(scratch);
    const char* ws = reinterpret_cast<const char*>(workspace);
    lsr::DeformBwdArgs b{};
    b.f = forward_args(net, workspace, P);
    b.f.means3D = means3D;
    b.f.time = time;
    auto hi_lo = [&](size_t off, size_t count, const __bf16*& hi, const __bf16*& lo) {
        hi = reinterpret_cast<const __bf16*>(ws + off);
        lo = reinterpret_cast<const __bf16*>(ws + off + align256(count * sizeof(__bf16)));
    };
    hi_lo(L.wft, 32 * 128, b.wft_h, b.wft_l);
    hi_lo(L.w1t, 5 * 128 * 128, b.w1t_h, b.w1t_l);
    hi_lo(L.w2t, 5 * 128 * 64, b.w2t_h, b.w2t_l);
    b.up[0] = d_out_means3D; b.up[1] = d_out_scales; b.up[2] = d_out_rotations; b.up[3] = d_out_opacity;
    b.up[4] = d_out_shs;
    b.d_means3D = d_means3D;
    b.dplanes = reinterpret_cast<float*>(sc + S.dplanes);
    b.sX = reinterpret_cast<float*>(sc + S.X);
    b.sA0 = reinterpret_cast<float*>(sc + S.A0);
    b.sdH0 = reinterpret_cast<float*>(sc + S.dH0);
    b.sA1 = reinterpret_cast<float*>(sc + S.A1);
    b.sdZ1 = reinterpret_cast<float*>(sc + S.dZ1);
    b.replicas = kGradReplicas;
    b.plane_stride = (int64_t)(L.planes_end / sizeof(float));
    if (hipMemsetAsync(b.dplanes, 0, kGradReplicas * L.planes_end, st) != hipSuccess) return lsr::fail(LSR_EHIP, "memset");
    lsr::launch_deform_bwd_a(b, st);
    // weight gradients: 5 x (dW1, dW2) + feature_out, split-K over ~256 row blocks
    lsr::AtbArgs g{};
    g.P = P;
    const int64_t per = ((int64_t)P + 255) / 256;
    g.rows_per_block = (int)std::max<int64_t>(64, (per + 63) / 64 * 64);
    const size_t PW = (size_t)P * 128;
    for (int hd = 0; hd < 5; ++hd) {
        g.job[hd] = lsr::AtbJob{b.sdZ1 + hd * PW, b.sA0, grads->w1[hd], grads->b1[hd], 128, 128};
        g.job[5 + hd] = lsr::AtbJob{b.up[hd], b.sA1 + hd * PW, grads->w2[hd], grads->b2[hd], kHeadOut[hd], 128};
    }
    g.job[10] = lsr::AtbJob{b.sdH0, b.sX, grads->w_feat, grads->b_feat, 128, 32};
    lsr::launch_atb(g, 11, st);
    for (int s = 0; s < net->n_scales; ++s)
        for (int ci = 0; ci < 6; ++ci) {
            int W, H;
            plane_dims(net, s, ci, W, H);
            lsr::launch_unpack_plane_grad(reinterpret_cast<const float*>(sc + S.dplanes + L.plane_off[6 * s + ci]),
                                          grads->planes[s][ci], H, W, b.replicas, b.plane_stride, st);
        }
    if (hipGetLastError() != hipSuccess) return lsr::fail(LSR_EHIP, "deformation backward launch failed");
    return LSR_OK;
}
