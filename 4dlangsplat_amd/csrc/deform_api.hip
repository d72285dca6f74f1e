// deform_api.hip -- C ABI of the deformation field (include/lsr_deform.h).
#include <hip/hip_runtime.h>

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
    size_t wf, w1, w2;      // bytes: hi arrays, lo right after each
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
    const size_t bf = sizeof(__bf16);
    L.wf = o; o += align256((size_t)128 * 32 * bf) * 2;
    L.w1 = o; o += align256((size_t)5 * 128 * 128 * bf) * 2;
    L.w2 = o; o += align256((size_t)5 * kW2Rows * 128 * bf) * 2;
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
    if (hipGetLastError() != hipSuccess) return lsr::fail(LSR_EHIP, "deformation packing launch failed");
    return LSR_OK;
}

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
    const Layout L = layout(net);
    const char* ws = reinterpret_cast<const char*>(workspace);
    lsr::DeformArgs a{};
    a.P = P;
    a.means3D = means3D;
    a.time = time;
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
    a.in[0] = means3D; a.in[1] = scales; a.in[2] = rotations; a.in[3] = opacity; a.in[4] = shs;
    a.out[0] = out_means3D; a.out[1] = out_scales; a.out[2] = out_rotations; a.out[3] = out_opacity; a.out[4] = out_shs;
    lsr::launch_deform_fwd(a, reinterpret_cast<hipStream_t>(stream));
    if (hipGetLastError() != hipSuccess) return lsr::fail(LSR_EHIP, "deformation forward launch failed");
    return LSR_OK;
}
