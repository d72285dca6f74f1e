// deform_api.hip -- C ABI of the deformation field (include/lsr_deform.h).
#include <atomic>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>

#include "../../include/lsr.h"
#include "../../include/lsr_deform.h"
#include "lsr_internal.h"
#include <cstdlib>
#include <vector>

static_assert(lsr::DEF_UNPACK_MAX == 6 * LSR_DEFORM_MAX_SCALES, "one unpack slot per plane");

namespace lsr {
int fail(int code, const std::string& msg);   // lsr_api.hip (thread-local lsr_last_error)
}

namespace {

constexpr int kCombos[6][2] = {{0, 1}, {0, 2}, {0, 3}, {1, 2}, {1, 3}, {2, 3}};
constexpr int kHeadOut[5] = {3, 3, 4, 1, 48};
constexpr int kW = 128;   // MLP width

size_t align256(size_t x) { return (x + 255) / 256 * 256; }
int nlayers(const lsr_deform_net* n) { return std::max(n->depth, 1); }
int head_out(const lsr_deform_net* n, int hd) { return hd < 5 ? kHeadOut[hd] : n->centers; }
bool head_on(const lsr_deform_net* n, int hd) { return (n->heads >> hd) & 1u; }
int feat_dim(const lsr_deform_net* n) { return 16 * n->n_scales; }
int lang_kin(const lsr_deform_net* n) { return n->lang_dim + 1 + 2 * n->time_pe; }
int lang_kpad(const lsr_deform_net* n) { return (lang_kin(n) + 15) / 16 * 16; }
bool lang_mlp(const lsr_deform_net* n) {
    return n->lang_mode == LSR_DEFORM_LANG_RESIDUAL || n->lang_mode == LSR_DEFORM_LANG_NORESNET;
}
int lang_in(const lsr_deform_net* n) {
    return n->lang_mode == LSR_DEFORM_LANG_DISCRETE ? n->lang_dim * n->centers : n->lang_dim;
}

// plane 6 s + ci: width (along coordinate c0) and height (along c1)
void plane_dims(const lsr_deform_net* n, int s, int ci, int& W, int& H) {
    auto res = [&](int c) { return c < 3 ? n->res[c] * n->multires[s] : n->res[3]; };
    W = res(kCombos[ci][0]);
    H = res(kCombos[ci][1]);
}

// one packed bf16 hi / lo pair of `count` elements
struct Pack {
    size_t off = 0, count = 0;
};
struct Layout {
    size_t plane_off[24];   // bytes
    size_t planes_end;      // bytes of the packed planes
    Pack wf[LSR_DEFORM_MAX_DEPTH], wft[LSR_DEFORM_MAX_DEPTH];
    Pack w1[LSR_DEFORM_HEADS], w2[LSR_DEFORM_HEADS], w1t[LSR_DEFORM_HEADS], w2t[LSR_DEFORM_HEADS];
    Pack wl[3], wlt[3];
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
    auto take = [&](Pack& p, size_t count) {
        p.off = o;
        p.count = count;
        o += align256(count * sizeof(__bf16)) * 2;
    };
    const int F = feat_dim(n), Fpad = (F + 31) / 32 * 32;
    for (int k = 0; k < nlayers(n); ++k) {
        take(L.wf[k], (size_t)kW * (k == 0 ? F : kW));          // [128][K_k]
        take(L.wft[k], (size_t)(k == 0 ? Fpad : kW) * kW);     // [K_k pad 32][128]
    }
    for (int hd = 0; hd < LSR_DEFORM_HEADS; ++hd) {
        if (!head_on(n, hd)) continue;
        take(L.w1[hd], (size_t)kW * kW);
        take(L.w2[hd], (size_t)lsr::DEF_W2ROWS * kW);
        take(L.w1t[hd], (size_t)kW * kW);
        take(L.w2t[hd], (size_t)kW * 64);
    }
    if (lang_mlp(n)) {
        const int kp = lang_kpad(n);
        take(L.wl[0], (size_t)kW * kp);
        take(L.wl[1], (size_t)kW * kW);
        take(L.wl[2], (size_t)32 * kW);
        take(L.wlt[0], (size_t)((kp + 31) / 32 * 32) * kW);
        take(L.wlt[1], (size_t)kW * kW);
        take(L.wlt[2], (size_t)kW * 32);
    }
    L.total = o;
    return L;
}

// the lsr_deform.h version the caller declared (lsr_deform_require_api); 0 = none yet
std::atomic<int> g_deform_caller_api{0};

int check(const lsr_deform_net* n) {
    if (g_deform_caller_api.load() != LSR_DEFORM_API_VERSION)   // the structs' layout is this header's only
        return lsr::fail(LSR_EINVAL, "call lsr_deform_require_api(LSR_DEFORM_API_VERSION) first: the caller must be "
                                     "built against lsr_deform.h version " + std::to_string(LSR_DEFORM_API_VERSION));
    if (!n) return lsr::fail(LSR_EINVAL, "null deformation net");
    if (n->n_scales < 1 || n->n_scales > LSR_DEFORM_MAX_SCALES || n->channels != 16 || n->width != kW)
        return lsr::fail(LSR_EINVAL, "supported: 1..4 scales x 16 channels, width 128 (every HyperNeRF / Neu3D config)");
    if (n->depth < 0 || n->depth > LSR_DEFORM_MAX_DEPTH) return lsr::fail(LSR_EINVAL, "defor_depth must be in [0, 4]");
    for (int c = 0; c < 4; ++c)
        if (n->res[c] < 2) return lsr::fail(LSR_EINVAL, "plane resolutions must be >= 2");
    for (int s = 0; s < n->n_scales; ++s) {
        if (n->multires[s] < 1) return lsr::fail(LSR_EINVAL, "multires must be >= 1");
        for (int ci = 0; ci < 6; ++ci)
            if (!n->planes[s][ci]) return lsr::fail(LSR_EINVAL, "missing plane");
    }
    if (!n->aabb) return lsr::fail(LSR_EINVAL, "missing aabb");
    for (int k = 0; k < nlayers(n); ++k)
        if (!n->w_feat[k] || !n->b_feat[k]) return lsr::fail(LSR_EINVAL, "missing feature_out layer");
    if (n->lang_mode < LSR_DEFORM_LANG_PASS || n->lang_mode > LSR_DEFORM_LANG_DISCRETE)
        return lsr::fail(LSR_EINVAL, "unknown language mode");
    if (n->heads >> LSR_DEFORM_HEADS) return lsr::fail(LSR_EINVAL, "head mask has bits past the 6 heads");
    if (head_on(n, 5) != (n->lang_mode == LSR_DEFORM_LANG_DISCRETE))
        return lsr::fail(LSR_EINVAL, "the coff head (bit 5) runs exactly in the discrete language mode");
    if (n->lang_dim < 0 || n->lang_dim > 32) return lsr::fail(LSR_EINVAL, "lang_dim must be in [0, 32]");
    if (n->lang_mode == LSR_DEFORM_LANG_DISCRETE && (n->centers < 1 || n->centers > 8 || n->lang_dim < 1))
        return lsr::fail(LSR_EINVAL, "discrete mode: centers in [1, 8], lang_dim >= 1");
    if (lang_mlp(n) && (n->lang_dim < 1 || n->time_pe < 0 || lang_kin(n) > 64))
        return lsr::fail(LSR_EINVAL, "lang_deform: lang_dim >= 1 and 2 time_pe + 1 + lang_dim <= 64");
    if (n->apply_rotation && !head_on(n, 2)) return lsr::fail(LSR_EINVAL, "apply_rotation needs the rotation head");
    for (int h = 0; h < LSR_DEFORM_HEADS; ++h)
        if (head_on(n, h) && (!n->w1[h] || !n->b1[h] || !n->w2[h] || !n->b2[h]))
            return lsr::fail(LSR_EINVAL, "missing head weights");
    if (lang_mlp(n))
        for (int k = 0; k < 3; ++k)
            if (!n->w_lang[k] || !n->b_lang[k]) return lsr::fail(LSR_EINVAL, "missing lang_deform weights");
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
    std::vector<lsr::PackJob> jobs;   // every packing job, then one launch (lsr::launch_pack_batch)
    auto plane = [&](const float* src, float* dst, int H, int W) {
        lsr::PackJob q{};
        q.kind = lsr::PACK_PLANE; q.a = H * W; q.src = src; q.hi = dst;
        jobs.push_back(q);
    };
    auto wt = [&](int kind, const float* src, __bf16* h, __bf16* l, int a, int b, int c, int d) {
        lsr::PackJob q{};
        q.kind = kind; q.a = a; q.b = b; q.c = c; q.d = d; q.src = src; q.hi = h; q.lo = l;
        jobs.push_back(q);
    };
    for (int s = 0; s < net->n_scales; ++s)
        for (int ci = 0; ci < 6; ++ci) {
            int W, H;
            plane_dims(net, s, ci, W, H);
            plane(net->planes[s][ci], reinterpret_cast<float*>(ws + L.plane_off[6 * s + ci]), H, W);
        }
    auto hi = [&](const Pack& p) { return reinterpret_cast<__bf16*>(ws + p.off); };
    auto lo = [&](const Pack& p) { return reinterpret_cast<__bf16*>(ws + p.off + align256(p.count * sizeof(__bf16))); };
    const int F = feat_dim(net), Fpad = (F + 31) / 32 * 32;
    constexpr int PW = lsr::PACK_WEIGHT, PT = lsr::PACK_WEIGHT_T;
    for (int k = 0; k < nlayers(net); ++k) {
        const int K = k == 0 ? F : kW;
        wt(PW, net->w_feat[k], hi(L.wf[k]), lo(L.wf[k]), kW, kW, K, K);
        wt(PT, net->w_feat[k], hi(L.wft[k]), lo(L.wft[k]), kW, K, kW, k == 0 ? Fpad : kW);
    }
    for (int hd = 0; hd < LSR_DEFORM_HEADS; ++hd) {
        if (!head_on(net, hd)) continue;
        const int nout = head_out(net, hd);
        wt(PW, net->w1[hd], hi(L.w1[hd]), lo(L.w1[hd]), kW, kW, kW, kW);
        wt(PW, net->w2[hd], hi(L.w2[hd]), lo(L.w2[hd]), nout, lsr::DEF_W2ROWS, kW, kW);
        wt(PT, net->w1[hd], hi(L.w1t[hd]), lo(L.w1t[hd]), kW, kW, kW, kW);
        wt(PT, net->w2[hd], hi(L.w2t[hd]), lo(L.w2t[hd]), nout, kW, 64, kW);
    }
    if (lang_mlp(net)) {
        const int kin = lang_kin(net), kp = lang_kpad(net), C = net->lang_dim;
        wt(PW, net->w_lang[0], hi(L.wl[0]), lo(L.wl[0]), kW, kW, kin, kp);
        wt(PW, net->w_lang[1], hi(L.wl[1]), lo(L.wl[1]), kW, kW, kW, kW);
        wt(PW, net->w_lang[2], hi(L.wl[2]), lo(L.wl[2]), C, 32, kW, kW);
        wt(PT, net->w_lang[0], hi(L.wlt[0]), lo(L.wlt[0]), kW, kin, kW, (kp + 31) / 32 * 32);
        wt(PT, net->w_lang[1], hi(L.wlt[1]), lo(L.wlt[1]), kW, kW, kW, kW);
        wt(PT, net->w_lang[2], hi(L.wlt[2]), lo(L.wlt[2]), C, kW, 32, kW);
    }
    lsr::launch_pack_batch(jobs.data(), (int)jobs.size(), st);
    if (hipGetLastError() != hipSuccess) return lsr::fail(LSR_EHIP, "deformation packing launch failed");
    return LSR_OK;
}

namespace {

template <typename T>
const T* chi(const char* ws, const Pack& p) { return reinterpret_cast<const T*>(ws + p.off); }
template <typename T>
const T* clo(const char* ws, const Pack& p) {
    return reinterpret_cast<const T*>(ws + p.off + align256(p.count * sizeof(__bf16)));
}

// forward kernel arguments common to the forward and the backward (planes, packed weights, biases)
lsr::DeformArgs forward_args(const lsr_deform_net* net, const void* workspace, int32_t P) {
    const Layout L = layout(net);
    const char* ws = reinterpret_cast<const char*>(workspace);
    lsr::DeformArgs a{};
    a.P = P;
    a.n_scales = net->n_scales;
    a.nlayers = nlayers(net);
    a.heads = net->heads;
    a.apply_rotation = net->apply_rotation;
    a.lang_mode = net->lang_mode;
    a.lang_dim = net->lang_dim;
    a.centers = net->centers;
    a.lang_in = lang_in(net);
    a.aabb = net->aabb;
    a.planes = reinterpret_cast<const float*>(ws);
    for (int s = 0; s < net->n_scales; ++s)
        for (int ci = 0; ci < 6; ++ci) {
            int W, H;
            plane_dims(net, s, ci, W, H);
            a.poff[6 * s + ci] = (int64_t)(L.plane_off[6 * s + ci] / sizeof(float));
            a.pw[6 * s + ci] = W;
            a.ph[6 * s + ci] = H;
        }
    for (int k = 0; k < a.nlayers; ++k) {
        a.wf_h[k] = chi<__bf16>(ws, L.wf[k]);
        a.wf_l[k] = clo<__bf16>(ws, L.wf[k]);
        a.b_feat[k] = net->b_feat[k];
    }
    for (int hd = 0; hd < LSR_DEFORM_HEADS; ++hd) {
        if (!head_on(net, hd)) continue;
        a.w1_h[hd] = chi<__bf16>(ws, L.w1[hd]); a.w1_l[hd] = clo<__bf16>(ws, L.w1[hd]);
        a.w2_h[hd] = chi<__bf16>(ws, L.w2[hd]); a.w2_l[hd] = clo<__bf16>(ws, L.w2[hd]);
        a.b1[hd] = net->b1[hd];
        a.b2[hd] = net->b2[hd];
    }
    return a;
}

lsr::LangDeformArgs lang_args(const lsr_deform_net* net, const void* workspace, int32_t P) {
    const Layout L = layout(net);
    const char* ws = reinterpret_cast<const char*>(workspace);
    lsr::LangDeformArgs a{};
    a.P = P;
    a.lang_dim = net->lang_dim;
    a.time_pe = net->time_pe;
    a.kin = lang_kin(net);
    a.residual = net->lang_mode == LSR_DEFORM_LANG_RESIDUAL;
    for (int k = 0; k < 3; ++k) {
        a.w_h[k] = chi<__bf16>(ws, L.wl[k]); a.w_l[k] = clo<__bf16>(ws, L.wl[k]);
        a.wt_h[k] = chi<__bf16>(ws, L.wlt[k]); a.wt_l[k] = clo<__bf16>(ws, L.wlt[k]);
        a.b[k] = net->b_lang[k];
    }
    return a;
}

// backward scratch: saved activations, then deform_replicas(P) copies of the packed gradient planes
constexpr int kGradReplicas = 16;   // the most LSR_DEFORM_REPLICAS may ask for
// Replica count of a call (every copy is zeroed and summed by the unpack, 9.5 MB each for the Neu3D
// planes).  LSR_DEFORM_REPLICAS overrides (diagnostic A/B).
int deform_replicas(size_t P) {
    static const int forced = [] {
        const char* e = std::getenv("LSR_DEFORM_REPLICAS");
        return e ? std::max(1, std::min(kGradReplicas, std::atoi(e))) : 0;
    }();
    if (forced) return forced;
    // measured (tools/gpu.sh deform_ab): 4 copies backward 12.20 vs 12.22 ms at 2M (the atomics do
    // not contend more), configs[4] stand-in 159 vs 139-152 iterations/s at 100k (less to zero and sum);
    // with the time planes through x-rows (round 5, tools/gpu.sh deform_ab) 2 copies 10.08 vs 10.12
    // ms at 2M and 1.257-1.261 vs 1.257-1.273 ms per configs[4] iteration, 8 copies 10.10-10.19 / 1.29
    (void)P;
    return 2;
}
struct BwdScratch {
    size_t X, A[LSR_DEFORM_MAX_DEPTH], dH[LSR_DEFORM_MAX_DEPTH];
    size_t Grot, Gcoff, U0, U1, U2, dv, dZ2l, dZ1l, daabb, dplanes, trow, total;
};
// the time planes' x-rows (DeformBwdArgs.trow): copies, their floats, each plane's offset (-1: not a
// time plane).  LSR_DEFORM_TIME_ROWS=0 turns them off (A/B).
constexpr int kTimeRowReps = 32;
int time_row_reps() {   // LSR_DEFORM_TIME_ROWS=n (A/B): n copies, 0 = off
    static const int reps = [] {
        const char* e = std::getenv("LSR_DEFORM_TIME_ROWS");
        return e ? std::max(0, std::min(256, std::atoi(e))) : kTimeRowReps;
    }();
    return reps;
}
size_t time_row_floats(const lsr_deform_net* net, int64_t* toff) {
    size_t o = 0;
    for (int s = 0; s < net->n_scales; ++s)
        for (int ci = 0; ci < 6; ++ci) {
            int W, H;
            plane_dims(net, s, ci, W, H);
            const bool tp = ci == 2 || ci >= 4;
            if (toff) toff[6 * s + ci] = tp ? (int64_t)o : -1;
            if (tp) o += (size_t)W * 16;
        }
    return o;
}
BwdScratch bwd_scratch(const lsr_deform_net* net, size_t P) {
    BwdScratch s{};
    size_t o = 0;
    const size_t f = sizeof(float);
    auto take = [&](size_t floats) {
        const size_t at = o;
        o += align256(floats * f);
        return at;
    };
    s.X = take(P * feat_dim(net));
    for (int k = 0; k < nlayers(net); ++k) {
        s.A[k] = take(P * kW);
        s.dH[k] = take(P * kW);
    }
    s.Grot = take(net->apply_rotation ? P * 4 : 1);
    s.Gcoff = take(net->lang_mode == LSR_DEFORM_LANG_DISCRETE ? P * net->centers : 1);
    if (lang_mlp(net)) {
        s.U0 = take(P * lang_kin(net));
        s.U1 = take(P * kW);
        s.U2 = take(P * kW);
        s.dv = take(P * net->lang_dim);
        s.dZ2l = take(P * kW);
        s.dZ1l = take(P * kW);
    }
    s.daabb = take(lsr::DEF_AABB_SLOTS * 16);   // zeroed with the gradient planes (contiguous)
    s.dplanes = o;
    o += (size_t)deform_replicas(P) * layout(net).planes_end;   // the count every call of this process uses
    s.trow = o;                                                  // zeroed with the planes (contiguous)
    o += align256((size_t)time_row_reps() * time_row_floats(net, nullptr) * f);
    s.total = o;
    return s;
}

}  // namespace

extern "C" int lsr_deform_require_api(int32_t caller_version) {
    if (caller_version != LSR_DEFORM_API_VERSION)
        return lsr::fail(LSR_EINVAL, "lsr_deform.h version mismatch: caller " + std::to_string(caller_version) +
                                         ", library " + std::to_string(LSR_DEFORM_API_VERSION));
    g_deform_caller_api.store(caller_version);
    return LSR_OK;
}

extern "C" int lsr_deform_forward(const lsr_deform_net* net, const void* workspace, int32_t P, const float* means3D,
                                  const float* scales, const float* rotations, const float* opacity,
                                  const float* shs, const float* lang, const float* time, float* out_means3D,
                                  float* out_scales, float* out_rotations, float* out_opacity, float* out_shs,
                                  float* out_lang, float* out_coff, void* stream) {
    int rc = check(net);
    if (rc) return rc;
    if (P < 0) return lsr::fail(LSR_EINVAL, "P must be >= 0");
    if (P == 0) return LSR_OK;
    const float* ins[5] = {means3D, scales, rotations, opacity, shs};
    float* outs[5] = {out_means3D, out_scales, out_rotations, out_opacity, out_shs};
    if (!workspace || !means3D || !time) return lsr::fail(LSR_EINVAL, "workspace, means3D and time are required");
    for (int hd = 0; hd < 5; ++hd)
        if (head_on(net, hd) && (!ins[hd] || !outs[hd]))
            return lsr::fail(LSR_EINVAL, "the input and output of every computed head are required");
    if (net->lang_mode != LSR_DEFORM_LANG_PASS && (!lang || !out_lang))
        return lsr::fail(LSR_EINVAL, "lang and out_lang are required unless the language passes through");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    lsr::DeformArgs a = forward_args(net, workspace, P);
    a.means3D = means3D;
    a.time = time;
    a.lang = lang;
    for (int hd = 0; hd < 5; ++hd) {
        a.in[hd] = ins[hd];
        a.out[hd] = outs[hd];
    }
    a.out_lang = out_lang;
    a.out_coff = out_coff;
    lsr::launch_deform_fwd(a, st);
    if (lang_mlp(net)) {
        lsr::LangDeformArgs la = lang_args(net, workspace, P);
        la.lang = lang;
        la.time = time;
        la.out_lang = out_lang;
        lsr::launch_lang_deform_fwd(la, st);
    }
    if (hipGetLastError() != hipSuccess) return lsr::fail(LSR_EHIP, "deformation forward launch failed");
    return LSR_OK;
}

extern "C" int64_t lsr_deform_backward_scratch_bytes(const lsr_deform_net* net, int32_t P) {
    if (check(net) || P < 0) return -1;
    return (int64_t)bwd_scratch(net, (size_t)(P > 0 ? P : 1)).total;
}

extern "C" int lsr_deform_backward(const lsr_deform_net* net, const void* workspace, int32_t P, const float* means3D,
                                   const float* rotations, const float* lang, const float* time,
                                   const float* d_out_means3D, const float* d_out_scales, const float* d_out_rotations,
                                   const float* d_out_opacity, const float* d_out_shs, const float* d_out_lang,
                                   const float* d_out_coff, float* d_means3D, float* d_rotations, float* d_lang,
                                   const lsr_deform_grads* grads, void* scratch, void* stream) {
    int rc = check(net);
    if (rc) return rc;
    if (P < 0) return lsr::fail(LSR_EINVAL, "P must be >= 0");
    if (P == 0) return LSR_OK;
    const float* ups[5] = {d_out_means3D, d_out_scales, d_out_rotations, d_out_opacity, d_out_shs};
    if (!workspace || !means3D || !time || !d_out_means3D || !d_means3D || !grads || !scratch)
        return lsr::fail(LSR_EINVAL, "means3D, time, d_out_means3D, d_means3D, grads, scratch and the workspace are "
                                     "required");
    for (int hd = 0; hd < 5; ++hd)
        if (head_on(net, hd) && !ups[hd]) return lsr::fail(LSR_EINVAL, "the gradient of every computed head's output is required");
    if (net->apply_rotation && (!rotations || !d_rotations))
        return lsr::fail(LSR_EINVAL, "apply_rotation: rotations and d_rotations are required");
    if (net->lang_mode != LSR_DEFORM_LANG_PASS && (!lang || !d_lang))
        return lsr::fail(LSR_EINVAL, "lang and d_lang are required unless the language passes through");
    for (int k = 0; k < nlayers(net); ++k)
        if (!grads->w_feat[k] || !grads->b_feat[k]) return lsr::fail(LSR_EINVAL, "missing feature_out gradients");
    for (int h = 0; h < LSR_DEFORM_HEADS; ++h)
        if (head_on(net, h) && (!grads->w1[h] || !grads->b1[h] || !grads->w2[h] || !grads->b2[h]))
            return lsr::fail(LSR_EINVAL, "missing head gradients");
    if (lang_mlp(net))
        for (int k = 0; k < 3; ++k)
            if (!grads->w_lang[k] || !grads->b_lang[k]) return lsr::fail(LSR_EINVAL, "missing lang_deform gradients");
    for (int s = 0; s < net->n_scales; ++s)
        for (int ci = 0; ci < 6; ++ci)
            if (!grads->planes[s][ci]) return lsr::fail(LSR_EINVAL, "missing plane gradient");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const Layout L = layout(net);
    const BwdScratch S = bwd_scratch(net, (size_t)P);
    char* sc = reinterpret_cast<char*>(scratch);
    const char* ws = reinterpret_cast<const char*>(workspace);
    auto fp = [&](size_t off) { return reinterpret_cast<float*>(sc + off); };
    lsr::DeformBwdArgs b{};
    b.f = forward_args(net, workspace, P);
    b.f.means3D = means3D;
    b.f.time = time;
    b.f.lang = lang;
    b.f.in[2] = rotations;
    for (int k = 0; k < b.f.nlayers; ++k) {
        b.wft_h[k] = chi<__bf16>(ws, L.wft[k]); b.wft_l[k] = clo<__bf16>(ws, L.wft[k]);
        b.sA[k] = fp(S.A[k]);
        b.sdH[k] = fp(S.dH[k]);
    }
    for (int hd = 0; hd < LSR_DEFORM_HEADS; ++hd) {
        if (!head_on(net, hd)) continue;
        b.w1t_h[hd] = chi<__bf16>(ws, L.w1t[hd]); b.w1t_l[hd] = clo<__bf16>(ws, L.w1t[hd]);
        b.w2t_h[hd] = chi<__bf16>(ws, L.w2t[hd]); b.w2t_l[hd] = clo<__bf16>(ws, L.w2t[hd]);
    }
    for (int hd = 0; hd < 5; ++hd) b.up[hd] = ups[hd];
    b.up_lang = d_out_lang;
    b.up_coff = d_out_coff;
    b.d_means3D = d_means3D;
    b.d_rotations = d_rotations;
    b.d_lang = d_lang;
    b.sX = fp(S.X);
    b.sG_rot = fp(S.Grot);
    b.sG_coff = fp(S.Gcoff);
    b.dplanes = fp(S.dplanes);
    b.daabb = grads->aabb;
    b.daabb_part = fp(S.daabb);
    b.replicas = deform_replicas((size_t)P);
    b.plane_stride = (int64_t)(L.planes_end / sizeof(float));
    b.trow_reps = time_row_reps();
    b.trow = b.trow_reps ? fp(S.trow) : nullptr;
    b.trow_stride = (int64_t)time_row_floats(net, b.toff);
    if (hipMemsetAsync(sc + S.daabb, 0, S.total - S.daabb, st) != hipSuccess)
        return lsr::fail(LSR_EHIP, "memset");
    lsr::launch_deform_bwd_a(b, st);
    lsr::LangDeformArgs la{};
    if (lang_mlp(net)) {
        la = lang_args(net, workspace, P);
        la.lang = lang;
        la.time = time;
        la.up_lang = d_out_lang;
        la.d_lang = d_lang;
        la.sU0 = fp(S.U0); la.sU1 = fp(S.U1); la.sU2 = fp(S.U2);
        la.sdv = fp(S.dv); la.sdZ2 = fp(S.dZ2l); la.sdZ1 = fp(S.dZ1l);
        lsr::launch_lang_deform_bwd(la, st);
    }
    // weight gradients, split-K over row blocks: the feature_out chain and lang_deform as A^T B
    // products of saved rows (k_atb); every computed head by recompute from the trunk's last
    // activation (k_head_wgrad: no per-head rows saved)
    lsr::AtbArgs g{};
    g.P = P;
    // ~1024 blocks per job (4 per CU: the per-block row loops are latency-bound; 256 blocks measured
    // 11.20 vs 10.92-10.95 ms for the 2M backward)
    const int64_t per = ((int64_t)P + 1023) / 1024;
    g.rows_per_block = (int)std::max<int64_t>(64, (per + 63) / 64 * 64);
    int nj = 0;
    const int F = feat_dim(net);
    for (int k = 0; k < b.f.nlayers; ++k)
        g.job[nj++] = lsr::AtbJob{b.sdH[k], k == 0 ? b.sX : b.sA[k - 1], grads->w_feat[k], grads->b_feat[k], kW,
                                  k == 0 ? F : kW};
    lsr::HeadWgradArgs hw{};
    hw.A = b.sA[b.f.nlayers - 1];
    hw.P = P;
    int nh = 0;
    for (int hd = 0; hd < LSR_DEFORM_HEADS; ++hd) {
        if (!head_on(net, hd)) continue;
        const float* G = hd == 5 ? b.sG_coff : (hd == 2 && net->apply_rotation) ? b.sG_rot : ups[hd];
        hw.job[nh++] = lsr::HeadWgradJob{G, b.f.w1_h[hd], b.f.w1_l[hd], b.f.b1[hd], b.w2t_h[hd], b.w2t_l[hd],
                                         b.f.w2_h[hd], b.f.w2_l[hd], grads->w1[hd], grads->b1[hd], grads->w2[hd],
                                         grads->b2[hd], head_out(net, hd)};
    }
    lsr::launch_head_wgrad(hw, nh, st);
    if (lang_mlp(net)) {
        g.job[nj++] = lsr::AtbJob{la.sdZ1, la.sU0, grads->w_lang[0], grads->b_lang[0], kW, la.kin};
        g.job[nj++] = lsr::AtbJob{la.sdZ2, la.sU1, grads->w_lang[1], grads->b_lang[1], kW, kW};
        g.job[nj++] = lsr::AtbJob{la.sdv, la.sU2, grads->w_lang[2], grads->b_lang[2], net->lang_dim, kW};
    }
    lsr::launch_atb(g, nj, st);
    lsr::UnpackBatch u{};
    u.src = fp(S.dplanes);
    u.replicas = b.replicas;
    u.stride = b.plane_stride;
    u.daabb_part = b.daabb_part;
    u.daabb = grads->aabb;
    u.trow = b.trow;
    u.trow_reps = b.trow_reps;
    u.trow_stride = b.trow_stride;
    u.time0 = time;
    for (int s = 0; s < net->n_scales; ++s)
        for (int ci = 0; ci < 6; ++ci) {
            int W, H;
            plane_dims(net, s, ci, W, H);
            const int j = u.n++;
            u.off[j] = (int64_t)(L.plane_off[6 * s + ci] / sizeof(float));
            u.toff[j] = b.toff[6 * s + ci];
            u.dst[j] = grads->planes[s][ci];
            u.H[j] = H;
            u.W[j] = W;
            u.block0[j + 1] = u.block0[j] + (H * W + 15) / 16;
        }
    lsr::launch_unpack_planes(u, st);
    if (hipGetLastError() != hipSuccess) return lsr::fail(LSR_EHIP, "deformation backward launch failed");
    return LSR_OK;
}
