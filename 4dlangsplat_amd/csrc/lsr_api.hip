// lsr_api.hip -- the C ABI (include/lsr.h): argument checks, workspace carving, launch order.
//
// Forward  = preprocess -> depth sort of the P Gaussians -> tile counts in depth order -> scan
//            -> (host reads K) -> emit K instances -> stable tile sort -> tile ranges -> composite.
// Backward = composite backward (per-Gaussian screen-space sums) -> preprocess backward.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/lsr.h"
#include "lsr_common.h"
#include "lsr_internal.h"

namespace {

thread_local std::string g_err;
std::atomic<int32_t> g_caller_api{0};   // lsr_require_api: the lsr.h version the caller was built against

int fail(int code, const std::string& msg) {
    g_err = msg;
    return code;
}

#define LSR_HIP(expr)                                                                        \
    do {                                                                                     \
        hipError_t e_ = (expr);                                                              \
        if (e_ != hipSuccess) return fail(LSR_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define LSR_LAUNCHED(name, st, debug)                                                        \
    do {                                                                                     \
        hipError_t e_ = hipGetLastError();                                                   \
        if (e_ == hipSuccess && (debug)) e_ = hipStreamSynchronize(st);                      \
        if (e_ != hipSuccess) return fail(LSR_EHIP, std::string(name) + ": " + hipGetErrorString(e_)); \
    } while (0)

// ---- per-phase event timing (lsr_profile_*) ----------------------------------------------------
struct Profiler {
    std::mutex mu;
    bool on = false;
    uint32_t mask = ~0u;   // phases timed while on (bit LSR_PHASE_*)
    std::vector<hipEvent_t> pool;
    struct Rec { int phase; hipEvent_t a, b; };
    std::vector<Rec> pending;
    double ms[LSR_NUM_PHASES] = {};
    int64_t n[LSR_NUM_PHASES] = {};
    hipEvent_t get() {
        if (!pool.empty()) { hipEvent_t e = pool.back(); pool.pop_back(); return e; }
        hipEvent_t e = nullptr;
        if (hipEventCreate(&e) != hipSuccess) return nullptr;
        return e;
    }
};
Profiler g_prof;

struct PhaseTimer {
    int phase;
    hipStream_t st;
    hipEvent_t a = nullptr, b = nullptr;
    PhaseTimer(int p, hipStream_t s) : phase(p), st(s) {
        std::lock_guard<std::mutex> l(g_prof.mu);
        if (!g_prof.on || !((g_prof.mask >> p) & 1u)) return;
        a = g_prof.get();
        b = g_prof.get();
        if (a) (void)hipEventRecord(a, st);
    }
    ~PhaseTimer() {
        if (!a || !b) return;
        (void)hipEventRecord(b, st);
        std::lock_guard<std::mutex> l(g_prof.mu);
        g_prof.pending.push_back({phase, a, b});
    }
};

constexpr size_t kAlign = 256;
inline size_t al(size_t x) { return (x + kAlign - 1) / kAlign * kAlign; }

// Bump allocator over a caller-owned workspace; the same carve order gives the size query.
struct Carver {
    char* base;
    size_t off = 0;
    explicit Carver(void* b) : base(static_cast<char*>(b)) {}
    template <typename T>
    T* take(size_t n) {
        T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
        off += al(n * sizeof(T));
        return p;
    }
};

struct Geom {
    float2* xy;
    float4* conic_o;
    float4* rgbd;
    uint8_t* clamped;
    uint32_t* tiles;
    uint32_t *key_a, *key_b, *val_a, *val_b;
    uint32_t* counts;
    uint32_t* offsets;
    uint32_t* inst_off;
    int* radius;
    uint2* rect;          // by id, written by preprocess
    uint2* rect_sorted;   // depth order
    uint32_t* total;
    void* sort_tmp;
    void* scan_tmp;
    float4* acc;          // [P, ACC_PITCH] split-backward accumulators (rows of listed Gaussians
                          // zeroed by the preprocess; lsr_backward_composite adds into them)
};
Geom carve_geom(void* base, size_t P, size_t* bytes) {
    Carver c(base);
    Geom g;
    g.xy = c.take<float2>(P);
    g.conic_o = c.take<float4>(P);
    g.rgbd = c.take<float4>(P);
    g.clamped = c.take<uint8_t>(P);
    g.tiles = c.take<uint32_t>(P);
    g.key_a = c.take<uint32_t>(P);
    g.key_b = c.take<uint32_t>(P);
    g.val_a = c.take<uint32_t>(P);
    g.val_b = c.take<uint32_t>(P);
    g.counts = c.take<uint32_t>(P);
    g.offsets = c.take<uint32_t>(P);
    g.inst_off = c.take<uint32_t>(P);
    g.radius = c.take<int>(P);
    g.rect = c.take<uint2>(P);
    g.rect_sorted = c.take<uint2>(P);
    g.total = c.take<uint32_t>(4);
    g.sort_tmp = c.take<char>(lsr::radix_temp_bytes(P));
    g.scan_tmp = c.take<char>(lsr::scan_temp_bytes(P));
    g.acc = c.take<float4>(P * (lsr::ACC_PITCH / 4));
    if (bytes) *bytes = c.off;
    return g;
}

struct Binning {
    uint32_t *key_a, *key_b, *val_a, *val_b;
    void* sort_tmp;
    uint32_t* kept;   // the tile sort's listed-instance count (its first pass drops the unlisted)
};
Binning carve_binning(void* base, size_t K, size_t* bytes) {
    Carver c(base);
    Binning b;
    b.key_a = c.take<uint32_t>(K);
    b.key_b = c.take<uint32_t>(K);
    b.val_a = c.take<uint32_t>(K);
    b.val_b = c.take<uint32_t>(K);
    b.sort_tmp = c.take<char>(lsr::radix_temp_bytes(K));
    b.kept = c.take<uint32_t>(4);
    if (bytes) *bytes = c.off;
    return b;
}

// the tile-bucket binning's workspace: the sort path's layout (its point list buffer is where the
// compositors read; key_a..key_b hold the 64-bit bucket keys: 8K bytes <= 2 al(4K)), then the
// per-block tile count table and the long buckets' merge workspace
struct BinningTb {
    Binning b;
    uint32_t* table;
    uint64_t* tmp;
};
BinningTb carve_binning_tb(void* base, size_t K, size_t P, size_t ntiles, size_t* bytes) {
    size_t head;
    BinningTb t;
    t.b = carve_binning(base, K, &head);
    Carver c(base);
    c.off = head;
    t.table = c.take<uint32_t>((size_t)lsr::tb_blocks((int)P) * ntiles);
    t.tmp = c.take<uint64_t>(K);
    if (bytes) *bytes = c.off;
    return t;
}

struct Img {
    uint2* ranges;
    uint32_t* tile_max;
    float* final_T;
    uint32_t* n_contrib;
    uint32_t* tile_order;   // backward scratch: tiles by descending replay length
};
Img carve_img(void* base, int W, int H, size_t* bytes) {
    const size_t gx = (W + LSR_TILE_X - 1) / LSR_TILE_X, gy = (H + LSR_TILE_Y - 1) / LSR_TILE_Y;
    Carver c(base);
    Img m;
    m.ranges = c.take<uint2>(gx * gy);
    m.tile_max = c.take<uint32_t>(gx * gy);
    m.final_T = c.take<float>((size_t)W * H);
    m.n_contrib = c.take<uint32_t>((size_t)W * H);
    m.tile_order = c.take<uint32_t>(gx * gy);
    if (bytes) *bytes = c.off;
    return m;
}

struct Scratch {
    float* acc_small;    // [P,12] atomic mode accumulators (zeroed per call)
    float* rec;          // [K, record_floats(C)] deterministic mode records
    uint8_t* flags;      // [K] record written
};
Scratch carve_scratch(void* base, size_t P, size_t K, int recq, bool det, size_t* bytes) {
    Carver c(base);
    Scratch s{};
    if (det) {
        s.rec = c.take<float>(K * (size_t)recq);
        s.flags = c.take<uint8_t>(K);
    } else {
        s.acc_small = c.take<float>(P * lsr::ACC_PITCH);
    }
    if (bytes) *bytes = c.off;
    return s;
}

// tile-sort key bits: keys are tile ids 0..ntiles-1 plus ntiles for instances whose splat
// reaches no quadrant of their tile (binning.hip k_emit): they sort past every tile's list
int tile_bits(int ntiles) {
    int b = 1;
    while ((1 << b) <= ntiles) ++b;
    return b;
}
bool tile_sort_in_b(int ntiles) { return ((tile_bits(ntiles) + 7) / 8) % 2 == 1; }
int depth_sort_result_in_b() { return 0; }  // 4 passes, or 3 planned on the device: either way in the (a) buffers

int check_common(const lsr_settings* s, const lsr_fwd_in* in) {
    if (g_caller_api.load() != LSR_API_VERSION)   // the structs' layout is that of this lsr.h only
        return fail(LSR_EINVAL, "call lsr_require_api(LSR_API_VERSION) first: the caller must be built against lsr.h "
                                "version " + std::to_string(LSR_API_VERSION));
    if (!s || !in) return fail(LSR_EINVAL, "null settings or inputs");
    if (s->image_width <= 0 || s->image_height <= 0) return fail(LSR_EINVAL, "image size must be positive");
    if (s->image_width > 4095 * LSR_TILE_X || s->image_height > 4095 * LSR_TILE_Y)
        return fail(LSR_EINVAL, "image size exceeds 4095 tiles per axis");
    if (in->P < 0) return fail(LSR_EINVAL, "P must be >= 0");
    // point lists carry 28-bit Gaussian ids (the top 4 bits: the tile's quadrants the splat may
    // reach) and the compositors address rows with 32-bit byte offsets
    if (in->P >= (1 << 28)) return fail(LSR_EINVAL, "P must be < 2^28");
    if ((uint64_t)in->P * (uint64_t)(in->C > 16 ? in->C : 16) * 4u >= (1ull << 32))
        return fail(LSR_EINVAL, "P * max(C, 16) * 4 bytes must be < 2^32");
    if (!s->viewmatrix || !s->projmatrix || !s->bg || !s->campos)
        return fail(LSR_EINVAL, "viewmatrix, projmatrix, bg and campos are required");
    if (in->P > 0 && (!in->means3D || !in->opacities)) return fail(LSR_EINVAL, "means3D and opacities are required");
    if (in->P == 0) return LSR_OK;   // nothing to validate or render (upstream returns early too)
    if ((in->shs == nullptr) == (in->colors_precomp == nullptr))
        return fail(LSR_EINVAL, "Please provide excatly one of either SHs or precomputed colors!");
    const bool sr = in->scales != nullptr || in->rotations != nullptr;
    if ((!(in->scales && in->rotations) && !in->cov3D_precomp) || (sr && in->cov3D_precomp))
        return fail(LSR_EINVAL, "Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!");
    if (in->shs && (s->sh_degree < 0 || s->sh_degree > 3 || in->M < (s->sh_degree + 1) * (s->sh_degree + 1)))
        return fail(LSR_EINVAL, "sh_degree must be in [0, 3] and shs must hold (sh_degree + 1)^2 coefficients");
    if (in->C < 0 || in->C > 64) return fail(LSR_EINVAL, "language feature channels must be in [0, 64]");
    if (s->include_feature && in->C > 0 && in->P > 0 && !in->language_feature)
        return fail(LSR_EINVAL, "language_feature is required when C > 0");
    return LSR_OK;
}

// The Gaussians' side of a preprocess launch (shared by its views).
void preprocess_shared(lsr::PreprocessArgs& a, const lsr_settings* s, const lsr_fwd_in* in) {
    const int W = s->image_width, H = s->image_height;
    a.P = in->P; a.M = in->M; a.deg = s->sh_degree; a.W = W; a.H = H;
    a.grid_x = (W + LSR_TILE_X - 1) / LSR_TILE_X; a.grid_y = (H + LSR_TILE_Y - 1) / LSR_TILE_Y;
    a.scale_modifier = s->scale_modifier;
    a.means3D = in->means3D; a.scales = in->scales; a.rotations = in->rotations; a.opacities = in->opacities;
    a.shs = in->shs; a.colors_precomp = in->colors_precomp; a.cov3D_precomp = in->cov3D_precomp;
}
// One view's camera and outputs.  The preprocess also writes the depth sort's initial values
// (ids), zeroes the split-backward accumulator rows of listed Gaussians, and clears the counters
// [0] K, [1..2] reserved (reported as 0), [3] visible count: no separate fill launches.
void preprocess_view(lsr::PreprocessView& v, const lsr_settings* s, const Geom& g, int* radii) {
    v.tanfovx = s->tanfovx; v.tanfovy = s->tanfovy;
    v.focal_x = (float)s->image_width / (2.0f * s->tanfovx);
    v.focal_y = (float)s->image_height / (2.0f * s->tanfovy);
    v.view = s->viewmatrix; v.proj = s->projmatrix; v.campos = s->campos;
    v.radii = radii; v.radius = g.radius; v.tiles = g.tiles; v.rect = g.rect; v.key = g.key_a; v.xy = g.xy;
    v.conic_o = g.conic_o; v.rgbd = g.rgbd; v.clamped = g.clamped;
    v.order = g.val_a;
    v.rank_counts = g.counts;
    v.acc = g.acc;
    v.clear.p[0] = g.total;
    v.clear.n[0] = 4;
}

}  // namespace

extern "C" {

int lsr_version(void) { return LSR_API_VERSION; }
int lsr_require_api(int32_t caller_version) {
    if (caller_version != LSR_API_VERSION)
        return fail(LSR_EINVAL, "lsr.h version mismatch: caller " + std::to_string(caller_version) + ", library " +
                                    std::to_string(LSR_API_VERSION));
    g_caller_api.store(caller_version);
    return LSR_OK;
}
const char* lsr_last_error(void) { return g_err.c_str(); }

int64_t lsr_geom_bytes(int32_t P) {
    size_t b;
    carve_geom(nullptr, (size_t)(P > 0 ? P : 1), &b);
    return (int64_t)b;
}
int64_t lsr_binning_bytes(int64_t K) {
    size_t b;
    carve_binning(nullptr, (size_t)(K > 0 ? K : 1), &b);
    return (int64_t)b;
}
int64_t lsr_binning_bytes_tb(int64_t K, int32_t P, int32_t W, int32_t H) {
    if (W <= 0 || H <= 0 || P < 0) return -1;
    const size_t ntiles = (size_t)((W + LSR_TILE_X - 1) / LSR_TILE_X) * ((H + LSR_TILE_Y - 1) / LSR_TILE_Y);
    size_t b;
    carve_binning_tb(nullptr, (size_t)(K > 0 ? K : 1), (size_t)(P > 0 ? P : 1), ntiles, &b);
    return (int64_t)b;
}
int64_t lsr_img_bytes(int32_t W, int32_t H) {
    size_t b;
    carve_img(nullptr, W, H, &b);
    return (int64_t)b;
}
int64_t lsr_backward_bytes(int32_t P, int64_t K, int32_t C, int32_t deterministic) {
    size_t b;
    carve_scratch(nullptr, (size_t)(P > 0 ? P : 1), (size_t)(K > 0 ? K : 1), lsr::record_floats(C > 0 ? C : 0),
                  deterministic != 0, &b);
    return (int64_t)b;
}

int lsr_forward_preprocess_async(const lsr_settings* s, const lsr_fwd_in* in, lsr_fwd_out* out, void* geom,
                                 uint32_t* host_count, lsr_stream_t stream) {
    int rc = check_common(s, in);
    if (rc) return rc;
    if (!out || (!out->radii && in->P > 0)) return fail(LSR_EINVAL, "radii output is required");
    if (!geom || !host_count) return fail(LSR_EINVAL, "geom workspace and host_count are required");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int P = in->P;
    Geom g = carve_geom(geom, (size_t)(P > 0 ? P : 1), nullptr);
    if (P == 0) {
        host_count[0] = host_count[1] = 0;
        return LSR_OK;
    }
    lsr::PreprocessArgs a{};
    preprocess_shared(a, s, in);
    a.nv = 1;
    preprocess_view(a.v[0], s, g, out->radii);
    {
        PhaseTimer t(LSR_PHASE_PREPROCESS, st);
        lsr::launch_preprocess(a, st);
    }
    LSR_LAUNCHED("preprocess", st, s->debug);
    // depth order of all Gaussians (culled ones carry key 0xFFFFFFFF and sort last), stable in id
    bool in_b;
    {
        PhaseTimer t(LSR_PHASE_DEPTH_SORT, st);
        // culled Gaussians (key 0xFFFFFFFF) are dropped by the first pass: the visible count goes
        // to g.total[3] and only those are sorted (and gathered below)
        // ... and its last pass writes the depth-ranked rectangles and instance counts (the ranks
        // of culled Gaussians keep the zero counts the preprocess wrote)
        const lsr::SortGather gather{g.rect, g.counts, g.rect_sorted};
        in_b = lsr::radix_sort_pairs(g.key_a, g.val_a, g.key_b, g.val_b, (size_t)P, 0, 32, g.sort_tmp, st, g.total + 3,
                                     &gather, g.offsets);   // offsets: free until the instance scan
    }
    if (in_b != (bool)depth_sort_result_in_b()) return fail(LSR_EHIP, "internal: depth sort parity");
    LSR_LAUNCHED("depth sort", st, s->debug);
    {
        PhaseTimer t(LSR_PHASE_INSTANCE_SCAN, st);
        lsr::exclusive_scan_u32(g.counts, g.offsets, (size_t)P, g.total, g.scan_tmp, st);
    }
    LSR_LAUNCHED("instance scan", st, s->debug);
    LSR_HIP(hipMemcpyAsync(host_count, g.total, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost, st));
    return LSR_OK;
}

namespace {
int check_views(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in, void* const* geom) {
    if (n_views < 1 || !s || !geom) return fail(LSR_EINVAL, "n_views >= 1 and the per-view arrays are required");
    for (int v = 0; v < n_views; ++v) {
        int rc = check_common(s[v], in);
        if (rc) return rc;
        if (!geom[v]) return fail(LSR_EINVAL, "geom workspaces are required");
        if (s[v]->image_width != s[0]->image_width || s[v]->image_height != s[0]->image_height ||
            s[v]->sh_degree != s[0]->sh_degree || s[v]->scale_modifier != s[0]->scale_modifier)
            return fail(LSR_EINVAL, "batched views must share the image size, sh_degree and scale_modifier");
    }
    return LSR_OK;
}

// depth order + instance count of n_views preprocessed views (their geom workspaces), one set of
// launches per 8 views; page-locked host_counts get the counts from the scan itself
int depth_order_views(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in, void* const* geom,
                      uint32_t* host_counts, hipStream_t st) {
    const int P = in->P;
    uint32_t* mapped = nullptr;
    {
        void* dptr = nullptr;
        if (hipHostGetDevicePointer(&dptr, host_counts, 0) == hipSuccess && dptr) mapped = static_cast<uint32_t*>(dptr);
        else (void)hipGetLastError();   // clear the sticky error of the failed query
    }
    for (int v0 = 0; v0 < n_views; v0 += lsr::LSR_MAX_VIEWS) {
        const int nv = std::min(n_views - v0, lsr::LSR_MAX_VIEWS);
        lsr::SortSeg ss[lsr::LSR_MAX_VIEWS] = {};
        lsr::ScanSeg sc[lsr::LSR_MAX_VIEWS] = {};
        for (int k = 0; k < nv; ++k) {
            Geom g = carve_geom(geom[v0 + k], (size_t)P, nullptr);
            // depth order of the visible Gaussians (the first pass drops culled keys, kept count in
            // g.total[3]; the last pass writes the depth-ranked rectangles and instance counts)
            ss[k] = lsr::SortSeg{g.key_a, g.val_a, g.key_b, g.val_b, g.sort_tmp, g.total + 3,
                                 lsr::SortGather{g.rect, g.counts, g.rect_sorted}, (size_t)P};
            ss[k].vals_c = g.offsets;   // the device-planned passes' scratch (free until the instance scan)
            sc[k] = lsr::ScanSeg{g.counts, g.offsets, g.total, reinterpret_cast<uint32_t*>(g.scan_tmp), (size_t)P};
            if (mapped) {   // the scan writes K straight to the caller's pinned word (the preprocess
                sc[k].host_total = mapped + 2 * (v0 + k);   // zeroed a view's reserved word only on the
                host_counts[2 * (v0 + k) + 1] = 0;           // device: the host clears it here)
            }
        }
        {
            PhaseTimer t(LSR_PHASE_DEPTH_SORT, st);
            if (lsr::radix_sort_batch(ss, nv, 0, 32, st) != depth_sort_result_in_b())
                return fail(LSR_EHIP, "internal: depth sort batch or parity");
        }
        LSR_LAUNCHED("depth sort", st, s[v0]->debug);
        uint32_t wrote;
        {
            PhaseTimer t(LSR_PHASE_INSTANCE_SCAN, st);
            wrote = lsr::exclusive_scan_batch(sc, nv, st);
        }
        LSR_LAUNCHED("instance scan", st, s[v0]->debug);
        for (int k = 0; k < nv; ++k) {
            if ((wrote >> k) & 1u) continue;
            Geom g = carve_geom(geom[v0 + k], (size_t)P, nullptr);
            LSR_HIP(hipMemcpyAsync(host_counts + 2 * (v0 + k), g.total, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   st));
        }
    }
    return LSR_OK;
}
}  // namespace

int lsr_forward_preprocess_views_split_async(int32_t n_views, int32_t n_ordered, const lsr_settings* const* s,
                                             const lsr_fwd_in* in, lsr_fwd_out* const* out, void* const* geom,
                                             uint32_t* host_counts, lsr_stream_t stream) {
    int rc = check_views(n_views, s, in, geom);
    if (rc) return rc;
    if (!out || (n_ordered > 0 && !host_counts) || n_ordered < 0 || n_ordered > n_views)
        return fail(LSR_EINVAL, "0 <= n_ordered <= n_views, the outputs and host_counts are required");
    for (int v = 0; v < n_views; ++v)
        if (!out[v] || (!out[v]->radii && in->P > 0)) return fail(LSR_EINVAL, "radii output is required");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int P = in->P;
    if (P == 0) {
        for (int v = 0; v < 2 * n_ordered; ++v) host_counts[v] = 0;
        return LSR_OK;
    }
    for (int v0 = 0; v0 < n_views; v0 += lsr::LSR_MAX_VIEWS) {
        const int nv = std::min(n_views - v0, lsr::LSR_MAX_VIEWS);
        lsr::PreprocessArgs a{};
        preprocess_shared(a, s[v0], in);
        a.nv = nv;
        for (int k = 0; k < nv; ++k) {
            Geom g = carve_geom(geom[v0 + k], (size_t)P, nullptr);
            preprocess_view(a.v[k], s[v0 + k], g, out[v0 + k]->radii);
        }
        {
            PhaseTimer t(LSR_PHASE_PREPROCESS, st);
            lsr::launch_preprocess(a, st);
        }
        LSR_LAUNCHED("preprocess", st, s[v0]->debug);
    }
    return n_ordered > 0 ? depth_order_views(n_ordered, s, in, geom, host_counts, st) : LSR_OK;
}

namespace {
// preprocess of rows [row0, row1) of n_views views, one launch per 8 views; counts_tiles: each
// view's counts array gets the per-Gaussian instance counts by id (the tile-bucket binning's input)
// instead of zeros (the depth sort's last pass fills it by depth rank)
int preprocess_rows(int32_t n_views, int32_t row0, int32_t row1, int counts_tiles, const lsr_settings* const* s,
                    const lsr_fwd_in* in, lsr_fwd_out* const* out, void* const* geom, hipStream_t st) {
    int rc = check_views(n_views, s, in, geom);
    if (rc) return rc;
    if (!out || row0 < 0 || row1 < row0 || row1 > in->P || row0 % 256 != 0)
        return fail(LSR_EINVAL, "0 <= row0 <= row1 <= P with row0 a multiple of 256, and the outputs are required");
    for (int v = 0; v < n_views; ++v)
        if (!out[v] || (!out[v]->radii && in->P > 0)) return fail(LSR_EINVAL, "radii output is required");
    const int P = in->P;
    if (row1 == row0) return LSR_OK;
    for (int v0 = 0; v0 < n_views; v0 += lsr::LSR_MAX_VIEWS) {
        const int nv = std::min(n_views - v0, lsr::LSR_MAX_VIEWS);
        lsr::PreprocessArgs a{};
        preprocess_shared(a, s[v0], in);
        a.nv = nv;
        a.row0 = row0;
        a.P = row1;   // the launch's bound (every per-Gaussian array is indexed by the global row)
        a.counts_tiles = counts_tiles;
        for (int k = 0; k < nv; ++k) {
            Geom g = carve_geom(geom[v0 + k], (size_t)P, nullptr);
            preprocess_view(a.v[k], s[v0 + k], g, out[v0 + k]->radii);
        }
        {
            PhaseTimer t(LSR_PHASE_PREPROCESS, st);
            lsr::launch_preprocess(a, st);
        }
        LSR_LAUNCHED("preprocess", st, s[v0]->debug);
    }
    return LSR_OK;
}

// the tile-bucket binning's instance count: the exclusive scan of the per-Gaussian counts in id
// order (no depth sort), one launch set per 8 views; K to the page-locked host_counts as above
int instance_scan_views(int32_t n_views, const lsr_fwd_in* in, void* const* geom, uint32_t* host_counts,
                        hipStream_t st, bool debug) {
    const int P = in->P;
    uint32_t* mapped = nullptr;
    {
        void* dptr = nullptr;
        if (hipHostGetDevicePointer(&dptr, host_counts, 0) == hipSuccess && dptr) mapped = static_cast<uint32_t*>(dptr);
        else (void)hipGetLastError();
    }
    for (int v0 = 0; v0 < n_views; v0 += lsr::LSR_MAX_VIEWS) {
        const int nv = std::min(n_views - v0, lsr::LSR_MAX_VIEWS);
        lsr::ScanSeg sc[lsr::LSR_MAX_VIEWS] = {};
        for (int k = 0; k < nv; ++k) {
            Geom g = carve_geom(geom[v0 + k], (size_t)P, nullptr);
            sc[k] = lsr::ScanSeg{g.counts, g.offsets, g.total, reinterpret_cast<uint32_t*>(g.scan_tmp), (size_t)P};
            if (mapped) {
                sc[k].host_total = mapped + 2 * (v0 + k);
                host_counts[2 * (v0 + k) + 1] = 0;
            }
        }
        uint32_t wrote;
        {
            PhaseTimer t(LSR_PHASE_INSTANCE_SCAN, st);
            wrote = lsr::exclusive_scan_batch(sc, nv, st);
        }
        LSR_LAUNCHED("instance scan", st, debug);
        for (int k = 0; k < nv; ++k) {
            if ((wrote >> k) & 1u) continue;
            Geom g = carve_geom(geom[v0 + k], (size_t)P, nullptr);
            LSR_HIP(hipMemcpyAsync(host_counts + 2 * (v0 + k), g.total, 2 * sizeof(uint32_t), hipMemcpyDeviceToHost,
                                   st));
        }
    }
    return LSR_OK;
}
}  // namespace

int lsr_forward_preprocess_views_rows_async(int32_t n_views, int32_t row0, int32_t row1, const lsr_settings* const* s,
                                            const lsr_fwd_in* in, lsr_fwd_out* const* out, void* const* geom,
                                            lsr_stream_t stream) {
    return preprocess_rows(n_views, row0, row1, 0, s, in, out, geom, reinterpret_cast<hipStream_t>(stream));
}

int lsr_forward_preprocess_views_tb_async(int32_t n_views, int32_t row0, int32_t row1, const lsr_settings* const* s,
                                          const lsr_fwd_in* in, lsr_fwd_out* const* out, void* const* geom,
                                          lsr_stream_t stream) {
    return preprocess_rows(n_views, row0, row1, 1, s, in, out, geom, reinterpret_cast<hipStream_t>(stream));
}

int lsr_forward_instance_scan_views_async(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in,
                                          void* const* geom, uint32_t* host_counts, lsr_stream_t stream) {
    int rc = check_views(n_views, s, in, geom);
    if (rc) return rc;
    if (!host_counts) return fail(LSR_EINVAL, "host_counts is required");
    if (in->P == 0) {
        for (int v = 0; v < 2 * n_views; ++v) host_counts[v] = 0;
        return LSR_OK;
    }
    return instance_scan_views(n_views, in, geom, host_counts, reinterpret_cast<hipStream_t>(stream), s[0]->debug);
}

int lsr_forward_depth_order_views_async(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in,
                                        void* const* geom, uint32_t* host_counts, lsr_stream_t stream) {
    int rc = check_views(n_views, s, in, geom);
    if (rc) return rc;
    if (!host_counts) return fail(LSR_EINVAL, "host_counts is required");
    if (in->P == 0) {
        for (int v = 0; v < 2 * n_views; ++v) host_counts[v] = 0;
        return LSR_OK;
    }
    return depth_order_views(n_views, s, in, geom, host_counts, reinterpret_cast<hipStream_t>(stream));
}

int lsr_forward_preprocess_views_async(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in,
                                       lsr_fwd_out* const* out, void* const* geom, uint32_t* host_counts,
                                       lsr_stream_t stream) {
    if (!host_counts) return fail(LSR_EINVAL, "host_counts is required");
    return lsr_forward_preprocess_views_split_async(n_views, n_views, s, in, out, geom, host_counts, stream);
}

int lsr_forward_preprocess(const lsr_settings* s, const lsr_fwd_in* in, lsr_fwd_out* out, void* geom,
                           int64_t* num_rendered, lsr_stream_t stream) {
    if (!num_rendered) return fail(LSR_EINVAL, "geom workspace and num_rendered are required");
    uint32_t tot[2] = {0, 0};   // pageable: the copy completes by the synchronisation below
    int rc = lsr_forward_preprocess_async(s, in, out, geom, tot, stream);
    if (rc) return rc;
    LSR_HIP(hipStreamSynchronize(reinterpret_cast<hipStream_t>(stream)));
    *num_rendered = (int64_t)tot[0];
    return LSR_OK;
}

int lsr_forward_binning(const lsr_settings* s, const lsr_fwd_in* in, void* geom, void* binning, void* img,
                        int64_t num_rendered, lsr_stream_t stream) {
    return lsr_forward_binning_views(1, &s, in, &geom, &binning, &img, &num_rendered, stream);
}

int lsr_forward_binning_views(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in, void* const* geom,
                              void* const* binning, void* const* img, const int64_t* num_rendered,
                              lsr_stream_t stream) {
    if (n_views < 1 || !s || !geom || !binning || !img || !num_rendered)
        return fail(LSR_EINVAL, "n_views >= 1 and the per-view arrays are required");
    for (int v = 0; v < n_views; ++v) {
        int rc = check_common(s[v], in);
        if (rc) return rc;
        if (s[v]->image_width != s[0]->image_width || s[v]->image_height != s[0]->image_height)
            return fail(LSR_EINVAL, "batched views must share the image size");
        if (!geom[v] || !img[v] || (num_rendered[v] > 0 && !binning[v])) return fail(LSR_EINVAL, "workspaces are required");
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int P = in->P, W = s[0]->image_width, H = s[0]->image_height;
    const int gx = (W + LSR_TILE_X - 1) / LSR_TILE_X, gy = (H + LSR_TILE_Y - 1) / LSR_TILE_Y;
    const size_t ntiles = (size_t)gx * gy;
    const int tbits = tile_bits((int)ntiles);
    for (int v0 = 0; v0 < n_views; v0 += lsr::LSR_MAX_VIEWS) {
        const int nv = std::min(n_views - v0, lsr::LSR_MAX_VIEWS);
        lsr::EmitBatch eb{};
        eb.P = P; eb.grid_x = gx; eb.grid_y = gy; eb.W = W; eb.H = H;
        lsr::SortSeg ss[lsr::LSR_MAX_VIEWS] = {};
        int ne = 0;
        for (int k = 0; k < nv; ++k) {
            const int v = v0 + k;
            const size_t K = (size_t)num_rendered[v];
            Geom g = carve_geom(geom[v], (size_t)(P > 0 ? P : 1), nullptr);
            Img m = carve_img(img[v], W, H, nullptr);
            if (K == 0) {
                LSR_HIP(hipMemsetAsync(m.ranges, 0, sizeof(uint2) * ntiles, st));
                LSR_HIP(hipMemsetAsync(m.tile_max, 0, sizeof(uint32_t) * ntiles, st));
                continue;
            }
            Binning b = carve_binning(binning[v], K, nullptr);
            // the emission also presets the tile ranges (0xFFFFFFFF, 0) for the tile sort's last pass,
            // which makes them, and clears the per-tile replay bounds (no separate fill launches); the
            // forward compositor turns the ranges of empty tiles back into (0, 0)
            lsr::EmitView& e = eb.v[ne];
            e.order = g.val_a; e.offsets = g.offsets; e.counts = g.counts; e.rect_sorted = g.rect_sorted;
            e.xy = g.xy; e.conic_o = g.conic_o; e.keys = b.key_a; e.vals = b.val_a;
            e.clear.p[0] = reinterpret_cast<uint32_t*>(m.ranges);
            e.clear.n[0] = (uint32_t)(2 * ntiles);
            e.clear.even[0] = 0xFFFFFFFFu;
            e.clear.p[1] = m.tile_max;
            e.clear.n[1] = (uint32_t)ntiles;
            // kept: the first pass drops the instances that reach no quadrant (key 0xFFFFFFFF, about
            // 10 % of them on the headline scene), the second sorts only the listed ones
            ss[ne++] = lsr::SortSeg{b.key_a, b.val_a, b.key_b, b.val_b, b.sort_tmp, b.kept,
                                    lsr::SortGather{nullptr, nullptr, nullptr}, K, m.ranges, (uint32_t)ntiles};
        }
        if (ne == 0) continue;
        {
            PhaseTimer t(LSR_PHASE_EMIT, st);
            lsr::launch_emit_instances(eb, ne, st);
        }
        LSR_LAUNCHED("emit", st, s[0]->debug);
        {
            PhaseTimer t(LSR_PHASE_TILE_SORT, st);
            const int in_b = lsr::radix_sort_batch(ss, ne, 0, tbits, st);   // one set of launches for all views
            if (in_b < 0 || (in_b == 1) != tile_sort_in_b((int)ntiles))
                return fail(LSR_EHIP, "internal: tile sort batch or parity");
        }
        LSR_LAUNCHED("tile sort", st, s[0]->debug);
    }
    return LSR_OK;
}

int lsr_forward_binning_views_tb(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in, void* const* geom,
                                 void* const* binning, void* const* img, const int64_t* num_rendered,
                                 lsr_stream_t stream) {
    if (n_views < 1 || !s || !geom || !binning || !img || !num_rendered)
        return fail(LSR_EINVAL, "n_views >= 1 and the per-view arrays are required");
    for (int v = 0; v < n_views; ++v) {
        int rc = check_common(s[v], in);
        if (rc) return rc;
        if (s[v]->image_width != s[0]->image_width || s[v]->image_height != s[0]->image_height)
            return fail(LSR_EINVAL, "batched views must share the image size");
        if (!geom[v] || !img[v] || (num_rendered[v] > 0 && !binning[v])) return fail(LSR_EINVAL, "workspaces are required");
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int P = in->P, W = s[0]->image_width, H = s[0]->image_height;
    const int gx = (W + LSR_TILE_X - 1) / LSR_TILE_X, gy = (H + LSR_TILE_Y - 1) / LSR_TILE_Y;
    const size_t ntiles = (size_t)gx * gy;
    // the per-block tile histograms live in LDS (4 bytes a tile)
    if (ntiles > 12288)
        return fail(LSR_EINVAL, "tile-bucket binning: more than 12288 tiles (use lsr_forward_binning_views)");
    for (int v0 = 0; v0 < n_views; v0 += lsr::LSR_MAX_VIEWS) {
        const int nv = std::min(n_views - v0, lsr::LSR_MAX_VIEWS);
        lsr::TbBatch tb{};
        tb.P = P; tb.grid_x = gx; tb.grid_y = gy; tb.W = W; tb.H = H; tb.ntiles = (int)ntiles;
        int ne = 0;
        for (int k = 0; k < nv; ++k) {
            const int v = v0 + k;
            const size_t K = (size_t)num_rendered[v];
            Geom g = carve_geom(geom[v], (size_t)(P > 0 ? P : 1), nullptr);
            Img m = carve_img(img[v], W, H, nullptr);
            if (K == 0) {
                LSR_HIP(hipMemsetAsync(m.ranges, 0, sizeof(uint2) * ntiles, st));
                LSR_HIP(hipMemsetAsync(m.tile_max, 0, sizeof(uint32_t) * ntiles, st));
                continue;
            }
            BinningTb b = carve_binning_tb(binning[v], K, (size_t)P, ntiles, nullptr);
            lsr::TbView& t = tb.v[ne++];
            t.counts = g.counts; t.offsets = g.offsets; t.rect = g.rect; t.xy = g.xy; t.conic_o = g.conic_o;
            t.depth = g.key_a;
            t.table = b.table;
            t.tile_total = m.tile_order;   // backward scratch, written by the backward's tile order
            t.tile_start = m.tile_max;     // zeroed again by the bucket sort
            t.ranges = m.ranges;
            t.keys = reinterpret_cast<uint64_t*>(b.b.key_a);
            t.tmp = b.tmp;
            t.words = tile_sort_in_b((int)ntiles) ? b.b.val_b : b.b.val_a;   // where the compositors read
            t.tile_max = m.tile_max;
        }
        if (ne == 0) continue;
        {
            PhaseTimer t(LSR_PHASE_TILE_SORT, st);
            const hipError_t e = lsr::launch_tile_bucket_binning(tb, ne, st);
            if (e != hipSuccess)
                return fail(LSR_EHIP, std::string("tile-bucket binning: dynamic LDS attribute: ") + hipGetErrorString(e));
        }
        LSR_LAUNCHED("tile-bucket binning", st, s[0]->debug);
    }
    return LSR_OK;
}

int lsr_forward_composite(const lsr_settings* s, const lsr_fwd_in* in, lsr_fwd_out* out, const void* geom,
                          const void* binning, void* img, int64_t num_rendered, lsr_stream_t stream) {
    lsr_fwd_out* o[1] = {out};
    return lsr_forward_composite_views(1, &s, in, o, &geom, &binning, &img, &num_rendered, stream);
}

int lsr_forward_composite_views(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in,
                                lsr_fwd_out* const* out, const void* const* geom, const void* const* binning,
                                void* const* img, const int64_t* num_rendered, lsr_stream_t stream) {
    if (n_views < 1 || !s || !out || !geom || !binning || !img || !num_rendered)
        return fail(LSR_EINVAL, "n_views >= 1 and the per-view arrays are required");
    for (int v = 0; v < n_views; ++v) {   // every view validated before anything is launched
        int rc = check_common(s[v], in);
        if (rc) return rc;
        if (!out[v] || !out[v]->out_color || !out[v]->out_depth) return fail(LSR_EINVAL, "color and depth outputs are required");
        if (in->C > 0 && !out[v]->out_language_feature)
            return fail(LSR_EINVAL, "language feature output is required when C > 0");
        if (!geom[v] || !img[v] || (num_rendered[v] > 0 && !binning[v])) return fail(LSR_EINVAL, "workspaces are required");
        if (s[v]->image_width != s[0]->image_width || s[v]->image_height != s[0]->image_height ||
            (s[v]->include_feature != 0) != (s[0]->include_feature != 0))
            return fail(LSR_EINVAL, "batched views must share the image size and include_feature");
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int P = in->P, W = s[0]->image_width, H = s[0]->image_height, C = in->C;
    const int gx = (W + LSR_TILE_X - 1) / LSR_TILE_X, gy = (H + LSR_TILE_Y - 1) / LSR_TILE_Y;
    for (int v0 = 0; v0 < n_views; v0 += lsr::LSR_MAX_VIEWS) {
        const int nv = std::min(n_views - v0, lsr::LSR_MAX_VIEWS);
        lsr::RenderFwdArgs r[lsr::LSR_MAX_VIEWS] = {};
        for (int k = 0; k < nv; ++k) {
            const int v = v0 + k;
            const size_t K = (size_t)num_rendered[v];
            Geom g = carve_geom(const_cast<void*>(geom[v]), (size_t)(P > 0 ? P : 1), nullptr);
            Binning b = carve_binning(const_cast<void*>(binning[v]), K > 0 ? K : 1, nullptr);
            Img m = carve_img(img[v], W, H, nullptr);   // tile_max was zeroed by the binning (atomicMax: idempotent)
            lsr::RenderFwdArgs& a = r[k];
            a.W = W; a.H = H; a.grid_x = gx; a.grid_y = gy; a.C = C; a.include_feature = s[v]->include_feature;
            a.ranges = m.ranges; a.point_list = K > 0 ? (tile_sort_in_b(gx * gy) ? b.val_b : b.val_a) : nullptr;
            a.xy = g.xy; a.conic_o = g.conic_o; a.rgbd = g.rgbd;
            a.lang = in->language_feature;
            a.lang_split = in->C == 32 ? in->language_feature_split : nullptr;
            a.bg = s[v]->bg; a.final_T = m.final_T; a.n_contrib = m.n_contrib;
            a.tile_max_contrib = m.tile_max; a.tile_order = m.tile_order;
            a.out_color = out[v]->out_color; a.out_lang = out[v]->out_language_feature;
            a.out_depth = out[v]->out_depth;
            if (C > 0 && !s[v]->include_feature)
                LSR_HIP(hipMemsetAsync(out[v]->out_language_feature, 0, sizeof(float) * (size_t)C * W * H, st));
        }
        {
            PhaseTimer t(LSR_PHASE_RENDER_FWD, st);
            lsr::launch_render_fwd_views(r, nv, st);
        }
        LSR_LAUNCHED("render forward", st, s[0]->debug);
    }
    return LSR_OK;
}

int lsr_language_split(int32_t P, int32_t C, const float* language_feature, uint16_t* out, lsr_stream_t stream) {
    if (P < 0 || C != 32 || (P > 0 && (!language_feature || !out)))
        return fail(LSR_EINVAL, "lsr_language_split: P >= 0, C == 32 and both buffers are required");
    if ((size_t)P * 32 * 4 >= (size_t)1 << 32) return fail(LSR_EINVAL, "lsr_language_split: P * C * 4 must be < 2^32");
    if (P == 0) return LSR_OK;
    lsr::launch_language_split(P, language_feature, out, reinterpret_cast<hipStream_t>(stream));
    LSR_LAUNCHED("language split", reinterpret_cast<hipStream_t>(stream), false);
    return LSR_OK;
}

int lsr_forward_render(const lsr_settings* s, const lsr_fwd_in* in, lsr_fwd_out* out, void* geom, void* binning,
                       void* img, int64_t num_rendered, lsr_stream_t stream) {
    if (!out || !out->out_color || !out->out_depth) return fail(LSR_EINVAL, "color and depth outputs are required");
    int rc = lsr_forward_binning(s, in, geom, binning, img, num_rendered, stream);
    if (rc) return rc;
    return lsr_forward_composite(s, in, out, geom, binning, img, num_rendered, stream);
}

int lsr_backward(const lsr_settings* s, const lsr_fwd_in* in, const lsr_bwd_in* gin, lsr_bwd_out* gout,
                 const void* geom, const void* binning, const void* img, void* scratch, int64_t num_rendered,
                 int32_t accumulate, lsr_stream_t stream) {
    int rc = check_common(s, in);
    if (rc) return rc;
    if (!gin || !gin->dL_dout_color || !gout) return fail(LSR_EINVAL, "dL_dout_color and outputs are required");
    if (!geom || !img || !scratch || (num_rendered > 0 && !binning)) return fail(LSR_EINVAL, "workspaces are required");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int P = in->P, W = s->image_width, H = s->image_height, C = in->C;
    if (P == 0) return LSR_OK;
    const int gx = (W + LSR_TILE_X - 1) / LSR_TILE_X, gy = (H + LSR_TILE_Y - 1) / LSR_TILE_Y;
    const size_t K = (size_t)num_rendered;
    Geom g = carve_geom(const_cast<void*>(geom), (size_t)P, nullptr);
    Binning b = carve_binning(const_cast<void*>(binning), K > 0 ? K : 1, nullptr);
    Img m = carve_img(const_cast<void*>(img), W, H, nullptr);
    const int Ceff = s->include_feature ? C : 0;
    const int recq = lsr::record_floats(Ceff);
    const bool det = gin->deterministic != 0;
    Scratch sc = carve_scratch(scratch, (size_t)P, K > 0 ? K : 1, recq, det, nullptr);
    if (det && K > 0) {
        LSR_HIP(hipMemsetAsync(sc.flags, 0, K, st));
        lsr::launch_scatter_inst_off(P, g.val_a, g.offsets, g.counts, g.inst_off, st);
    }
    if (!det) LSR_HIP(hipMemsetAsync(sc.acc_small, 0, sizeof(float) * lsr::ACC_PITCH * (size_t)P, st));
    // dL/dlanguage: the atomic path adds into it, so zero it unless accumulating; with the language
    // channels off (include_feature = 0) it is exactly zero (the deterministic path writes it only
    // when they are on)
    if (!accumulate && C > 0 && gout->dL_dlanguage_feature && (!det || Ceff == 0))
        LSR_HIP(hipMemsetAsync(gout->dL_dlanguage_feature, 0, sizeof(float) * (size_t)P * C, st));
    const uint32_t* point_list = tile_sort_in_b(gx * gy) ? b.val_b : b.val_a;
    if (K > 0) {
        lsr::RenderBwdArgs r{};
        r.W = W; r.H = H; r.grid_x = gx; r.grid_y = gy; r.C = C; r.include_feature = s->include_feature;
        r.ranges = m.ranges; r.point_list = point_list; r.xy = g.xy; r.conic_o = g.conic_o; r.rgbd = g.rgbd;
        r.rect = g.rect; r.inst_off = g.inst_off;
        r.lang = in->language_feature;
    r.lang_split = in->C == 32 ? in->language_feature_split : nullptr; r.bg = s->bg; r.final_T = m.final_T; r.n_contrib = m.n_contrib;
        r.tile_max_contrib = m.tile_max; r.tile_order = m.tile_order;
        r.dL_dcolor = gin->dL_dout_color; r.dL_dlang = gin->dL_dout_language_feature; r.dL_ddepth = gin->dL_dout_depth;
        r.rec = sc.rec; r.flags = sc.flags; r.recq = recq; r.deterministic = det;
        r.acc_small = sc.acc_small; r.acc_lang = gout->dL_dlanguage_feature;
        {
            PhaseTimer t(LSR_PHASE_RENDER_BWD, st);
            lsr::launch_render_bwd(r, st);
        }
        LSR_LAUNCHED("render backward", st, s->debug);
    }
    lsr::PreprocessBwdArgs a{};
    a.P = P; a.M = in->M; a.deg = s->sh_degree;
    a.tanfovx = s->tanfovx; a.tanfovy = s->tanfovy;
    a.focal_x = (float)W / (2.0f * s->tanfovx);
    a.focal_y = (float)H / (2.0f * s->tanfovy);
    a.scale_modifier = s->scale_modifier;
    a.means3D = in->means3D; a.scales = in->scales; a.rotations = in->rotations; a.shs = in->shs;
    a.cov3D_precomp = in->cov3D_precomp; a.view = s->viewmatrix; a.proj = s->projmatrix; a.campos = s->campos;
    a.tiles = g.tiles;
    a.clamped = g.clamped;
    a.rec = sc.rec; a.flags = sc.flags; a.inst_off = g.inst_off; a.recq = recq;
    a.deterministic = det; a.acc_small = sc.acc_small;
    a.dopacity = gout->dL_dopacity;
    a.dmeans3D = gout->dL_dmeans3D; a.dmeans2D = gout->dL_dmeans2D; a.dcolors = gout->dL_dcolors;
    a.dcov3D = gout->dL_dcov3D; a.dsh = in->shs ? gout->dL_dsh : nullptr; a.dscales = gout->dL_dscales;
    a.drots = gout->dL_drotations;
    {
        PhaseTimer t(LSR_PHASE_PREPROCESS_BWD, st);
        lsr::launch_preprocess_bwd(a, accumulate != 0, st);
        if (Ceff > 0 && det)
            lsr::launch_reduce_lang(P, C, lsr::lang_pad(C), recq, sc.rec, sc.flags, g.inst_off, g.tiles,
                                    gout->dL_dlanguage_feature, accumulate != 0, st);
    }
    LSR_LAUNCHED("preprocess backward", st, s->debug);
    return LSR_OK;
}

int lsr_backward_composite(const lsr_settings* s, const lsr_fwd_in* in, const lsr_bwd_in* gin, float* dL_dlanguage,
                           void* geom, const void* binning, const void* img, int64_t num_rendered,
                           lsr_stream_t stream) {
    return lsr_backward_composite_views(1, &s, in, &gin, dL_dlanguage, &geom, &binning, &img, &num_rendered, stream);
}

int lsr_backward_composite_views(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in,
                                 const lsr_bwd_in* const* gin, float* dL_dlanguage, void* const* geom,
                                 const void* const* binning, const void* const* img, const int64_t* num_rendered,
                                 lsr_stream_t stream) {
    if (n_views < 1 || !s || !gin || !geom || !binning || !img || !num_rendered)
        return fail(LSR_EINVAL, "n_views >= 1 and the per-view arrays are required");
    for (int v = 0; v < n_views; ++v) {   // every view validated before anything is launched
        int rc = check_common(s[v], in);
        if (rc) return rc;
        if (!gin[v] || !gin[v]->dL_dout_color) return fail(LSR_EINVAL, "dL_dout_color is required");
        if (gin[v]->deterministic)
            return fail(LSR_EINVAL, "the split backward reduces with float atomics; use lsr_backward for deterministic "
                                    "gradients");
        if (!geom[v] || !img[v] || (num_rendered[v] > 0 && !binning[v])) return fail(LSR_EINVAL, "workspaces are required");
        if (s[v]->image_width != s[0]->image_width || s[v]->image_height != s[0]->image_height ||
            (s[v]->include_feature != 0) != (s[0]->include_feature != 0))
            return fail(LSR_EINVAL, "batched views must share the image size and include_feature");
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int P = in->P, C = in->C, W = s[0]->image_width, H = s[0]->image_height;
    if (P == 0) return LSR_OK;
    const int gx = (W + LSR_TILE_X - 1) / LSR_TILE_X, gy = (H + LSR_TILE_Y - 1) / LSR_TILE_Y;
    const int recq = lsr::record_floats(s[0]->include_feature ? C : 0);
    lsr::RenderBwdArgs r[lsr::LSR_MAX_VIEWS] = {};
    int nr = 0;
    auto launch = [&]() {
        if (nr == 0) return;
        {
            PhaseTimer t(LSR_PHASE_RENDER_BWD, st);
            if (C <= 32) lsr::launch_render_bwd_wave_views(r, nr, st);
            else
                for (int k = 0; k < nr; ++k) lsr::launch_render_bwd(r[k], st);   // 64 channels: per-tile kernel
        }
        nr = 0;
    };
    for (int v = 0; v < n_views; ++v) {
        const size_t K = (size_t)num_rendered[v];
        if (K == 0) continue;   // nothing listed: no compositor work
        Geom g = carve_geom(geom[v], (size_t)P, nullptr);   // g.acc: rows of listed Gaussians zeroed by the preprocess
        Binning b = carve_binning(const_cast<void*>(binning[v]), K, nullptr);
        Img m = carve_img(const_cast<void*>(img[v]), W, H, nullptr);
        lsr::RenderBwdArgs& a = r[nr++];
        a.W = W; a.H = H; a.grid_x = gx; a.grid_y = gy; a.C = C; a.include_feature = s[v]->include_feature;
        a.ranges = m.ranges; a.point_list = tile_sort_in_b(gx * gy) ? b.val_b : b.val_a;
        a.xy = g.xy; a.conic_o = g.conic_o; a.rgbd = g.rgbd;
        a.rect = g.rect; a.inst_off = g.inst_off;
        a.lang = in->language_feature;
        a.lang_split = in->C == 32 ? in->language_feature_split : nullptr;
        a.bg = s[v]->bg; a.final_T = m.final_T; a.n_contrib = m.n_contrib;
        a.tile_max_contrib = m.tile_max; a.tile_order = m.tile_order;
        a.dL_dcolor = gin[v]->dL_dout_color; a.dL_dlang = gin[v]->dL_dout_language_feature;
        a.dL_ddepth = gin[v]->dL_dout_depth;
        a.recq = recq; a.deterministic = 0;
        a.acc_small = reinterpret_cast<float*>(g.acc); a.acc_lang = dL_dlanguage;
        if (nr == lsr::LSR_MAX_VIEWS) launch();
    }
    launch();
    LSR_LAUNCHED("render backward", st, s[0]->debug);
    return LSR_OK;
}

int lsr_backward_preprocess_views(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in,
                                  lsr_bwd_out* gout, const void* const* geom, int32_t accumulate,
                                  lsr_stream_t stream) {
    if (!in) return fail(LSR_EINVAL, "null argument");
    return lsr_backward_preprocess_views_rows(n_views, s, in, gout, geom, accumulate, 0, in->P, stream);
}

int lsr_backward_preprocess_views_rows(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in,
                                       lsr_bwd_out* gout, const void* const* geom, int32_t accumulate,
                                       int32_t row_begin, int32_t row_count, lsr_stream_t stream) {
    if (n_views < 1) return fail(LSR_EINVAL, "n_views must be >= 1");
    if (!s || !in || !gout || !geom) return fail(LSR_EINVAL, "null argument");
    for (int v = 0; v < n_views; ++v) {
        int rc = check_common(s[v], in);
        if (rc) return rc;
        if (!geom[v]) return fail(LSR_EINVAL, "the geom workspace is required for every view");
        if (s[v]->scale_modifier != s[0]->scale_modifier) return fail(LSR_EINVAL, "all views must share scale_modifier");
    }
    if (row_begin < 0 || row_count < 0 || (int64_t)row_begin + row_count > in->P)
        return fail(LSR_EINVAL, "rows [row_begin, row_begin + row_count) must lie inside [0, P)");
    if (row_begin % 256 != 0) return fail(LSR_EINVAL, "row_begin must be a multiple of 256");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int P = in->P, n = row_count;
    const size_t r0 = (size_t)row_begin;
    if (n == 0) return LSR_OK;
    const int M = in->M;
    // one launch per LSR_MAX_VIEWS views: Gaussian rows read and gradient rows written once; a row
    // range is the same kernel over pointers advanced to row_begin (gout already addresses it)
    for (int v0 = 0; v0 < n_views; v0 += lsr::LSR_MAX_VIEWS) {
        const int nv = std::min(lsr::LSR_MAX_VIEWS, n_views - v0);
        lsr::PreprocessBwdViewsArgs a{};
        a.P = n; a.M = M; a.nv = nv; a.scale_modifier = s[0]->scale_modifier;
        a.means3D = in->means3D + 3 * r0;
        a.scales = in->scales ? in->scales + 3 * r0 : nullptr;
        a.rotations = in->rotations ? in->rotations + 4 * r0 : nullptr;
        a.shs = in->shs ? in->shs + (size_t)M * 3 * r0 : nullptr;
        a.cov3D_precomp = in->cov3D_precomp ? in->cov3D_precomp + 6 * r0 : nullptr;
        for (int j = 0; j < nv; ++j) {
            const int v = v0 + j;
            const lsr_settings* sv = s[v];
            Geom g = carve_geom(const_cast<void*>(geom[v]), (size_t)P, nullptr);
            lsr::ViewCam& c = a.cam[j];
            c.view = sv->viewmatrix; c.proj = sv->projmatrix; c.campos = sv->campos;
            c.tanfovx = sv->tanfovx; c.tanfovy = sv->tanfovy;
            c.focal_x = (float)sv->image_width / (2.0f * sv->tanfovx);
            c.focal_y = (float)sv->image_height / (2.0f * sv->tanfovy);
            c.deg = sv->sh_degree;
            c.tiles = g.tiles + r0; c.clamped = g.clamped + r0;
            c.acc_small = reinterpret_cast<const float*>(g.acc) + lsr::ACC_PITCH * r0;
        }
        a.dopacity = gout->dL_dopacity;
        a.dmeans3D = gout->dL_dmeans3D; a.dmeans2D = gout->dL_dmeans2D; a.dcolors = gout->dL_dcolors;
        a.dcov3D = gout->dL_dcov3D; a.dsh = in->shs ? gout->dL_dsh : nullptr; a.dscales = gout->dL_dscales;
        a.drots = gout->dL_drotations;
        {
            PhaseTimer t(LSR_PHASE_PREPROCESS_BWD_VIEWS, st);
            lsr::launch_preprocess_bwd_views(a, accumulate != 0 || v0 > 0, st);
        }
        LSR_LAUNCHED("preprocess backward (views)", st, s[0]->debug);
    }
    return LSR_OK;
}

int lsr_backward_views(int32_t n_views, const lsr_settings* const* s, const lsr_fwd_in* in,
                       const lsr_bwd_in* const* gin, lsr_bwd_out* gout, void* const* geom,
                       const void* const* binning, const void* const* img, const int64_t* num_rendered,
                       int32_t accumulate, lsr_stream_t stream) {
    if (n_views < 1) return fail(LSR_EINVAL, "n_views must be >= 1");
    if (!s || !in || !gin || !gout || !geom || !binning || !img || !num_rendered)
        return fail(LSR_EINVAL, "null argument");
    for (int v = 0; v < n_views; ++v) {   // validate every view before anything is launched
        int rc = check_common(s[v], in);
        if (rc) return rc;
        if (!gin[v] || !gin[v]->dL_dout_color) return fail(LSR_EINVAL, "dL_dout_color is required for every view");
        if (gin[v]->deterministic)
            return fail(LSR_EINVAL, "lsr_backward_views reduces with float atomics; use lsr_backward per view for "
                                    "deterministic gradients");
        if (s[v]->scale_modifier != s[0]->scale_modifier) return fail(LSR_EINVAL, "all views must share scale_modifier");
    }
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    const int P = in->P, C = in->C;
    if (P == 0) return LSR_OK;
    if (!accumulate && C > 0 && gout->dL_dlanguage_feature)
        LSR_HIP(hipMemsetAsync(gout->dL_dlanguage_feature, 0, sizeof(float) * (size_t)P * C, st));
    int rc = lsr_backward_composite_views(n_views, s, in, gin, gout->dL_dlanguage_feature, geom, binning, img,
                                          num_rendered, stream);
    if (rc) return rc;
    return lsr_backward_preprocess_views(n_views, s, in, gout, const_cast<const void* const*>(geom), accumulate,
                                         stream);
}

int lsr_radii_max(int32_t P, int32_t n_views, const int32_t* const* radii, int32_t* out, int32_t accumulate,
                  lsr_stream_t stream) {
    if (P < 0 || n_views < 0 || (P > 0 && n_views > 0 && (!radii || !out))) return fail(LSR_EINVAL, "bad lsr_radii_max arguments");
    for (int v = 0; v < n_views; ++v)
        if (P > 0 && (!radii[v] || (reinterpret_cast<uintptr_t>(radii[v]) & 15)))
            return fail(LSR_EINVAL, "lsr_radii_max: every radii array must be a 16-byte aligned device pointer");
    if (P > 0 && (reinterpret_cast<uintptr_t>(out) & 15)) return fail(LSR_EINVAL, "lsr_radii_max: out must be 16-byte aligned");
    if (P == 0 || n_views == 0) return LSR_OK;
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    lsr::launch_radii_max(P, n_views, reinterpret_cast<const int* const*>(radii), out, accumulate != 0, st);
    LSR_LAUNCHED("radii max", st, false);
    return LSR_OK;
}

int lsr_mark_visible(int32_t P, const float* means3D, const float* viewmatrix, const float* projmatrix,
                     uint8_t* present, lsr_stream_t stream) {
    (void)projmatrix;
    if (P < 0 || (P > 0 && (!means3D || !viewmatrix || !present))) return fail(LSR_EINVAL, "bad mark_visible arguments");
    hipStream_t st = reinterpret_cast<hipStream_t>(stream);
    lsr::launch_mark_visible(P, means3D, viewmatrix, present, st);
    LSR_LAUNCHED("mark_visible", st, false);
    return LSR_OK;
}

int lsr_profile_phases(uint32_t mask) {
    std::lock_guard<std::mutex> l(g_prof.mu);
    g_prof.mask = mask;
    return LSR_OK;
}

int lsr_profile_enable(int32_t on) {
    std::lock_guard<std::mutex> l(g_prof.mu);
    for (auto& r : g_prof.pending) {
        (void)hipEventSynchronize(r.b);
        g_prof.pool.push_back(r.a);
        g_prof.pool.push_back(r.b);
    }
    g_prof.pending.clear();
    for (int i = 0; i < LSR_NUM_PHASES; ++i) { g_prof.ms[i] = 0.0; g_prof.n[i] = 0; }
    g_prof.on = on != 0;
    return LSR_OK;
}

int lsr_profile_read(double* ms_total, int64_t* launches, int32_t n) {
    std::lock_guard<std::mutex> l(g_prof.mu);
    for (auto& r : g_prof.pending) {
        if (hipEventSynchronize(r.b) != hipSuccess) return fail(LSR_EHIP, "profile: event synchronize failed");
        float ms = 0.0f;
        if (hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            g_prof.ms[r.phase] += ms;
            g_prof.n[r.phase] += 1;
        }
        g_prof.pool.push_back(r.a);
        g_prof.pool.push_back(r.b);
    }
    g_prof.pending.clear();
    for (int i = 0; i < n && i < LSR_NUM_PHASES; ++i) {
        if (ms_total) ms_total[i] = g_prof.ms[i];
        if (launches) launches[i] = g_prof.n[i];
    }
    return LSR_NUM_PHASES;
}

}  // extern "C"

namespace lsr {
// shared with the other C-ABI translation units (deform_api.hip)
int fail(int code, const std::string& msg) { return ::fail(code, msg); }
}  // namespace lsr
