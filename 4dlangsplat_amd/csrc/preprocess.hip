// preprocess.hip -- per-Gaussian projection (forward) and the matching backward.
//
// Forward restates the upstream preprocessCUDA (call site gaussian_renderer/__init__.py:219-228;
// constants in SURVEY.md 8a row a8): near cull z <= 0.2, EWA covariance with the 1.3 tan-fov clamp
// and +0.3 low-pass, conic, 3-sigma radius, tile count, SH degree <= 3 colour.  One lane per
// Gaussian; outputs are written as packed SoA records the compositor gathers in 8/16-byte pieces:
//   xy      float2  pixel-space mean
//   conic_o float4  (conic a, b, c, opacity)
//   rgbd    float4  (r, g, b, view-space depth)
//   key     u32     depth bits of visible Gaussians, 0xFFFFFFFF for culled ones (sort key)
// Backward (rows a12 of SURVEY.md 8a) is fused with the per-Gaussian reduction of the
// compositor's screen-space gradients: one lane per Gaussian walks conic -> cov2D -> cov3D ->
// (scale, rotation), the projection Jacobian for means2D, the depth row, and the SH chain.
#include "lsr_common.h"
#include "lsr_internal.h"

namespace lsr {

struct m3 { float m[3][3]; };  // glm layout: m[column][row]

__device__ __forceinline__ m3 mul(const m3& a, const m3& b) {
    m3 o;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r)
            o.m[c][r] = a.m[0][r] * b.m[c][0] + a.m[1][r] * b.m[c][1] + a.m[2][r] * b.m[c][2];
    return o;
}
__device__ __forceinline__ m3 tr(const m3& a) {
    m3 o;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) o.m[c][r] = a.m[r][c];
    return o;
}
__device__ __forceinline__ m3 quat_R(float4 q) {
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    m3 R;
    R.m[0][0] = 1.0f - 2.0f * (y * y + z * z); R.m[0][1] = 2.0f * (x * y - r * z); R.m[0][2] = 2.0f * (x * z + r * y);
    R.m[1][0] = 2.0f * (x * y + r * z); R.m[1][1] = 1.0f - 2.0f * (x * x + z * z); R.m[1][2] = 2.0f * (y * z - r * x);
    R.m[2][0] = 2.0f * (x * z - r * y); R.m[2][1] = 2.0f * (y * z + r * x); R.m[2][2] = 1.0f - 2.0f * (x * x + y * y);
    return R;
}
__device__ __forceinline__ m3 zero3() {
    m3 o;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int r = 0; r < 3; ++r) o.m[c][r] = 0.0f;
    return o;
}

__device__ __forceinline__ void cov3d(float3 s, float mod, float4 q, float* cov) {
    m3 S = zero3();
    S.m[0][0] = mod * s.x; S.m[1][1] = mod * s.y; S.m[2][2] = mod * s.z;
    const m3 Rm = quat_R(q);
    const m3 M = mul(S, Rm);
    const m3 Sig = mul(tr(M), M);
    cov[0] = Sig.m[0][0]; cov[1] = Sig.m[0][1]; cov[2] = Sig.m[0][2];
    cov[3] = Sig.m[1][1]; cov[4] = Sig.m[1][2]; cov[5] = Sig.m[2][2];
}

__device__ __forceinline__ m3 view_W(const float* __restrict__ v) {
    m3 W;
    W.m[0][0] = v[0]; W.m[0][1] = v[4]; W.m[0][2] = v[8];
    W.m[1][0] = v[1]; W.m[1][1] = v[5]; W.m[1][2] = v[9];
    W.m[2][0] = v[2]; W.m[2][1] = v[6]; W.m[2][2] = v[10];
    return W;
}
__device__ __forceinline__ m3 sym3(const float* c) {
    m3 V;
    V.m[0][0] = c[0]; V.m[0][1] = c[1]; V.m[0][2] = c[2];
    V.m[1][0] = c[1]; V.m[1][1] = c[3]; V.m[1][2] = c[4];
    V.m[2][0] = c[2]; V.m[2][1] = c[4]; V.m[2][2] = c[5];
    return V;
}

__constant__ float SH_C0 = 0.28209479177387814f;
__constant__ float SH_C1 = 0.4886025119029199f;
__constant__ float SH_C2[5] = {1.0925484305920792f, -1.0925484305920792f, 0.31539156525252005f,
                               -1.0925484305920792f, 0.5462742152960396f};
__constant__ float SH_C3[7] = {-0.5900435899266435f, 2.890611442640554f, -0.4570457994644658f,
                               0.3731763325901154f, -0.4570457994644658f, 1.445305721320277f,
                               -0.5900435899266435f};

// ---------------------------------------------------------------------------------------------
// Copy the [rows x M3] SH block of this workgroup into LDS rows of pitch M3 + 1 with coalesced
// loads (the per-Gaussian 48-float rows are otherwise read 64 rows at a time per instruction).
template <int M3>
__device__ __forceinline__ void stage_rows(float* __restrict__ lds, const float* __restrict__ src, int rows) {
    if constexpr (M3 > 0) {
        constexpr int SP = M3 + 1;
        const int n = rows * M3;
        for (int e = threadIdx.x; e < n; e += blockDim.x) {
            const int r = e / M3, c = e - r * M3;
            lds[r * SP + c] = src[e];
        }
    }
}

// A Gaussian's view-independent inputs.  One view: read where the projection first needs them
// (culled Gaussians skip the scale / rotation / SH reads).  Several views: read once, cov3D built
// once, kept in registers for every view.
template <int MS>
struct GaussIn {
    float3 p;
    float op;
    float c3[6];
    float sh[MS > 0 ? 3 * MS : 1];
};
__device__ __forceinline__ float3 load_mean(const PreprocessArgs& a, int i) {
    return make_float3(a.means3D[3 * i], a.means3D[3 * i + 1], a.means3D[3 * i + 2]);
}
__device__ __forceinline__ void load_cov3d(const PreprocessArgs& a, int i, float (&c3)[6]) {
    if (a.cov3D_precomp) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3[k] = a.cov3D_precomp[6 * (size_t)i + k];
    } else {
        const float3 s = make_float3(a.scales[3 * i], a.scales[3 * i + 1], a.scales[3 * i + 2]);
        const float4 q = reinterpret_cast<const float4*>(a.rotations)[i];
        cov3d(s, a.scale_modifier, q, c3);
    }
}
// the SH row in registers, every load in flight at once (float4 when 16-byte aligned)
template <int MS, int N>
__device__ __forceinline__ void load_sh(const PreprocessArgs& a, int i, float (&shr)[N]) {
    constexpr int M3 = MS * 3;
    const float* src = a.shs + (size_t)i * M3;
    if (M3 % 4 == 0 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
#pragma unroll
        for (int q = 0; q < M3 / 4; ++q) {
            const float4 t = reinterpret_cast<const float4*>(src)[q];
            shr[4 * q] = t.x; shr[4 * q + 1] = t.y; shr[4 * q + 2] = t.z; shr[4 * q + 3] = t.w;
        }
    } else {
#pragma unroll
        for (int q = 0; q < M3; ++q) shr[q] = src[q];
    }
}
template <int MS>
__device__ __forceinline__ void load_gauss(const PreprocessArgs& a, int i, GaussIn<MS>& g) {
    g.p = load_mean(a, i);
    g.op = a.opacities[i];
    load_cov3d(a, i, g.c3);
    if constexpr (MS > 0) {
        if (a.shs && !a.colors_precomp) load_sh<MS>(a, i, g.sh);
    }
}

template <int MS, bool PRE>  // MS: SH coefficients per Gaussian (0 = any M, read from global); PRE: g holds the inputs
__device__ __forceinline__ bool preprocess_one(const PreprocessArgs& a, const PreprocessView& v, const GaussIn<MS>& g,
                                               int i) {   // true: rectangle
    v.radii[i] = 0;
    v.radius[i] = 0;
    v.tiles[i] = 0;
    v.rect[i] = make_uint2(0u, 0u);
    v.clamped[i] = 0;
    if (v.order) v.order[i] = (uint32_t)i;
    if (v.rank_counts) v.rank_counts[i] = 0u;
    if (v.key) v.key[i] = 0xFFFFFFFFu;
    const float3 p = PRE ? g.p : load_mean(a, i);
    const float4 ph = xform4x4(v.proj, p);
    const float3 pv = xform4x3(v.view, p);
    if (pv.z <= 0.2f) return false;
    const float pw = 1.0f / (ph.w + 0.0000001f);
    const float3 pp = make_float3(ph.x * pw, ph.y * pw, ph.z * pw);

    float c3[6];
    if constexpr (PRE) {
#pragma unroll
        for (int k = 0; k < 6; ++k) c3[k] = g.c3[k];
    } else {
        load_cov3d(a, i, c3);
    }
    // EWA projection (computeCov2D)
    float3 t = pv;
    const float limx = 1.3f * v.tanfovx, limy = 1.3f * v.tanfovy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    m3 J = zero3();
    J.m[0][0] = v.focal_x / t.z; J.m[0][2] = -(v.focal_x * t.x) / (t.z * t.z);
    J.m[1][1] = v.focal_y / t.z; J.m[1][2] = -(v.focal_y * t.y) / (t.z * t.z);
    const m3 T = mul(view_W(v.view), J);
    const m3 V = sym3(c3);
    const m3 A = mul(tr(T), tr(V));
    const m3 cv = mul(A, T);
    const float ca = cv.m[0][0] + 0.3f, cb = cv.m[0][1], cc = cv.m[1][1] + 0.3f;
    const float det = ca * cc - cb * cb;
    if (det == 0.0f) return false;
    const float det_inv = 1.0f / det;
    const float4 conic = make_float4(cc * det_inv, -cb * det_inv, ca * det_inv, PRE ? g.op : a.opacities[i]);
    const float mid = 0.5f * (ca + cc);
    const float l1 = mid + sqrtf(fmaxf(0.1f, mid * mid - det));
    const float l2 = mid - sqrtf(fmaxf(0.1f, mid * mid - det));
    const int radius = (int)ceilf(3.0f * sqrtf(fmaxf(l1, l2)));
    const float2 pix = make_float2(ndc2pix(pp.x, a.W), ndc2pix(pp.y, a.H));
    int2 rmin, rmax;
    tile_rect(pix, radius, a.grid_x, a.grid_y, rmin, rmax);
    if ((rmax.y - rmin.y) * (rmax.x - rmin.x) == 0) return false;   // upstream: culled (radius 0)
    // Binning rectangle: upstream's 3-sigma square intersected with the bounding box of the ellipse
    // where a pixel can pass the compositors' exact alpha prefilter (power >= skip_power(o), i.e.
    // q(d) <= -2 skip_power(o)).  Every dropped (Gaussian, tile) would be skipped at every pixel of
    // the tile, so the rendered result is unchanged; radii (user-visible) stay upstream's.  The
    // margin covers the float evaluation of q at the pixels (terms bounded inside the square).
    const float thr = skip_power(conic.w);
    int ntiles = 0;
    int2 cmin = make_int2(0, 0), cmax = make_int2(0, 0);
    if (thr <= 0.0f) {
        const float rr = (float)radius + 16.0f;
        const float mt = (fabsf(conic.x) + fabsf(conic.z) + 2.0f * fabsf(conic.y)) * rr * rr;
        const float qm = -2.0f * thr + 1e-6f * mt + 1e-4f;
        const float hx = sqrtf(qm * ca) + 0.01f, hy = sqrtf(qm * cc) + 0.01f;
        cmin.x = max(rmin.x, (int)floorf((pix.x - hx) / (float)LSR_TILE_X));
        cmin.y = max(rmin.y, (int)floorf((pix.y - hy) / (float)LSR_TILE_Y));
        cmax.x = min(rmax.x, (int)floorf((pix.x + hx) / (float)LSR_TILE_X) + 1);
        cmax.y = min(rmax.y, (int)floorf((pix.y + hy) / (float)LSR_TILE_Y) + 1);
        if (cmax.x > cmin.x && cmax.y > cmin.y) ntiles = (cmax.x - cmin.x) * (cmax.y - cmin.y);
        else cmin = cmax = make_int2(0, 0);
    }

    float rgb[3];
    if (a.colors_precomp) {
        rgb[0] = a.colors_precomp[3 * i]; rgb[1] = a.colors_precomp[3 * i + 1]; rgb[2] = a.colors_precomp[3 * i + 2];
    } else {
        float3 dir = make_float3(p.x - v.campos[0], p.y - v.campos[1], p.z - v.campos[2]);
        const float len = sqrtf(dir.x * dir.x + dir.y * dir.y + dir.z * dir.z);
        dir.x = dir.x / len; dir.y = dir.y / len; dir.z = dir.z / len;
        float shr[48];   // static indices reach coefficient 15; only the first M3 are loaded (deg validated)
        if constexpr (MS > 0) {
            if constexpr (PRE) {
#pragma unroll
                for (int q = 0; q < 3 * MS; ++q) shr[q] = g.sh[q];
            } else {
                load_sh<MS>(a, i, shr);
            }
        }
        const float* sh = MS > 0 ? shr : a.shs + (size_t)i * a.M * 3;
        uint8_t cl = 0;
        const int deg = a.deg;
#pragma unroll
        for (int ch = 0; ch < 3; ++ch) {
#define SHc(k) sh[(k) * 3 + ch]
            float res = SH_C0 * SHc(0);
            if (deg > 0) {
                const float x = dir.x, y = dir.y, z = dir.z;
                res = res - SH_C1 * y * SHc(1) + SH_C1 * z * SHc(2) - SH_C1 * x * SHc(3);
                if (deg > 1) {
                    const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                    res = res + SH_C2[0] * xy * SHc(4) + SH_C2[1] * yz * SHc(5) +
                          SH_C2[2] * (2.0f * zz - xx - yy) * SHc(6) + SH_C2[3] * xz * SHc(7) +
                          SH_C2[4] * (xx - yy) * SHc(8);
                    if (deg > 2) {
                        res = res + SH_C3[0] * y * (3.0f * xx - yy) * SHc(9) + SH_C3[1] * xy * z * SHc(10) +
                              SH_C3[2] * y * (4.0f * zz - xx - yy) * SHc(11) +
                              SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy) * SHc(12) +
                              SH_C3[4] * x * (4.0f * zz - xx - yy) * SHc(13) + SH_C3[5] * z * (xx - yy) * SHc(14) +
                              SH_C3[6] * x * (xx - 3.0f * yy) * SHc(15);
                    }
                }
            }
#undef SHc
            res = res + 0.5f;
            cl |= (res < 0.0f ? 1 : 0) << ch;
            rgb[ch] = res < 0.0f ? 0.0f : res;
        }
        v.clamped[i] = cl;
    }
    v.radii[i] = radius;
    v.radius[i] = radius;
    uint32_t qmap = 0;   // quadrant map of a rectangle of <= 2 x 2 tiles (the binning's emit_quad_mask)
    if (ntiles > 0 && cmax.x - cmin.x <= 2 && cmax.y - cmin.y <= 2) {
        // emit_quad_mask per tile, with each 8-row band's extent computed once for the tile row
        // (bit 8 (ty - y0) + 4 band + 2 (tx - x0) + column; the same arithmetic and bits)
        const EmitSplat es = emit_splat(pix, conic);
        const float ex = emit_margin(es);
        for (int ty = cmin.y; ty < cmax.y; ++ty)
#pragma unroll
            for (int band = 0; band < 2; ++band) {
                bool ok;
                float xmin, xmax;
                emit_band(es, ty * LSR_TILE_Y + 8 * band, a.H, ex, ok, xmin, xmax);
                for (int tx = cmin.x; tx < cmax.x; ++tx)
#pragma unroll
                    for (int col = 0; col < 2; ++col)
                        qmap |= emit_col_hit(es, ok, xmin, xmax, tx * LSR_TILE_X + 8 * col, a.W)
                                    ? 1u << (8 * (ty - cmin.y) + 4 * band + 2 * (tx - cmin.x) + col) : 0u;
            }
    }
    const uint2 rc = rect_pack((uint32_t)cmin.x, (uint32_t)cmin.y, (uint32_t)cmax.x, (uint32_t)cmax.y, qmap);
    v.rect[i] = rc;
    // instances it will emit: a small rectangle's tiles with a reachable quadrant (none: the
    // Gaussian blends no pixel and is not listed -- its gradient is exactly zero)
    v.tiles[i] = rect_count(rc);
    if (v.rank_counts && a.counts_tiles) v.rank_counts[i] = rect_count(rc);
    if (v.key) v.key[i] = __float_as_uint(pv.z);
    v.xy[i] = pix;
    v.conic_o[i] = conic;
    v.rgbd[i] = make_float4(rgb[0], rgb[1], rgb[2], pv.z);
    return ntiles > 0;
}

// Only rectangles receive backward atomics (a superset of the listed): zero their accumulator
// rows, the wave's 64 rows written as whole float4 runs (coalesced; a row per lane would write 64
// strided partial lines per store).  Every lane of the wave calls this.
__device__ __forceinline__ void zero_acc_rows(float4* acc, bool rect, int i) {
    if (!acc) return;
    const uint64_t m = __ballot(rect);
    if (m == 0) return;
    const int ln = threadIdx.x & 63;
    float4* w = acc + (size_t)(i - ln) * (ACC_PITCH / 4);
#pragma unroll
    for (int q = 0; q < ACC_PITCH / 4; ++q) {
        const int e = q * 64 + ln;
        if ((m >> (e / (ACC_PITCH / 4))) & 1) w[e] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    }
}

template <int MS, bool MULTI>
__global__ void __launch_bounds__(256) k_preprocess(PreprocessArgs a) {
    const int i = a.row0 + blockIdx.x * blockDim.x + threadIdx.x;
    GaussIn<MS> g;
    if constexpr (!MULTI) {
        clear_words(a.v[0].clear);
        const bool rect = i < a.P && preprocess_one<MS, false>(a, a.v[0], g, i);
        zero_acc_rows(a.v[0].acc, rect, i);
    } else {
        const bool ok = i < a.P;
        if (ok) load_gauss<MS>(a, i, g);
        for (int k = 0; k < a.nv; ++k) {   // uniform: the view's fields are scalar loads
            const PreprocessView& v = a.v[k];
            clear_words(v.clear);
            const bool rect = ok && preprocess_one<MS, true>(a, v, g, i);
            zero_acc_rows(v.acc, rect, i);
        }
    }
}

void launch_preprocess(const PreprocessArgs& a, hipStream_t st) {
    if (a.P <= a.row0 || a.nv <= 0) return;
    const dim3 grid((a.P - a.row0 + 255) / 256), block(256);
#define LSR_PP(MS)                                                                   \
    do {                                                                             \
        if (a.nv > 1) hipLaunchKernelGGL((k_preprocess<MS, true>), grid, block, 0, st, a);  \
        else hipLaunchKernelGGL((k_preprocess<MS, false>), grid, block, 0, st, a);          \
    } while (0)
    switch ((a.shs && !a.colors_precomp) ? a.M : 0) {
        case 1: LSR_PP(1); break;
        case 4: LSR_PP(4); break;
        case 9: LSR_PP(9); break;
        case 16: LSR_PP(16); break;
        default: LSR_PP(0); break;
    }
#undef LSR_PP
}

// ---------------------------------------------------------------------------------------------
// mark_visible
__global__ void k_mark_visible(int P, const float* __restrict__ means3D, const float* __restrict__ view,
                               uint8_t* __restrict__ present) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= P) return;
    const float3 p = make_float3(means3D[3 * i], means3D[3 * i + 1], means3D[3 * i + 2]);
    present[i] = xform4x3(view, p).z > 0.2f;
}
// out[i] = max(out[i] (accumulate) or 0, radii_0[i], ..., radii_{n-1}[i]): the radii MAX over a
// step's views (train.py:270) in one pass, int4 vectors (P % 4 == 0 rows; the tail scalar)
struct RadiiMaxArgs { const int* r[LSR_MAX_VIEWS]; };
__global__ void __launch_bounds__(256) k_radii_max(int P, int n, RadiiMaxArgs ra, int* __restrict__ out, int accumulate) {
    const int i4 = blockIdx.x * 256 + threadIdx.x, i = 4 * i4;
    if (i >= P) return;
    if (i + 4 <= P) {
        int4 m = accumulate ? reinterpret_cast<const int4*>(out)[i4] : make_int4(0, 0, 0, 0);
        for (int v = 0; v < n; ++v) {
            const int4 x = reinterpret_cast<const int4*>(ra.r[v])[i4];
            m = make_int4(max(m.x, x.x), max(m.y, x.y), max(m.z, x.z), max(m.w, x.w));
        }
        reinterpret_cast<int4*>(out)[i4] = m;
    } else {
        for (int k = i; k < P; ++k) {
            int m = accumulate ? out[k] : 0;
            for (int v = 0; v < n; ++v) m = max(m, ra.r[v][k]);
            out[k] = m;
        }
    }
}
void launch_radii_max(int P, int n, const int* const* radii, int* out, bool accumulate, hipStream_t st) {
    for (int v0 = 0; v0 < n; v0 += LSR_MAX_VIEWS) {
        RadiiMaxArgs ra{};
        const int nv = n - v0 < LSR_MAX_VIEWS ? n - v0 : LSR_MAX_VIEWS;
        for (int k = 0; k < nv; ++k) ra.r[k] = radii[v0 + k];
        hipLaunchKernelGGL(k_radii_max, dim3((unsigned)((P + 1023) / 1024)), dim3(256), 0, st, P, nv, ra, out,
                           (accumulate || v0 > 0) ? 1 : 0);
    }
}

void launch_mark_visible(int P, const float* means3D, const float* view, uint8_t* present, hipStream_t st) {
    if (P == 0) return;
    hipLaunchKernelGGL(k_mark_visible, dim3((P + 255) / 256), dim3(256), 0, st, P, means3D, view, present);
}

// ---------------------------------------------------------------------------------------------
// Backward.  g_* are the per-Gaussian screen-space gradients summed by the compositor backward.
__device__ void cov2d_bwd(float3 mean, const float* c3, float fx, float fy, float tanfovx, float tanfovy,
                          const float* __restrict__ view, float3 dconic, float3& dmean, float* dcov) {
#pragma clang fp contract(fast)   // gradients only (no decisions): fma contraction allowed
    // Upstream's chain (T = W J, cov2D = T^T V T, then dT -> dJ -> dt) restated on the two nonzero
    // columns u0, u1 of T (J's third column is zero): W(r, c) = view[4r + c].  Reciprocals are the
    // hardware rcp (gradients only); the clamp decisions use the same exact quotients as the forward.
    float3 t = xform4x3(view, mean);
    const float limx = 1.3f * tanfovx, limy = 1.3f * tanfovy;
    const float txtz = t.x / t.z, tytz = t.y / t.z;
    t.x = fminf(limx, fmaxf(-limx, txtz)) * t.z;
    t.y = fminf(limy, fmaxf(-limy, tytz)) * t.z;
    const float x_grad_mul = (txtz < -limx || txtz > limx) ? 0.0f : 1.0f;
    const float y_grad_mul = (tytz < -limy || tytz > limy) ? 0.0f : 1.0f;
    const float tz = __builtin_amdgcn_rcpf(t.z), tz2 = tz * tz, tz3 = tz2 * tz;
    const float J00 = fx * tz, J11 = fy * tz, J02 = -(fx * t.x) * tz2, J12 = -(fy * t.y) * tz2;
    float u0[3], u1[3], Vu0[3], Vu1[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        u0[r] = view[4 * r] * J00 + view[4 * r + 2] * J02;
        u1[r] = view[4 * r + 1] * J11 + view[4 * r + 2] * J12;
    }
    const float V[3][3] = {{c3[0], c3[1], c3[2]}, {c3[1], c3[3], c3[4]}, {c3[2], c3[4], c3[5]}};
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        Vu0[r] = V[r][0] * u0[0] + V[r][1] * u0[1] + V[r][2] * u0[2];
        Vu1[r] = V[r][0] * u1[0] + V[r][1] * u1[1] + V[r][2] * u1[2];
    }
    const float a = u0[0] * Vu0[0] + u0[1] * Vu0[1] + u0[2] * Vu0[2] + 0.3f;
    const float b = u0[0] * Vu1[0] + u0[1] * Vu1[1] + u0[2] * Vu1[2];
    const float c = u1[0] * Vu1[0] + u1[1] * Vu1[1] + u1[2] * Vu1[2] + 0.3f;
    const float denom = a * c - b * b;
    float dL_da = 0.0f, dL_db = 0.0f, dL_dc = 0.0f;
    const float denom2inv = __builtin_amdgcn_rcpf((denom * denom) + 0.0000001f);
    if (denom2inv != 0.0f) {
        dL_da = denom2inv * (-c * c * dconic.x + 2.0f * b * c * dconic.y + (denom - a * c) * dconic.z);
        dL_dc = denom2inv * (-a * a * dconic.z + 2.0f * a * b * dconic.y + (denom - a * c) * dconic.x);
        dL_db = denom2inv * 2.0f * (b * c * dconic.x - (denom + 2.0f * b * b) * dconic.y + a * b * dconic.z);
    }
    dcov[0] = u0[0] * u0[0] * dL_da + u0[0] * u1[0] * dL_db + u1[0] * u1[0] * dL_dc;
    dcov[3] = u0[1] * u0[1] * dL_da + u0[1] * u1[1] * dL_db + u1[1] * u1[1] * dL_dc;
    dcov[5] = u0[2] * u0[2] * dL_da + u0[2] * u1[2] * dL_db + u1[2] * u1[2] * dL_dc;
    dcov[1] = 2.0f * u0[0] * u0[1] * dL_da + (u0[0] * u1[1] + u0[1] * u1[0]) * dL_db + 2.0f * u1[0] * u1[1] * dL_dc;
    dcov[2] = 2.0f * u0[0] * u0[2] * dL_da + (u0[0] * u1[2] + u0[2] * u1[0]) * dL_db + 2.0f * u1[0] * u1[2] * dL_dc;
    dcov[4] = 2.0f * u0[2] * u0[1] * dL_da + (u0[1] * u1[2] + u0[2] * u1[1]) * dL_db + 2.0f * u1[1] * u1[2] * dL_dc;
    // dT rows (upstream dL_dT00..dL_dT12) from the same V u products
    float dT0[3], dT1[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        dT0[k] = 2.0f * Vu0[k] * dL_da + Vu1[k] * dL_db;
        dT1[k] = 2.0f * Vu1[k] * dL_dc + Vu0[k] * dL_db;
    }
    const float dJ00 = view[0] * dT0[0] + view[4] * dT0[1] + view[8] * dT0[2];
    const float dJ02 = view[2] * dT0[0] + view[6] * dT0[1] + view[10] * dT0[2];
    const float dJ11 = view[1] * dT1[0] + view[5] * dT1[1] + view[9] * dT1[2];
    const float dJ12 = view[2] * dT1[0] + view[6] * dT1[1] + view[10] * dT1[2];
    const float dtx = x_grad_mul * -fx * tz2 * dJ02;
    const float dty = y_grad_mul * -fy * tz2 * dJ12;
    const float dtz = -fx * tz2 * dJ00 - fy * tz2 * dJ11 + (2.0f * fx * t.x) * tz3 * dJ02 + (2.0f * fy * t.y) * tz3 * dJ12;
    dmean.x = view[0] * dtx + view[1] * dty + view[2] * dtz;
    dmean.y = view[4] * dtx + view[5] * dty + view[6] * dtz;
    dmean.z = view[8] * dtx + view[9] * dty + view[10] * dtz;
}

__device__ void cov3d_bwd(float3 sc, float mod, float4 q, const float* dcov, float3& dscale, float4& drot) {
#pragma clang fp contract(fast)   // gradients only (no decisions): fma contraction allowed
    const float r = q.x, x = q.y, y = q.z, z = q.w;
    const m3 Rm = quat_R(q);
    const float s[3] = {mod * sc.x, mod * sc.y, mod * sc.z};
    m3 S = zero3();
    S.m[0][0] = s[0]; S.m[1][1] = s[1]; S.m[2][2] = s[2];
    const m3 M = mul(S, Rm);
    m3 dS;
    dS.m[0][0] = dcov[0]; dS.m[0][1] = 0.5f * dcov[1]; dS.m[0][2] = 0.5f * dcov[2];
    dS.m[1][0] = 0.5f * dcov[1]; dS.m[1][1] = dcov[3]; dS.m[1][2] = 0.5f * dcov[4];
    dS.m[2][0] = 0.5f * dcov[2]; dS.m[2][1] = 0.5f * dcov[4]; dS.m[2][2] = dcov[5];
    m3 M2;
#pragma unroll
    for (int c = 0; c < 3; ++c)
#pragma unroll
        for (int k = 0; k < 3; ++k) M2.m[c][k] = 2.0f * M.m[c][k];
    const m3 dM = mul(M2, dS);
    const m3 Rt = tr(Rm);
    m3 d = tr(dM);
    float ds[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) ds[k] = (Rt.m[k][0] * d.m[k][0] + Rt.m[k][1] * d.m[k][1] + Rt.m[k][2] * d.m[k][2]) * mod;
    dscale = make_float3(ds[0], ds[1], ds[2]);
#pragma unroll
    for (int k = 0; k < 3; ++k) { d.m[0][k] *= s[0]; d.m[1][k] *= s[1]; d.m[2][k] *= s[2]; }
    drot.x = 2.0f * z * (d.m[0][1] - d.m[1][0]) + 2.0f * y * (d.m[2][0] - d.m[0][2]) + 2.0f * x * (d.m[1][2] - d.m[2][1]);
    drot.y = 2.0f * y * (d.m[1][0] + d.m[0][1]) + 2.0f * z * (d.m[2][0] + d.m[0][2]) + 2.0f * r * (d.m[1][2] - d.m[2][1]) -
             4.0f * x * (d.m[2][2] + d.m[1][1]);
    drot.z = 2.0f * x * (d.m[1][0] + d.m[0][1]) + 2.0f * r * (d.m[2][0] - d.m[0][2]) + 2.0f * z * (d.m[1][2] + d.m[2][1]) -
             4.0f * y * (d.m[2][2] + d.m[0][0]);
    drot.w = 2.0f * r * (d.m[0][1] - d.m[1][0]) + 2.0f * x * (d.m[2][0] + d.m[0][2]) + 2.0f * y * (d.m[1][2] + d.m[2][1]) -
             4.0f * z * (d.m[1][1] + d.m[0][0]);
}

// SH backward (upstream computeColorFromSH backward): dL/dsh[k][ch] = b[k] * dR[ch] with b[k] the
// direction-only basis factors, computed once for the three colour channels.
__device__ __forceinline__ void sh_bwd_basis(int deg, float x, float y, float z, float (&b)[16]) {
#pragma clang fp contract(fast)   // gradients only
#pragma unroll
    for (int k = 0; k < 16; ++k) b[k] = 0.0f;
    b[0] = SH_C0;
    if (deg > 0) {
        b[1] = -SH_C1 * y; b[2] = SH_C1 * z; b[3] = -SH_C1 * x;
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            b[4] = SH_C2[0] * xy; b[5] = SH_C2[1] * yz; b[6] = SH_C2[2] * (2.0f * zz - xx - yy); b[7] = SH_C2[3] * xz;
            b[8] = SH_C2[4] * (xx - yy);
            if (deg > 2) {
                b[9] = SH_C3[0] * y * (3.0f * xx - yy);
                b[10] = SH_C3[1] * xy * z;
                b[11] = SH_C3[2] * y * (4.0f * zz - xx - yy);
                b[12] = SH_C3[3] * z * (2.0f * zz - 3.0f * xx - 3.0f * yy);
                b[13] = SH_C3[4] * x * (4.0f * zz - xx - yy);
                b[14] = SH_C3[5] * z * (xx - yy);
                b[15] = SH_C3[6] * x * (xx - 3.0f * yy);
            }
        }
    }
}

// Sum over the colour channels of dR[ch] * d colour_ch / d direction (the dL/dx, dL/dy, dL/dz that
// upstream forms from its per-channel dRGBdx, dRGBdy, dRGBdz), contracted per coefficient first:
// s_k = sum_ch SH[k][ch] dR[ch], then one pass of the basis derivatives over s_k.
__device__ __forceinline__ void sh_bwd_dirsum(const float* __restrict__ sh, int deg, float x, float y, float z,
                                              const float (&dR)[3], float& dLdx, float& dLdy, float& dLdz) {
#pragma clang fp contract(fast)   // gradients only
#define SK(k) (sh[(k) * 3] * dR[0] + sh[(k) * 3 + 1] * dR[1] + sh[(k) * 3 + 2] * dR[2])
    dLdx = 0.0f; dLdy = 0.0f; dLdz = 0.0f;
    if (deg > 0) {
        dLdx = -SH_C1 * SK(3); dLdy = -SH_C1 * SK(1); dLdz = SH_C1 * SK(2);
        if (deg > 1) {
            const float xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
            const float s4 = SK(4), s5 = SK(5), s6 = SK(6), s7 = SK(7), s8 = SK(8);
            dLdx += SH_C2[0] * y * s4 + SH_C2[2] * 2.0f * -x * s6 + SH_C2[3] * z * s7 + SH_C2[4] * 2.0f * x * s8;
            dLdy += SH_C2[0] * x * s4 + SH_C2[1] * z * s5 + SH_C2[2] * 2.0f * -y * s6 + SH_C2[4] * 2.0f * -y * s8;
            dLdz += SH_C2[1] * y * s5 + SH_C2[2] * 2.0f * 2.0f * z * s6 + SH_C2[3] * x * s7;
            if (deg > 2) {
                const float s9 = SK(9), s10 = SK(10), s11 = SK(11), s12 = SK(12), s13 = SK(13), s14 = SK(14), s15 = SK(15);
                dLdx += SH_C3[0] * s9 * 3.0f * 2.0f * xy + SH_C3[1] * s10 * yz + SH_C3[2] * s11 * -2.0f * xy +
                        SH_C3[3] * s12 * -3.0f * 2.0f * xz + SH_C3[4] * s13 * (-3.0f * xx + 4.0f * zz - yy) +
                        SH_C3[5] * s14 * 2.0f * xz + SH_C3[6] * s15 * 3.0f * (xx - yy);
                dLdy += SH_C3[0] * s9 * 3.0f * (xx - yy) + SH_C3[1] * s10 * xz +
                        SH_C3[2] * s11 * (-3.0f * yy + 4.0f * zz - xx) + SH_C3[3] * s12 * -3.0f * 2.0f * yz +
                        SH_C3[4] * s13 * -2.0f * xy + SH_C3[5] * s14 * -2.0f * yz + SH_C3[6] * s15 * -3.0f * 2.0f * xy;
                dLdz += SH_C3[1] * s10 * xy + SH_C3[2] * s11 * 4.0f * 2.0f * yz +
                        SH_C3[3] * s12 * 3.0f * (2.0f * zz - xx - yy) + SH_C3[4] * s13 * 4.0f * 2.0f * xz +
                        SH_C3[5] * s14 * (xx - yy);
            }
        }
    }
#undef SK
}

template <bool ACC>
__device__ __forceinline__ void put(float* p, float v) {
    if (ACC) *p += v; else *p = v;
}

// Rows of culled Gaussians (no tiles) are neither read nor, when accumulating, written: their
// gradient is exactly zero.  float4 loads (a row is 3*MS floats, 16-B aligned for MS = 16).
template <int M3>
__device__ __forceinline__ void stage_visible_rows(float* __restrict__ lds, const float* __restrict__ src, int rows,
                                                   const uint8_t* __restrict__ s_vis) {
    if constexpr (M3 > 0) {
        constexpr int SP = M3 + 1;
        if constexpr (M3 % 4 == 0) {
            constexpr int R4 = M3 / 4;
            const float4* s4 = reinterpret_cast<const float4*>(src);
            if (rows == 256 && (reinterpret_cast<uintptr_t>(src) & 15) == 0) {
                // full block: every load in flight at once (compile-time trip count)
                float4 v[R4];
#pragma unroll
                for (int j = 0; j < R4; ++j) {
                    const int e = threadIdx.x + 256 * j;
                    v[j] = s_vis[e / R4] ? s4[e] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                }
#pragma unroll
                for (int j = 0; j < R4; ++j) {
                    const int e = threadIdx.x + 256 * j, r = e / R4, c = 4 * (e - r * R4);
                    float* d = lds + r * SP + c;
                    d[0] = v[j].x; d[1] = v[j].y; d[2] = v[j].z; d[3] = v[j].w;
                }
                return;
            }
        }
        for (int e = threadIdx.x; e < rows * M3; e += blockDim.x) {
            const int r = e / M3, c = e - r * M3;
            if (s_vis[r]) lds[r * SP + c] = src[e];
        }
    }
}

// Coalesced write-out (or accumulation) of a block's staged SH gradient rows; culled rows are
// skipped when accumulating (their gradient is zero).
template <bool ACC, int M3>
__device__ __forceinline__ void write_rows(float* __restrict__ dst, const float* __restrict__ lds, int rows,
                                           const uint8_t* __restrict__ s_vis) {
    if constexpr (M3 > 0) {
        constexpr int SP = M3 + 1;
        if constexpr (M3 % 4 == 0) {
            constexpr int R4 = M3 / 4;
            float4* d4 = reinterpret_cast<float4*>(dst);
            if (rows == 256 && (reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
                float4 cur[R4];
                bool ok[R4];
#pragma unroll
                for (int j = 0; j < R4; ++j) {
                    const int e = threadIdx.x + 256 * j;
                    ok[j] = !ACC || s_vis[e / R4];
                    cur[j] = (ACC && ok[j]) ? d4[e] : make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                }
#pragma unroll
                for (int j = 0; j < R4; ++j) {
                    const int e = threadIdx.x + 256 * j, r = e / R4, c = 4 * (e - r * R4);
                    if (!ok[j]) continue;
                    const float* l = lds + r * SP + c;
                    d4[e] = make_float4(cur[j].x + l[0], cur[j].y + l[1], cur[j].z + l[2], cur[j].w + l[3]);
                }
                return;
            }
        }
        for (int e = threadIdx.x; e < rows * M3; e += blockDim.x) {
            const int r = e / M3, c = e - r * M3;
            if (!ACC || s_vis[r]) put<ACC>(dst + e, lds[r * SP + c]);
        }
    }
}

template <bool ACC, int MS>
__global__ void __launch_bounds__(256) k_preprocess_bwd(PreprocessBwdArgs a) {
#pragma clang fp contract(fast)   // backward: gradients only, fma contraction allowed
    constexpr int M3 = MS * 3, SP = M3 + 1;
    __shared__ float s_sh[MS > 0 ? 256 * SP : 1];
    __shared__ uint8_t s_vis[256];
    const int g0 = blockIdx.x * blockDim.x;
    const int rows = min(256, a.P - g0);
    const int i = g0 + threadIdx.x;
    const uint32_t ntile = i < a.P ? a.tiles[i] : 0u;
    const bool vis = ntile > 0;
    const bool stage = MS > 0 && a.shs != nullptr;
    if (stage) {
        s_vis[threadIdx.x] = vis ? 1 : 0;
        __syncthreads();
        stage_visible_rows<M3>(s_sh, a.shs + (size_t)g0 * M3, rows, s_vis);
        __syncthreads();
    }
    if (i < a.P && (vis || !ACC)) {
        // sum the compositor's per-(Gaussian, tile) records: contiguous per Gaussian
        float rs[12];
#pragma unroll
        for (int k = 0; k < 12; ++k) rs[k] = 0.0f;
        if (vis && !a.deterministic) {
            const float4* r4 = reinterpret_cast<const float4*>(a.acc_small + (size_t)i * ACC_PITCH);
#pragma unroll
            for (int k4 = 0; k4 < 3; ++k4) {
                const float4 v = r4[k4];
                rs[4 * k4] = v.x; rs[4 * k4 + 1] = v.y; rs[4 * k4 + 2] = v.z; rs[4 * k4 + 3] = v.w;
            }
        } else if (vis) {
            const uint32_t e0 = a.inst_off[i];
            for (uint32_t e = e0; e < e0 + ntile; ++e) {
                if (!a.flags[e]) continue;
                const float4* r4 = reinterpret_cast<const float4*>(a.rec + (size_t)e * a.recq);
#pragma unroll
                for (int k4 = 0; k4 < 3; ++k4) {
                    const float4 v = r4[k4];
                    rs[4 * k4] += v.x; rs[4 * k4 + 1] += v.y; rs[4 * k4 + 2] += v.z; rs[4 * k4 + 3] += v.w;
                }
            }
        }
        // record layout: rgb 0-2, depth 3, mean2D 4-5 (NDC), conic 6-8 (upstream x, y, w), opacity 9
        const float3 gcol = make_float3(rs[0], rs[1], rs[2]);
        const float gx = rs[4], gy = rs[5];
        if (a.dmeans2D) { put<ACC>(a.dmeans2D + 3 * (size_t)i, gx); put<ACC>(a.dmeans2D + 3 * (size_t)i + 1, gy); put<ACC>(a.dmeans2D + 3 * (size_t)i + 2, 0.0f); }
        if (a.dcolors) { put<ACC>(a.dcolors + 3 * (size_t)i, gcol.x); put<ACC>(a.dcolors + 3 * (size_t)i + 1, gcol.y); put<ACC>(a.dcolors + 3 * (size_t)i + 2, gcol.z); }
        if (a.dopacity) put<ACC>(a.dopacity + i, rs[9]);

        float3 dm = make_float3(0.0f, 0.0f, 0.0f);
        float dcov[6] = {0, 0, 0, 0, 0, 0};
        float3 dscale = make_float3(0.0f, 0.0f, 0.0f);
        float4 drot = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const int M = a.M;
        float* srow = stage ? s_sh + threadIdx.x * SP : nullptr;
        if (vis) {
            const float3 p = make_float3(a.means3D[3 * i], a.means3D[3 * i + 1], a.means3D[3 * i + 2]);
            float c3[6];
            float3 sc = make_float3(0.0f, 0.0f, 0.0f);
            float4 q = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (a.cov3D_precomp) {
#pragma unroll
                for (int k = 0; k < 6; ++k) c3[k] = a.cov3D_precomp[6 * (size_t)i + k];
            } else {
                sc = make_float3(a.scales[3 * i], a.scales[3 * i + 1], a.scales[3 * i + 2]);
                q = reinterpret_cast<const float4*>(a.rotations)[i];
                cov3d(sc, a.scale_modifier, q, c3);
            }
            cov2d_bwd(p, c3, a.focal_x, a.focal_y, a.tanfovx, a.tanfovy, a.view, make_float3(rs[6], rs[7], rs[8]), dm, dcov);
            // projection of the mean
            const float* pm = a.proj;
            const float4 mh = xform4x4(pm, p);
            const float mw = __builtin_amdgcn_rcpf(mh.w + 0.0000001f);
            const float mul1 = mh.x * mw * mw;
            const float mul2 = mh.y * mw * mw;
            dm.x += (pm[0] * mw - pm[3] * mul1) * gx + (pm[1] * mw - pm[3] * mul2) * gy;
            dm.y += (pm[4] * mw - pm[7] * mul1) * gx + (pm[5] * mw - pm[7] * mul2) * gy;
            dm.z += (pm[8] * mw - pm[11] * mul1) * gx + (pm[9] * mw - pm[11] * mul2) * gy;
            // depth row
            const float gd = rs[3];
            dm.x += a.view[2] * gd;
            dm.y += a.view[6] * gd;
            dm.z += a.view[10] * gd;
            // SH
            if (a.shs) {
                const float3 dir_orig = make_float3(p.x - a.campos[0], p.y - a.campos[1], p.z - a.campos[2]);
                const float sum2 = dir_orig.x * dir_orig.x + dir_orig.y * dir_orig.y + dir_orig.z * dir_orig.z;
                const float il = __builtin_amdgcn_rsqf(sum2);   // gradients only: hardware rsq
                const float x = dir_orig.x * il, y = dir_orig.y * il, z = dir_orig.z * il;
                const uint8_t cl = a.clamped[i];
                const float dR[3] = {(cl & 1) ? 0.0f : gcol.x, (cl & 2) ? 0.0f : gcol.y, (cl & 4) ? 0.0f : gcol.z};
                const float* sh = stage ? srow : a.shs + (size_t)i * M * 3;
                float* dsh = stage ? srow : (a.dsh ? a.dsh + (size_t)i * M * 3 : nullptr);
                const int deg = a.deg;
                float dLdx, dLdy, dLdz;
                sh_bwd_dirsum(sh, deg, x, y, z, dR, dLdx, dLdy, dLdz);
                // every coefficient has been read: overwrite the staged row with the gradient
                float bs[16];
                sh_bwd_basis(deg, x, y, z, bs);
#pragma unroll
                for (int ch = 0; ch < 3; ++ch) {
                    if (stage) {
#pragma unroll
                        for (int k = 0; k < MS; ++k) dsh[k * 3 + ch] = k < 16 ? bs[k] * dR[ch] : 0.0f;
                    } else if (dsh) {
                        for (int k = 0; k < M; ++k) put<ACC>(dsh + k * 3 + ch, k < 16 ? bs[k] * dR[ch] : 0.0f);
                    }
                }
                const float3 v = dir_orig;
                const float invsum32 = il * il * il;
                dm.x += ((sum2 - v.x * v.x) * dLdx - v.y * v.x * dLdy - v.z * v.x * dLdz) * invsum32;
                dm.y += (-v.x * v.y * dLdx + (sum2 - v.y * v.y) * dLdy - v.z * v.y * dLdz) * invsum32;
                dm.z += (-v.x * v.z * dLdx - v.y * v.z * dLdy + (sum2 - v.z * v.z) * dLdz) * invsum32;
            }
            if (!a.cov3D_precomp) cov3d_bwd(sc, a.scale_modifier, q, dcov, dscale, drot);
        } else if (stage) {
#pragma unroll
            for (int k = 0; k < M3; ++k) srow[k] = 0.0f;
        } else if (a.dsh && !ACC) {
            float* dsh = a.dsh + (size_t)i * M * 3;
            for (int k = 0; k < 3 * M; ++k) dsh[k] = 0.0f;
        }
        if (a.dmeans3D) { put<ACC>(a.dmeans3D + 3 * (size_t)i, dm.x); put<ACC>(a.dmeans3D + 3 * (size_t)i + 1, dm.y); put<ACC>(a.dmeans3D + 3 * (size_t)i + 2, dm.z); }
        if (a.dcov3D) {
#pragma unroll
            for (int k = 0; k < 6; ++k) put<ACC>(a.dcov3D + 6 * (size_t)i + k, dcov[k]);
        }
        if (a.dscales) { put<ACC>(a.dscales + 3 * (size_t)i, dscale.x); put<ACC>(a.dscales + 3 * (size_t)i + 1, dscale.y); put<ACC>(a.dscales + 3 * (size_t)i + 2, dscale.z); }
        if (a.drots) {
            put<ACC>(a.drots + 4 * (size_t)i, drot.x); put<ACC>(a.drots + 4 * (size_t)i + 1, drot.y);
            put<ACC>(a.drots + 4 * (size_t)i + 2, drot.z); put<ACC>(a.drots + 4 * (size_t)i + 3, drot.w);
        }
    }
    if (stage && a.dsh) {   // coalesced write-out of the block's SH gradient rows
        __syncthreads();
        write_rows<ACC, M3>(a.dsh + (size_t)g0 * M3, s_sh, rows, s_vis);
    }
}

// Several views at once (lsr_backward_views): the same per-view chain as k_preprocess_bwd, summed
// over the views in which the Gaussian has tiles.  The view-independent work is done once: the
// Gaussian's rows are read once, cov3D is built once, and the scale / rotation backward runs once
// on the summed dL/dcov3D (it is linear in it); the gradient rows are written once.
template <bool ACC, int MS>
__global__ void __launch_bounds__(256) k_preprocess_bwd_views(PreprocessBwdViewsArgs a) {
#pragma clang fp contract(fast)   // backward: gradients only, fma contraction allowed
    constexpr int M3 = MS * 3, SP = M3 + 1;
    __shared__ float s_sh[MS > 0 ? 256 * SP : 1];
    __shared__ uint8_t s_vis[256];
    const int g0 = blockIdx.x * blockDim.x;
    const int rows = min(256, a.P - g0);
    const int i = g0 + threadIdx.x;
    uint32_t vmask = 0;
#pragma unroll
    for (int v = 0; v < LSR_MAX_VIEWS; ++v)
        if (v < a.nv && i < a.P && a.cam[v].tiles[i] > 0) vmask |= 1u << v;
    const bool vis = vmask != 0;
    const bool stage = MS > 0 && a.shs != nullptr;
    if (stage) {
        s_vis[threadIdx.x] = vis ? 1 : 0;
        __syncthreads();
        stage_visible_rows<M3>(s_sh, a.shs + (size_t)g0 * M3, rows, s_vis);
        __syncthreads();
    }
    if (i < a.P && (vis || !ACC)) {
        float gcol[3] = {0.0f, 0.0f, 0.0f}, g2d[2] = {0.0f, 0.0f}, gop = 0.0f;
        float3 dm = make_float3(0.0f, 0.0f, 0.0f);
        float dcov[6] = {0, 0, 0, 0, 0, 0};
        float dsh[48];
#pragma unroll
        for (int k = 0; k < 48; ++k) dsh[k] = 0.0f;
        float3 dscale = make_float3(0.0f, 0.0f, 0.0f);
        float4 drot = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        const int M = a.M;
        float* srow = stage ? s_sh + threadIdx.x * SP : nullptr;
        if (vis) {
            const float3 p = make_float3(a.means3D[3 * i], a.means3D[3 * i + 1], a.means3D[3 * i + 2]);
            float c3[6];
            float3 sc = make_float3(0.0f, 0.0f, 0.0f);
            float4 q = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
            if (a.cov3D_precomp) {
#pragma unroll
                for (int k = 0; k < 6; ++k) c3[k] = a.cov3D_precomp[6 * (size_t)i + k];
            } else {
                sc = make_float3(a.scales[3 * i], a.scales[3 * i + 1], a.scales[3 * i + 2]);
                q = reinterpret_cast<const float4*>(a.rotations)[i];
                cov3d(sc, a.scale_modifier, q, c3);
            }
            const float* sh = stage ? srow : (a.shs ? a.shs + (size_t)i * M * 3 : nullptr);
#pragma unroll
            for (int v = 0; v < LSR_MAX_VIEWS; ++v) {
                if (!((vmask >> v) & 1u)) continue;
                const ViewCam& cm = a.cam[v];
                float rs[12];
                const float4* r4 = reinterpret_cast<const float4*>(cm.acc_small + (size_t)i * ACC_PITCH);
#pragma unroll
                for (int k4 = 0; k4 < 3; ++k4) {
                    const float4 t = r4[k4];
                    rs[4 * k4] = t.x; rs[4 * k4 + 1] = t.y; rs[4 * k4 + 2] = t.z; rs[4 * k4 + 3] = t.w;
                }
                gcol[0] += rs[0]; gcol[1] += rs[1]; gcol[2] += rs[2];
                const float gx = rs[4], gy = rs[5];
                g2d[0] += gx; g2d[1] += gy;
                gop += rs[9];
                float3 dmv;
                float dcv[6];
                cov2d_bwd(p, c3, cm.focal_x, cm.focal_y, cm.tanfovx, cm.tanfovy, cm.view, make_float3(rs[6], rs[7], rs[8]),
                          dmv, dcv);
#pragma unroll
                for (int k = 0; k < 6; ++k) dcov[k] += dcv[k];
                const float* pm = cm.proj;
                const float4 mh = xform4x4(pm, p);
                const float mw = __builtin_amdgcn_rcpf(mh.w + 0.0000001f);
                const float mul1 = mh.x * mw * mw;
                const float mul2 = mh.y * mw * mw;
                dmv.x += (pm[0] * mw - pm[3] * mul1) * gx + (pm[1] * mw - pm[3] * mul2) * gy;
                dmv.y += (pm[4] * mw - pm[7] * mul1) * gx + (pm[5] * mw - pm[7] * mul2) * gy;
                dmv.z += (pm[8] * mw - pm[11] * mul1) * gx + (pm[9] * mw - pm[11] * mul2) * gy;
                const float gd = rs[3];
                dmv.x += cm.view[2] * gd;
                dmv.y += cm.view[6] * gd;
                dmv.z += cm.view[10] * gd;
                if (sh) {
                    const float3 dir_orig = make_float3(p.x - cm.campos[0], p.y - cm.campos[1], p.z - cm.campos[2]);
                    const float sum2 = dir_orig.x * dir_orig.x + dir_orig.y * dir_orig.y + dir_orig.z * dir_orig.z;
                    const float il = __builtin_amdgcn_rsqf(sum2);   // gradients only: hardware rsq
                    const float x = dir_orig.x * il, y = dir_orig.y * il, z = dir_orig.z * il;
                    const uint8_t cl = cm.clamped[i];
                    const float dR[3] = {(cl & 1) ? 0.0f : rs[0], (cl & 2) ? 0.0f : rs[1], (cl & 4) ? 0.0f : rs[2]};
                    float bs[16];
                    sh_bwd_basis(cm.deg, x, y, z, bs);   // once for the three channels
#pragma unroll
                    for (int ch = 0; ch < 3; ++ch)
#pragma unroll
                        for (int k = 0; k < 16; ++k) dsh[k * 3 + ch] += bs[k] * dR[ch];
                    float dLdx, dLdy, dLdz;
                    sh_bwd_dirsum(sh, cm.deg, x, y, z, dR, dLdx, dLdy, dLdz);
                    const float3 w = dir_orig;
                    const float invsum32 = il * il * il;
                    dmv.x += ((sum2 - w.x * w.x) * dLdx - w.y * w.x * dLdy - w.z * w.x * dLdz) * invsum32;
                    dmv.y += (-w.x * w.y * dLdx + (sum2 - w.y * w.y) * dLdy - w.z * w.y * dLdz) * invsum32;
                    dmv.z += (-w.x * w.z * dLdx - w.y * w.z * dLdy + (sum2 - w.z * w.z) * dLdz) * invsum32;
                }
                dm.x += dmv.x; dm.y += dmv.y; dm.z += dmv.z;
            }
            if (!a.cov3D_precomp) cov3d_bwd(sc, a.scale_modifier, q, dcov, dscale, drot);
        }
        if (a.dmeans2D) { put<ACC>(a.dmeans2D + 3 * (size_t)i, g2d[0]); put<ACC>(a.dmeans2D + 3 * (size_t)i + 1, g2d[1]); put<ACC>(a.dmeans2D + 3 * (size_t)i + 2, 0.0f); }
        if (a.dcolors) { put<ACC>(a.dcolors + 3 * (size_t)i, gcol[0]); put<ACC>(a.dcolors + 3 * (size_t)i + 1, gcol[1]); put<ACC>(a.dcolors + 3 * (size_t)i + 2, gcol[2]); }
        if (a.dopacity) put<ACC>(a.dopacity + i, gop);
        if (a.dmeans3D) { put<ACC>(a.dmeans3D + 3 * (size_t)i, dm.x); put<ACC>(a.dmeans3D + 3 * (size_t)i + 1, dm.y); put<ACC>(a.dmeans3D + 3 * (size_t)i + 2, dm.z); }
        if (a.dcov3D) {
#pragma unroll
            for (int k = 0; k < 6; ++k) put<ACC>(a.dcov3D + 6 * (size_t)i + k, dcov[k]);
        }
        if (a.dscales) { put<ACC>(a.dscales + 3 * (size_t)i, dscale.x); put<ACC>(a.dscales + 3 * (size_t)i + 1, dscale.y); put<ACC>(a.dscales + 3 * (size_t)i + 2, dscale.z); }
        if (a.drots) {
            put<ACC>(a.drots + 4 * (size_t)i, drot.x); put<ACC>(a.drots + 4 * (size_t)i + 1, drot.y);
            put<ACC>(a.drots + 4 * (size_t)i + 2, drot.z); put<ACC>(a.drots + 4 * (size_t)i + 3, drot.w);
        }
        if (stage) {
#pragma unroll
            for (int k = 0; k < M3; ++k) srow[k] = k < 48 ? dsh[k] : 0.0f;
        } else if (a.dsh && a.shs) {
            float* d = a.dsh + (size_t)i * M * 3;
#pragma unroll
            for (int k = 0; k < 48; ++k)
                if (k < 3 * M) put<ACC>(d + k, dsh[k]);
            for (int k = 48; k < 3 * M; ++k) put<ACC>(d + k, 0.0f);
        }
    }
    if (stage && a.dsh) {
        __syncthreads();
        write_rows<ACC, M3>(a.dsh + (size_t)g0 * M3, s_sh, rows, s_vis);
    }
}

void launch_preprocess_bwd_views(const PreprocessBwdViewsArgs& a, bool accumulate, hipStream_t st) {
    if (a.P == 0 || a.nv == 0) return;
    const dim3 grid((a.P + 255) / 256), block(256);
#define LSR_GOV(ACC, MS) hipLaunchKernelGGL((k_preprocess_bwd_views<ACC, MS>), grid, block, 0, st, a)
    const int m = a.shs ? a.M : 0;
    if (accumulate) {
        switch (m) { case 1: LSR_GOV(true, 1); break; case 4: LSR_GOV(true, 4); break; case 9: LSR_GOV(true, 9); break;
                     case 16: LSR_GOV(true, 16); break; default: LSR_GOV(true, 0); break; }
    } else {
        switch (m) { case 1: LSR_GOV(false, 1); break; case 4: LSR_GOV(false, 4); break; case 9: LSR_GOV(false, 9); break;
                     case 16: LSR_GOV(false, 16); break; default: LSR_GOV(false, 0); break; }
    }
#undef LSR_GOV
}

template <bool ACC>
static void go_pbwd(const PreprocessBwdArgs& a, hipStream_t st) {
    const dim3 grid((a.P + 255) / 256), block(256);
    switch (a.shs ? a.M : 0) {
        case 1: hipLaunchKernelGGL((k_preprocess_bwd<ACC, 1>), grid, block, 0, st, a); break;
        case 4: hipLaunchKernelGGL((k_preprocess_bwd<ACC, 4>), grid, block, 0, st, a); break;
        case 9: hipLaunchKernelGGL((k_preprocess_bwd<ACC, 9>), grid, block, 0, st, a); break;
        case 16: hipLaunchKernelGGL((k_preprocess_bwd<ACC, 16>), grid, block, 0, st, a); break;
        default: hipLaunchKernelGGL((k_preprocess_bwd<ACC, 0>), grid, block, 0, st, a); break;
    }
}

void launch_preprocess_bwd(const PreprocessBwdArgs& a, bool accumulate, hipStream_t st) {
    if (a.P == 0) return;
    if (accumulate) go_pbwd<true>(a, st);
    else go_pbwd<false>(a, st);
}

// Language-feature gradient: sum of the records' C channels of each Gaussian.  A Gaussian's
// records are contiguous; CPAD/4 lanes per Gaussian read them as float4 (coalesced rows).
template <bool ACC, int CPAD>
__global__ void __launch_bounds__(256) k_reduce_lang(int P, int C, int recq, const float* __restrict__ rec,
                                                     const uint8_t* __restrict__ flags, const uint32_t* __restrict__ inst_off,
                                                     const uint32_t* __restrict__ tiles, float* __restrict__ dlang) {
    constexpr int LPG = CPAD / 4, GPB = 256 / LPG;
    const int g = blockIdx.x * GPB + threadIdx.x / LPG;
    const int c4 = threadIdx.x % LPG;
    if (g >= P) return;
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    const uint32_t n = tiles[g];
    if (n > 0) {
        const uint32_t e0 = inst_off[g];
        for (uint32_t e = e0; e < e0 + n; ++e) {
            if (!flags[e]) continue;
            const float4 v = reinterpret_cast<const float4*>(rec + (size_t)e * recq + 12)[c4];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
    }
    float* d = dlang + (size_t)g * C;
    const float vals[4] = {acc.x, acc.y, acc.z, acc.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int c = 4 * c4 + j;
        if (c < C) put<ACC>(d + c, vals[j]);
    }
}

void launch_reduce_lang(int P, int C, int cpad, int recq, const float* rec, const uint8_t* flags,
                        const uint32_t* inst_off, const uint32_t* tiles, float* dlang, bool accumulate, hipStream_t st) {
    if (P == 0 || C == 0 || !dlang) return;
#define LSR_GO(CP)                                                                                        \
    {                                                                                                     \
        constexpr int GPB = 256 / ((CP) / 4);                                                            \
        const dim3 grid((P + GPB - 1) / GPB);                                                             \
        if (accumulate) hipLaunchKernelGGL((k_reduce_lang<true, CP>), grid, dim3(256), 0, st, P, C, recq, rec, flags, inst_off, tiles, dlang); \
        else hipLaunchKernelGGL((k_reduce_lang<false, CP>), grid, dim3(256), 0, st, P, C, recq, rec, flags, inst_off, tiles, dlang); \
    }
    switch (cpad) {
        case 4: LSR_GO(4) break;
        case 8: LSR_GO(8) break;
        case 16: LSR_GO(16) break;
        case 32: LSR_GO(32) break;
        default: LSR_GO(64) break;
    }
#undef LSR_GO
}

}  // namespace lsr
