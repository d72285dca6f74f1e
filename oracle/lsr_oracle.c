/*
 * lsr_oracle.c -- CPU ORACLE for the 4D-LangSplat language-feature Gaussian rasterizer.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
 * leg may load this library, and only as the checker / CPU baseline.  The product path
 * (4dlangsplat_amd/, liblsr.so) never links, loads or calls anything under oracle/.
 *
 * What it restates
 *   The hot path behind gaussian_renderer.render() -> GaussianRasterizer
 *   (/root/reference/gaussian_renderer/__init__.py:15,49-63,79,219-228): preprocess, binning,
 *   front-to-back compositing of RGB + C language channels + depth, and the full backward.
 *   The rasterizer itself is the un-vendored submodule zrporz/4d-langsplat-rasterization
 *   (/root/reference/.gitmodules:4-6, directory empty, no commit pinned).  It is the graphdeco
 *   diff-gaussian-rasterization lineage with the LangSplat language-feature channels and the
 *   4DGS depth output.  Its published algorithm is restated here with every constant named
 *   (SURVEY.md section 8a rows a8-a12):
 *     near cull z_view <= 0.2, p_w = 1/(w + 1e-7), EWA cov2D with the 1.3*tanfov clamp and the
 *     +0.3 low-pass, det == 0 cull, lambda = mid +- sqrt(max(0.1, mid^2 - det)),
 *     radius = ceil(3 sqrt(lambda_max)), ndc2Pix, 16x16 tiles, SH deg <= 3 with +0.5 and a
 *     clamp at 0 (clamped channels get no gradient), alpha = min(0.99, o G), skip
 *     alpha < 1/255, stop when T (1 - alpha) < 1e-4, RGB += T bg, language channels without
 *     a background term, depth = sum z alpha T, per-tile order = (depth, index) (the upstream
 *     stable radix sort of (tile << 32 | depth bits) keys), backward replays back-to-front
 *     with the accum_rec recurrence, ignores the 0.99 alpha clamp, keeps the x/y gradient
 *     gate of the tan-fov clamp, and reports means2D gradients in NDC units (x 0.5 W, 0.5 H).
 *   Python twins inside the reference that this file agrees with:
 *     utils/sh_utils.py:26-112 (SH constants and eval_sh), utils/general_utils.py:84-116
 *     (quaternion -> R, R S, covariance), utils/graphics_utils.py:38-71 (matrix convention),
 *     gaussian_renderer/__init__.py:198-205 (+0.5 then clamp_min 0).
 *
 * Parity status
 *   PARITY UNPINNED against the CUDA rasterizer: its source is absent from /root/reference and
 *   cannot be built or imported here, and the reference ships no tests or fixtures for it
 *   (SURVEY.md section 0 and 8c).  The pieces that have a Python twin in the reference are
 *   pinned by golden vectors generated from the reference itself (tests/golden/make_golden.py):
 *   SH -> RGB, the camera matrices, and the quaternion/scale covariance.  The backward is
 *   pinned by fp64 finite differences (compile with -DORC_DOUBLE) wherever no clamp is active.
 *
 * Floating point
 *   Compiled with -ffp-contract=off.  exp() of the Gaussian falloff uses orc_exp, a
 *   Cody-Waite + degree-5 minimax exp (<= 2.16 ulp) written only with IEEE max, *, +, fmaf and
 *   exponent bit assembly, and the falloff exponent is orc_power (two fmaf), so that the product
 *   kernels reproduce the contributor decisions (alpha < 1/255, T < 1e-4) bit for bit.  The CUDA
 *   original uses expf (<= 2 ulp) and nvcc's default fma contraction.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifdef ORC_DOUBLE
typedef double real;
#define R(x) (x)
#define RSQRT sqrt
#define RCEIL ceil
#define RMIN fmin
#define RMAX fmax
static inline real orc_exp(real x) { return exp(x); }
#else
typedef float real;
#define R(x) (x##f)
#define RSQRT sqrtf
#define RCEIL ceilf
#define RMIN fminf
#define RMAX fmaxf
#endif

#if !defined(ORC_DOUBLE) && defined(ORC_UPSTREAM_ARITH)
/* Upstream-arithmetic float build (liborc_f32_up.so, compiled with -ffp-contract=fast -mfma):
 * libm expf and the upstream falloff expression, every a*b+c free to contract as nvcc's default
 * does.  It stands in for the CUDA build's rounding, so that tests can bound how far the
 * reproducible build's contributor decisions (orc_exp / orc_power below) drift from it. */
static inline float orc_exp(float x) { return expf(x); }
#elif !defined(ORC_DOUBLE)
/* exp for x <= 0; bit-reproducible with the HIP kernels' expf_repro (lsr_common.h): the same
 * sequence of correctly rounded operations (fmaxf, fmaf, +, *).  The argument is clamped at -87
 * (every alpha from exp(-87) ~ 1.6e-38 is far below 1/255); k = rint(x log2 e) is
 * fmaf(x, log2 e, 1.5 2^23) - 1.5 2^23, e^r by a degree-5 minimax polynomial on [-ln2/2, ln2/2]
 * (tools/exp_minimax.py, float coefficients, <= 2.16 ulp overall) and 2^k assembled from the low
 * bits of that fmaf's result. */
static inline float orc_exp(float x) {
    x = fmaxf(x, -87.0f);
    const float y = fmaf(x, 1.44269504088896341f, 12582912.0f);
    const float kf = y - 12582912.0f;
    float r = fmaf(kf, -0.693145751953125f, x);
    r = fmaf(kf, -1.428606765330187045e-06f, r);
    float p = 0.008314719423651695f;
    p = fmaf(p, r, 0.041890207678079605f);
    p = fmaf(p, r, 0.16667090356349945f);
    p = fmaf(p, r, 0.499992311000824f);
    p = fmaf(p, r, 1.0f);
    p = fmaf(p, r, 1.0f);
    union { uint32_t u; float f; } yb, s;
    yb.f = y;
    s.u = (yb.u << 23) + 0x3F800000u;
    return p * s.f;
}
#endif

/* Gaussian falloff exponent at d = (dx, dy) = centre - pixel:
 *   power = -(a dx^2 + c dy^2)/2 - b dx dy = dx (A dx + B dy) + (C dy) dy,  (A, B, C) = (-a/2, -b, -c/2)
 * the HIP kernels' gauss_power (lsr_common.h) operation for operation (the scalings are exact). */
static inline real orc_power(const real *co, real dx, real dy) {
#if defined(ORC_UPSTREAM_ARITH) && !defined(ORC_DOUBLE)
    return R(-0.5) * (co[0] * dx * dx + co[2] * dy * dy) - co[1] * dx * dy;   /* upstream renderCUDA */
#else
    const real A = R(-0.5) * co[0], B = -co[1], Cq = R(-0.5) * co[2];
#ifdef ORC_DOUBLE
    return fma(dx, fma(A, dx, B * dy), (Cq * dy) * dy);
#else
    return fmaf(dx, fmaf(A, dx, B * dy), (Cq * dy) * dy);
#endif
#endif
}

#define BLOCK_X 16
#define BLOCK_Y 16

static const real SH_C0 = R(0.28209479177387814);
static const real SH_C1 = R(0.4886025119029199);
static const real SH_C2[5] = {R(1.0925484305920792), R(-1.0925484305920792), R(0.31539156525252005),
                              R(-1.0925484305920792), R(0.5462742152960396)};
static const real SH_C3[7] = {R(-0.5900435899266435), R(2.890611442640554), R(-0.4570457994644658),
                              R(0.3731763325901154), R(-0.4570457994644658), R(1.445305721320277),
                              R(-0.5900435899266435)};

typedef struct orc_settings {
    int H, W;
    real tanfovx, tanfovy;
    real bg[3];
    real scale_modifier;
    real view[16];  /* world_view_transform, flat row-major torch tensor (row-vector convention) */
    real proj[16];  /* full_proj_transform */
    int sh_degree;
    real campos[3];
    int include_feature;
} orc_settings;

typedef struct orc_state {
    int P, M, C, H, W, tiles_x, tiles_y;
    int64_t num_rendered;
    real *xy;          /* [P,2] pixel-space means */
    real *depth;       /* [P]   view-space z */
    real *conic_o;     /* [P,4] conic (a, b, c) + opacity */
    real *rgb;         /* [P,3] SH colour (or colors_precomp copy) */
    uint8_t *clamped;  /* [P,3] */
    int *radii;        /* [P] */
    uint32_t *tiles;   /* [P] tiles touched */
    uint32_t *point_list; /* [K] Gaussian ids, tile-major, (depth, id) order inside a tile */
    uint32_t *tile_of;    /* [K] tile id of every list entry */
    uint32_t *ranges;     /* [tiles, 2] */
    real *final_T;        /* [H*W] */
    uint32_t *n_contrib;  /* [H*W] */
} orc_state;

/* ---- small helpers (auxiliary.h of the graphdeco lineage) ------------------------------- */
static inline real ndc2pix(real v, int S) { return ((v + R(1.0)) * (real)S - R(1.0)) * R(0.5); }

static inline void xform4x3(const real *m, const real *p, real *o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
}
static inline void xform4x4(const real *m, const real *p, real *o) {
    o[0] = m[0] * p[0] + m[4] * p[1] + m[8] * p[2] + m[12];
    o[1] = m[1] * p[0] + m[5] * p[1] + m[9] * p[2] + m[13];
    o[2] = m[2] * p[0] + m[6] * p[1] + m[10] * p[2] + m[14];
    o[3] = m[3] * p[0] + m[7] * p[1] + m[11] * p[2] + m[15];
}
static inline int imin(int a, int b) { return a < b ? a : b; }
static inline int imax(int a, int b) { return a > b ? a : b; }

static void get_rect(const real *p, int max_radius, int gx, int gy, int *rmin, int *rmax) {
    rmin[0] = imin(gx, imax(0, (int)((p[0] - (real)max_radius) / (real)BLOCK_X)));
    rmin[1] = imin(gy, imax(0, (int)((p[1] - (real)max_radius) / (real)BLOCK_Y)));
    rmax[0] = imin(gx, imax(0, (int)((p[0] + (real)max_radius + (real)(BLOCK_X - 1)) / (real)BLOCK_X)));
    rmax[1] = imin(gy, imax(0, (int)((p[1] + (real)max_radius + (real)(BLOCK_Y - 1)) / (real)BLOCK_Y)));
}

/* glm-style 3x3 (column-major m[c][r]) helpers so the operation order follows the original. */
typedef struct { real m[3][3]; } mat3;
static mat3 mat3_mul(const mat3 *a, const mat3 *b) {
    mat3 o;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r)
            o.m[c][r] = a->m[0][r] * b->m[c][0] + a->m[1][r] * b->m[c][1] + a->m[2][r] * b->m[c][2];
    return o;
}
static mat3 mat3_T(const mat3 *a) {
    mat3 o;
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) o.m[c][r] = a->m[r][c];
    return o;
}

/* quaternion (r, x, y, z) -> glm rotation (utils/general_utils.py:84-105 twin, column-major) */
static mat3 quat_to_R(const real *q) {
    const real r = q[0], x = q[1], y = q[2], z = q[3];
    mat3 R;
    R.m[0][0] = R(1.0) - R(2.0) * (y * y + z * z); R.m[0][1] = R(2.0) * (x * y - r * z); R.m[0][2] = R(2.0) * (x * z + r * y);
    R.m[1][0] = R(2.0) * (x * y + r * z); R.m[1][1] = R(1.0) - R(2.0) * (x * x + z * z); R.m[1][2] = R(2.0) * (y * z - r * x);
    R.m[2][0] = R(2.0) * (x * z - r * y); R.m[2][1] = R(2.0) * (y * z + r * x); R.m[2][2] = R(1.0) - R(2.0) * (x * x + y * y);
    return R;
}

/* cov3D (upper 6) from scale * mod and an (un-normalised) quaternion: Sigma = M^T M, M = S R */
static void compute_cov3d(const real *scale, real mod, const real *rot, real *cov) {
    mat3 S; memset(&S, 0, sizeof S);
    S.m[0][0] = mod * scale[0]; S.m[1][1] = mod * scale[1]; S.m[2][2] = mod * scale[2];
    mat3 Rm = quat_to_R(rot);
    mat3 M = mat3_mul(&S, &Rm);
    mat3 Mt = mat3_T(&M);
    mat3 Sig = mat3_mul(&Mt, &M);
    cov[0] = Sig.m[0][0]; cov[1] = Sig.m[0][1]; cov[2] = Sig.m[0][2];
    cov[3] = Sig.m[1][1]; cov[4] = Sig.m[1][2]; cov[5] = Sig.m[2][2];
}

/* EWA projection of cov3D: returns (a, b, c) of cov2D + 0.3 I */
static void compute_cov2d(const real *mean, real fx, real fy, real tanfovx, real tanfovy,
                          const real *cov3D, const real *view, real *out) {
    real t[3];
    xform4x3(view, mean, t);
    const real limx = R(1.3) * tanfovx, limy = R(1.3) * tanfovy;
    const real txtz = t[0] / t[2], tytz = t[1] / t[2];
    t[0] = RMIN(limx, RMAX(-limx, txtz)) * t[2];
    t[1] = RMIN(limy, RMAX(-limy, tytz)) * t[2];
    mat3 J; memset(&J, 0, sizeof J);
    J.m[0][0] = fx / t[2]; J.m[0][2] = -(fx * t[0]) / (t[2] * t[2]);
    J.m[1][1] = fy / t[2]; J.m[1][2] = -(fy * t[1]) / (t[2] * t[2]);
    mat3 Wm;
    Wm.m[0][0] = view[0]; Wm.m[0][1] = view[4]; Wm.m[0][2] = view[8];
    Wm.m[1][0] = view[1]; Wm.m[1][1] = view[5]; Wm.m[1][2] = view[9];
    Wm.m[2][0] = view[2]; Wm.m[2][1] = view[6]; Wm.m[2][2] = view[10];
    mat3 T = mat3_mul(&Wm, &J);
    mat3 V;
    V.m[0][0] = cov3D[0]; V.m[0][1] = cov3D[1]; V.m[0][2] = cov3D[2];
    V.m[1][0] = cov3D[1]; V.m[1][1] = cov3D[3]; V.m[1][2] = cov3D[4];
    V.m[2][0] = cov3D[2]; V.m[2][1] = cov3D[4]; V.m[2][2] = cov3D[5];
    mat3 Tt = mat3_T(&T), Vt = mat3_T(&V);
    mat3 A = mat3_mul(&Tt, &Vt);
    mat3 cov = mat3_mul(&A, &T);
    out[0] = cov.m[0][0] + R(0.3);
    out[1] = cov.m[0][1];
    out[2] = cov.m[1][1] + R(0.3);
}

/* SH -> RGB (utils/sh_utils.py:57-112 twin), +0.5, clamp at 0, record clamped channels */
static void color_from_sh(int deg, int M, const real *pos, const real *campos, const real *sh,
                          real *rgb, uint8_t *clamped) {
    real dir[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
    const real len = RSQRT(dir[0] * dir[0] + dir[1] * dir[1] + dir[2] * dir[2]);
    dir[0] = dir[0] / len; dir[1] = dir[1] / len; dir[2] = dir[2] / len;
    (void)M;
    for (int ch = 0; ch < 3; ++ch) {
#define SHc(k) sh[(k) * 3 + ch]
        real res = SH_C0 * SHc(0);
        if (deg > 0) {
            const real x = dir[0], y = dir[1], z = dir[2];
            res = res - SH_C1 * y * SHc(1) + SH_C1 * z * SHc(2) - SH_C1 * x * SHc(3);
            if (deg > 1) {
                const real xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                res = res + SH_C2[0] * xy * SHc(4) + SH_C2[1] * yz * SHc(5) +
                      SH_C2[2] * (R(2.0) * zz - xx - yy) * SHc(6) + SH_C2[3] * xz * SHc(7) +
                      SH_C2[4] * (xx - yy) * SHc(8);
                if (deg > 2) {
                    res = res + SH_C3[0] * y * (R(3.0) * xx - yy) * SHc(9) + SH_C3[1] * xy * z * SHc(10) +
                          SH_C3[2] * y * (R(4.0) * zz - xx - yy) * SHc(11) +
                          SH_C3[3] * z * (R(2.0) * zz - R(3.0) * xx - R(3.0) * yy) * SHc(12) +
                          SH_C3[4] * x * (R(4.0) * zz - xx - yy) * SHc(13) + SH_C3[5] * z * (xx - yy) * SHc(14) +
                          SH_C3[6] * x * (xx - R(3.0) * yy) * SHc(15);
                }
            }
        }
#undef SHc
        res = res + R(0.5);
        clamped[ch] = res < R(0.0);
        rgb[ch] = res < R(0.0) ? R(0.0) : res;
    }
}

/* ---- sort of (tile, depth bits, id) -------------------------------------------------------- */
typedef struct { uint32_t tile; real depth; uint32_t id; } orc_key;
static int key_cmp(const void *pa, const void *pb) {
    const orc_key *a = (const orc_key *)pa, *b = (const orc_key *)pb;
    if (a->tile != b->tile) return a->tile < b->tile ? -1 : 1;
    if (a->depth != b->depth) return a->depth < b->depth ? -1 : 1;  /* depth > 0.2: float order == bit order */
    if (a->id != b->id) return a->id < b->id ? -1 : 1;
    return 0;
}

/* ---- forward -------------------------------------------------------------------------------- */
orc_state *orc_forward(const orc_settings *s, int P, int M, int C,
                       const real *means3D, const real *shs, const real *colors_precomp,
                       const real *lang, const real *opacities, const real *scales,
                       const real *rotations, const real *cov3D_precomp,
                       real *out_color, real *out_lang, real *out_depth, int *out_radii, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    orc_state *st = (orc_state *)calloc(1, sizeof(orc_state));
    const int H = s->H, W = s->W;
    const int gx = (W + BLOCK_X - 1) / BLOCK_X, gy = (H + BLOCK_Y - 1) / BLOCK_Y;
    st->P = P; st->M = M; st->C = C; st->H = H; st->W = W; st->tiles_x = gx; st->tiles_y = gy;
    st->xy = (real *)calloc((size_t)P * 2 + 1, sizeof(real));
    st->depth = (real *)calloc((size_t)P + 1, sizeof(real));
    st->conic_o = (real *)calloc((size_t)P * 4 + 1, sizeof(real));
    st->rgb = (real *)calloc((size_t)P * 3 + 1, sizeof(real));
    st->clamped = (uint8_t *)calloc((size_t)P * 3 + 1, 1);
    st->radii = (int *)calloc((size_t)P + 1, sizeof(int));
    st->tiles = (uint32_t *)calloc((size_t)P + 1, sizeof(uint32_t));
    st->ranges = (uint32_t *)calloc((size_t)gx * gy * 2 + 1, sizeof(uint32_t));
    st->final_T = (real *)calloc((size_t)H * W + 1, sizeof(real));
    st->n_contrib = (uint32_t *)calloc((size_t)H * W + 1, sizeof(uint32_t));

    const real fx = (real)W / (R(2.0) * s->tanfovx);
    const real fy = (real)H / (R(2.0) * s->tanfovy);

    /* preprocess: one Gaussian at a time (preprocessCUDA) */
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; ++i) {
        st->radii[i] = 0; st->tiles[i] = 0;
        const real *p = means3D + 3 * (size_t)i;
        real ph[4], pv[3];
        xform4x4(s->proj, p, ph);
        xform4x3(s->view, p, pv);
        if (pv[2] <= R(0.2)) continue;                      /* in_frustum */
        const real pw = R(1.0) / (ph[3] + R(0.0000001));
        const real pp[3] = {ph[0] * pw, ph[1] * pw, ph[2] * pw};
        real cov3[6];
        const real *c3;
        if (cov3D_precomp) c3 = cov3D_precomp + 6 * (size_t)i;
        else { compute_cov3d(scales + 3 * (size_t)i, s->scale_modifier, rotations + 4 * (size_t)i, cov3); c3 = cov3; }
        real cov[3];
        compute_cov2d(p, fx, fy, s->tanfovx, s->tanfovy, c3, s->view, cov);
        const real det = cov[0] * cov[2] - cov[1] * cov[1];
        if (det == R(0.0)) continue;
        const real det_inv = R(1.0) / det;
        const real conic[3] = {cov[2] * det_inv, -cov[1] * det_inv, cov[0] * det_inv};
        const real mid = R(0.5) * (cov[0] + cov[2]);
        const real l1 = mid + RSQRT(RMAX(R(0.1), mid * mid - det));
        const real l2 = mid - RSQRT(RMAX(R(0.1), mid * mid - det));
        const int radius = (int)RCEIL(R(3.0) * RSQRT(RMAX(l1, l2)));
        const real pix[2] = {ndc2pix(pp[0], W), ndc2pix(pp[1], H)};
        int rmin[2], rmax[2];
        get_rect(pix, radius, gx, gy, rmin, rmax);
        if ((rmax[0] - rmin[0]) * (rmax[1] - rmin[1]) == 0) continue;
        if (!colors_precomp) {
            color_from_sh(s->sh_degree, M, p, s->campos, shs + (size_t)i * M * 3, st->rgb + 3 * (size_t)i,
                          st->clamped + 3 * (size_t)i);
        } else {
            for (int c = 0; c < 3; ++c) st->rgb[3 * (size_t)i + c] = colors_precomp[3 * (size_t)i + c];
        }
        st->depth[i] = pv[2];
        st->radii[i] = radius;
        st->xy[2 * (size_t)i] = pix[0]; st->xy[2 * (size_t)i + 1] = pix[1];
        st->conic_o[4 * (size_t)i + 0] = conic[0]; st->conic_o[4 * (size_t)i + 1] = conic[1];
        st->conic_o[4 * (size_t)i + 2] = conic[2]; st->conic_o[4 * (size_t)i + 3] = opacities[i];
        st->tiles[i] = (uint32_t)((rmax[1] - rmin[1]) * (rmax[0] - rmin[0]));
    }
    for (int i = 0; i < P; ++i) out_radii[i] = st->radii[i];

    /* binning: every (Gaussian, tile) instance, ordered by (tile, depth, id) */
    int64_t K = 0;
    for (int i = 0; i < P; ++i) K += st->tiles[i];
    st->num_rendered = K;
    orc_key *keys = (orc_key *)malloc(sizeof(orc_key) * (size_t)(K + 1));
    int64_t e = 0;
    for (int i = 0; i < P; ++i) {
        if (st->radii[i] <= 0) continue;
        int rmin[2], rmax[2];
        get_rect(st->xy + 2 * (size_t)i, st->radii[i], gx, gy, rmin, rmax);
        for (int y = rmin[1]; y < rmax[1]; ++y)
            for (int x = rmin[0]; x < rmax[0]; ++x) {
                keys[e].tile = (uint32_t)(y * gx + x);
                keys[e].depth = st->depth[i];
                keys[e].id = (uint32_t)i;
                ++e;
            }
    }
    qsort(keys, (size_t)K, sizeof(orc_key), key_cmp);
    st->point_list = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(K + 1));
    st->tile_of = (uint32_t *)malloc(sizeof(uint32_t) * (size_t)(K + 1));
    for (int64_t k = 0; k < K; ++k) { st->point_list[k] = keys[k].id; st->tile_of[k] = keys[k].tile; }
    free(keys);
    for (int64_t k = 0; k < K; ++k) {
        const uint32_t t = st->tile_of[k];
        if (k == 0 || st->tile_of[k - 1] != t) st->ranges[2 * t] = (uint32_t)k;
        if (k == K - 1 || st->tile_of[k + 1] != t) st->ranges[2 * t + 1] = (uint32_t)(k + 1);
    }

    /* render: one pixel at a time, front to back (renderCUDA) */
    const int feat = s->include_feature && C > 0;
    const size_t HW = (size_t)H * W;
#pragma omp parallel for schedule(dynamic, 1)
    for (int tile = 0; tile < gx * gy; ++tile) {
        const int tx = tile % gx, ty = tile / gx;
        const uint32_t r0 = st->ranges[2 * tile], r1 = st->ranges[2 * tile + 1];
        real *F = (real *)malloc(sizeof(real) * (size_t)(C > 0 ? C : 1));
        for (int py = ty * BLOCK_Y; py < imin(ty * BLOCK_Y + BLOCK_Y, H); ++py)
            for (int px = tx * BLOCK_X; px < imin(tx * BLOCK_X + BLOCK_X, W); ++px) {
                const size_t pid = (size_t)py * W + px;
                real T = R(1.0), Cc[3] = {0, 0, 0}, D = 0;
                for (int c = 0; c < C; ++c) F[c] = 0;
                uint32_t contributor = 0, last = 0;
                for (uint32_t k = r0; k < r1; ++k) {
                    contributor++;
                    const uint32_t g = st->point_list[k];
                    const real *xy = st->xy + 2 * (size_t)g, *co = st->conic_o + 4 * (size_t)g;
                    const real dx = xy[0] - (real)px, dy = xy[1] - (real)py;
                    const real power = orc_power(co, dx, dy);
                    if (power > R(0.0)) continue;
                    const real alpha = RMIN(R(0.99), co[3] * orc_exp(power));
                    if (alpha < R(1.0) / R(255.0)) continue;
                    const real test_T = T * (R(1.0) - alpha);
                    if (test_T < R(0.0001)) break;      /* done = true */
                    for (int c = 0; c < 3; ++c) Cc[c] += st->rgb[3 * (size_t)g + c] * alpha * T;
                    if (feat)
                        for (int c = 0; c < C; ++c) F[c] += lang[(size_t)g * C + c] * alpha * T;
                    D += st->depth[g] * alpha * T;
                    T = test_T;
                    last = contributor;
                }
                st->final_T[pid] = T;
                st->n_contrib[pid] = last;
                for (int c = 0; c < 3; ++c) out_color[c * HW + pid] = Cc[c] + T * s->bg[c];
                for (int c = 0; c < C; ++c) out_lang[c * HW + pid] = feat ? F[c] : R(0.0);
                out_depth[pid] = D;
            }
        free(F);
    }
    return st;
}

/* ---- backward ------------------------------------------------------------------------------- */
#ifdef _OPENMP
#define ATOMIC_ADD(dst, v) do { real _v = (v); _Pragma("omp atomic") (dst) += _v; } while (0)
#else
#define ATOMIC_ADD(dst, v) ((dst) += (v))
#endif

static void cov2d_backward(const real *mean, const real *cov3D, real fx, real fy, real tanfovx,
                           real tanfovy, const real *view, const real *dL_dconic /*x,y,w*/,
                           real *dL_dmean, real *dL_dcov) {
    real t[3];
    xform4x3(view, mean, t);
    const real limx = R(1.3) * tanfovx, limy = R(1.3) * tanfovy;
    const real txtz = t[0] / t[2], tytz = t[1] / t[2];
    t[0] = RMIN(limx, RMAX(-limx, txtz)) * t[2];
    t[1] = RMIN(limy, RMAX(-limy, tytz)) * t[2];
    const real x_grad_mul = (txtz < -limx || txtz > limx) ? R(0.0) : R(1.0);
    const real y_grad_mul = (tytz < -limy || tytz > limy) ? R(0.0) : R(1.0);
    mat3 J; memset(&J, 0, sizeof J);
    J.m[0][0] = fx / t[2]; J.m[0][2] = -(fx * t[0]) / (t[2] * t[2]);
    J.m[1][1] = fy / t[2]; J.m[1][2] = -(fy * t[1]) / (t[2] * t[2]);
    mat3 Wm;
    Wm.m[0][0] = view[0]; Wm.m[0][1] = view[4]; Wm.m[0][2] = view[8];
    Wm.m[1][0] = view[1]; Wm.m[1][1] = view[5]; Wm.m[1][2] = view[9];
    Wm.m[2][0] = view[2]; Wm.m[2][1] = view[6]; Wm.m[2][2] = view[10];
    mat3 V;
    V.m[0][0] = cov3D[0]; V.m[0][1] = cov3D[1]; V.m[0][2] = cov3D[2];
    V.m[1][0] = cov3D[1]; V.m[1][1] = cov3D[3]; V.m[1][2] = cov3D[4];
    V.m[2][0] = cov3D[2]; V.m[2][1] = cov3D[4]; V.m[2][2] = cov3D[5];
    mat3 T = mat3_mul(&Wm, &J);
    mat3 Tt = mat3_T(&T), Vt = mat3_T(&V);
    mat3 A = mat3_mul(&Tt, &Vt);
    mat3 cov2 = mat3_mul(&A, &T);
    const real a = cov2.m[0][0] + R(0.3), b = cov2.m[0][1], c = cov2.m[1][1] + R(0.3);
    const real denom = a * c - b * b;
    real dL_da = 0, dL_db = 0, dL_dc = 0;
    const real denom2inv = R(1.0) / ((denom * denom) + R(0.0000001));
    if (denom2inv != R(0.0)) {
        dL_da = denom2inv * (-c * c * dL_dconic[0] + R(2.0) * b * c * dL_dconic[1] + (denom - a * c) * dL_dconic[2]);
        dL_dc = denom2inv * (-a * a * dL_dconic[2] + R(2.0) * a * b * dL_dconic[1] + (denom - a * c) * dL_dconic[0]);
        dL_db = denom2inv * R(2.0) * (b * c * dL_dconic[0] - (denom + R(2.0) * b * b) * dL_dconic[1] + a * b * dL_dconic[2]);
        const real (*Tm)[3] = T.m;
        dL_dcov[0] = Tm[0][0] * Tm[0][0] * dL_da + Tm[0][0] * Tm[1][0] * dL_db + Tm[1][0] * Tm[1][0] * dL_dc;
        dL_dcov[3] = Tm[0][1] * Tm[0][1] * dL_da + Tm[0][1] * Tm[1][1] * dL_db + Tm[1][1] * Tm[1][1] * dL_dc;
        dL_dcov[5] = Tm[0][2] * Tm[0][2] * dL_da + Tm[0][2] * Tm[1][2] * dL_db + Tm[1][2] * Tm[1][2] * dL_dc;
        dL_dcov[1] = R(2.0) * Tm[0][0] * Tm[0][1] * dL_da + (Tm[0][0] * Tm[1][1] + Tm[0][1] * Tm[1][0]) * dL_db + R(2.0) * Tm[1][0] * Tm[1][1] * dL_dc;
        dL_dcov[2] = R(2.0) * Tm[0][0] * Tm[0][2] * dL_da + (Tm[0][0] * Tm[1][2] + Tm[0][2] * Tm[1][0]) * dL_db + R(2.0) * Tm[1][0] * Tm[1][2] * dL_dc;
        dL_dcov[4] = R(2.0) * Tm[0][2] * Tm[0][1] * dL_da + (Tm[0][1] * Tm[1][2] + Tm[0][2] * Tm[1][1]) * dL_db + R(2.0) * Tm[1][1] * Tm[1][2] * dL_dc;
    } else {
        for (int i = 0; i < 6; ++i) dL_dcov[i] = 0;
    }
    const real (*Tm)[3] = T.m;
    const real (*Vm)[3] = V.m;
    const real dL_dT00 = R(2.0) * (Tm[0][0] * Vm[0][0] + Tm[0][1] * Vm[0][1] + Tm[0][2] * Vm[0][2]) * dL_da +
                         (Tm[1][0] * Vm[0][0] + Tm[1][1] * Vm[0][1] + Tm[1][2] * Vm[0][2]) * dL_db;
    const real dL_dT01 = R(2.0) * (Tm[0][0] * Vm[1][0] + Tm[0][1] * Vm[1][1] + Tm[0][2] * Vm[1][2]) * dL_da +
                         (Tm[1][0] * Vm[1][0] + Tm[1][1] * Vm[1][1] + Tm[1][2] * Vm[1][2]) * dL_db;
    const real dL_dT02 = R(2.0) * (Tm[0][0] * Vm[2][0] + Tm[0][1] * Vm[2][1] + Tm[0][2] * Vm[2][2]) * dL_da +
                         (Tm[1][0] * Vm[2][0] + Tm[1][1] * Vm[2][1] + Tm[1][2] * Vm[2][2]) * dL_db;
    const real dL_dT10 = R(2.0) * (Tm[1][0] * Vm[0][0] + Tm[1][1] * Vm[0][1] + Tm[1][2] * Vm[0][2]) * dL_dc +
                         (Tm[0][0] * Vm[0][0] + Tm[0][1] * Vm[0][1] + Tm[0][2] * Vm[0][2]) * dL_db;
    const real dL_dT11 = R(2.0) * (Tm[1][0] * Vm[1][0] + Tm[1][1] * Vm[1][1] + Tm[1][2] * Vm[1][2]) * dL_dc +
                         (Tm[0][0] * Vm[1][0] + Tm[0][1] * Vm[1][1] + Tm[0][2] * Vm[1][2]) * dL_db;
    const real dL_dT12 = R(2.0) * (Tm[1][0] * Vm[2][0] + Tm[1][1] * Vm[2][1] + Tm[1][2] * Vm[2][2]) * dL_dc +
                         (Tm[0][0] * Vm[2][0] + Tm[0][1] * Vm[2][1] + Tm[0][2] * Vm[2][2]) * dL_db;
    const real (*Wq)[3] = Wm.m;
    const real dL_dJ00 = Wq[0][0] * dL_dT00 + Wq[0][1] * dL_dT01 + Wq[0][2] * dL_dT02;
    const real dL_dJ02 = Wq[2][0] * dL_dT00 + Wq[2][1] * dL_dT01 + Wq[2][2] * dL_dT02;
    const real dL_dJ11 = Wq[1][0] * dL_dT10 + Wq[1][1] * dL_dT11 + Wq[1][2] * dL_dT12;
    const real dL_dJ12 = Wq[2][0] * dL_dT10 + Wq[2][1] * dL_dT11 + Wq[2][2] * dL_dT12;
    const real tz = R(1.0) / t[2], tz2 = tz * tz, tz3 = tz2 * tz;
    const real dL_dtx = x_grad_mul * -fx * tz2 * dL_dJ02;
    const real dL_dty = y_grad_mul * -fy * tz2 * dL_dJ12;
    const real dL_dtz = -fx * tz2 * dL_dJ00 - fy * tz2 * dL_dJ11 + (R(2.0) * fx * t[0]) * tz3 * dL_dJ02 +
                        (R(2.0) * fy * t[1]) * tz3 * dL_dJ12;
    /* transformVec4x3Transpose */
    dL_dmean[0] = view[0] * dL_dtx + view[1] * dL_dty + view[2] * dL_dtz;
    dL_dmean[1] = view[4] * dL_dtx + view[5] * dL_dty + view[6] * dL_dtz;
    dL_dmean[2] = view[8] * dL_dtx + view[9] * dL_dty + view[10] * dL_dtz;
}

static void cov3d_backward(const real *scale, real mod, const real *rot, const real *dL_dcov,
                           real *dL_dscale, real *dL_drot) {
    const real r = rot[0], x = rot[1], y = rot[2], z = rot[3];
    mat3 Rm = quat_to_R(rot);
    const real s[3] = {mod * scale[0], mod * scale[1], mod * scale[2]};
    mat3 S; memset(&S, 0, sizeof S);
    S.m[0][0] = s[0]; S.m[1][1] = s[1]; S.m[2][2] = s[2];
    mat3 M = mat3_mul(&S, &Rm);
    mat3 dS;  /* dL_dSigma, symmetric, off-diagonals halved */
    dS.m[0][0] = dL_dcov[0]; dS.m[0][1] = R(0.5) * dL_dcov[1]; dS.m[0][2] = R(0.5) * dL_dcov[2];
    dS.m[1][0] = R(0.5) * dL_dcov[1]; dS.m[1][1] = dL_dcov[3]; dS.m[1][2] = R(0.5) * dL_dcov[4];
    dS.m[2][0] = R(0.5) * dL_dcov[2]; dS.m[2][1] = R(0.5) * dL_dcov[4]; dS.m[2][2] = dL_dcov[5];
    mat3 M2;
    for (int c = 0; c < 3; ++c)
        for (int q = 0; q < 3; ++q) M2.m[c][q] = R(2.0) * M.m[c][q];
    mat3 dM = mat3_mul(&M2, &dS);
    mat3 Rt = mat3_T(&Rm), dMt = mat3_T(&dM);
    /* dL/ds_k = dot(Rt[k], dMt[k]); times mod for dL/dscale ("x mod") */
    for (int k = 0; k < 3; ++k)
        dL_dscale[k] = (Rt.m[k][0] * dMt.m[k][0] + Rt.m[k][1] * dMt.m[k][1] + Rt.m[k][2] * dMt.m[k][2]) * mod;
    for (int q = 0; q < 3; ++q) { dMt.m[0][q] *= s[0]; dMt.m[1][q] *= s[1]; dMt.m[2][q] *= s[2]; }
    const real (*d)[3] = dMt.m;
    dL_drot[0] = R(2.0) * z * (d[0][1] - d[1][0]) + R(2.0) * y * (d[2][0] - d[0][2]) + R(2.0) * x * (d[1][2] - d[2][1]);
    dL_drot[1] = R(2.0) * y * (d[1][0] + d[0][1]) + R(2.0) * z * (d[2][0] + d[0][2]) + R(2.0) * r * (d[1][2] - d[2][1]) -
                 R(4.0) * x * (d[2][2] + d[1][1]);
    dL_drot[2] = R(2.0) * x * (d[1][0] + d[0][1]) + R(2.0) * r * (d[2][0] - d[0][2]) + R(2.0) * z * (d[1][2] + d[2][1]) -
                 R(4.0) * y * (d[2][2] + d[0][0]);
    dL_drot[3] = R(2.0) * r * (d[0][1] - d[1][0]) + R(2.0) * x * (d[2][0] + d[0][2]) + R(2.0) * y * (d[1][2] + d[2][1]) -
                 R(4.0) * z * (d[1][1] + d[0][0]);
}

static void sh_backward(int deg, int M, const real *pos, const real *campos, const real *sh,
                        const uint8_t *clamped, const real *dL_dcolor, real *dL_dsh, real *dL_dmean) {
    const real dir_orig[3] = {pos[0] - campos[0], pos[1] - campos[1], pos[2] - campos[2]};
    const real len = RSQRT(dir_orig[0] * dir_orig[0] + dir_orig[1] * dir_orig[1] + dir_orig[2] * dir_orig[2]);
    const real x = dir_orig[0] / len, y = dir_orig[1] / len, z = dir_orig[2] / len;
    real dRGB[3];
    for (int c = 0; c < 3; ++c) dRGB[c] = clamped[c] ? R(0.0) : dL_dcolor[c];
    (void)M;
    real dRdx[3] = {0, 0, 0}, dRdy[3] = {0, 0, 0}, dRdz[3] = {0, 0, 0};
    for (int c = 0; c < 3; ++c) {
#define SHc(k) sh[(k) * 3 + c]
#define DSH(k) dL_dsh[(k) * 3 + c]
        DSH(0) = SH_C0 * dRGB[c];
        if (deg > 0) {
            DSH(1) = -SH_C1 * y * dRGB[c];
            DSH(2) = SH_C1 * z * dRGB[c];
            DSH(3) = -SH_C1 * x * dRGB[c];
            dRdx[c] = -SH_C1 * SHc(3);
            dRdy[c] = -SH_C1 * SHc(1);
            dRdz[c] = SH_C1 * SHc(2);
            if (deg > 1) {
                const real xx = x * x, yy = y * y, zz = z * z, xy = x * y, yz = y * z, xz = x * z;
                DSH(4) = SH_C2[0] * xy * dRGB[c];
                DSH(5) = SH_C2[1] * yz * dRGB[c];
                DSH(6) = SH_C2[2] * (R(2.0) * zz - xx - yy) * dRGB[c];
                DSH(7) = SH_C2[3] * xz * dRGB[c];
                DSH(8) = SH_C2[4] * (xx - yy) * dRGB[c];
                dRdx[c] += SH_C2[0] * y * SHc(4) + SH_C2[2] * R(2.0) * -x * SHc(6) + SH_C2[3] * z * SHc(7) +
                           SH_C2[4] * R(2.0) * x * SHc(8);
                dRdy[c] += SH_C2[0] * x * SHc(4) + SH_C2[1] * z * SHc(5) + SH_C2[2] * R(2.0) * -y * SHc(6) +
                           SH_C2[4] * R(2.0) * -y * SHc(8);
                dRdz[c] += SH_C2[1] * y * SHc(5) + SH_C2[2] * R(2.0) * R(2.0) * z * SHc(6) + SH_C2[3] * x * SHc(7);
                if (deg > 2) {
                    DSH(9) = SH_C3[0] * y * (R(3.0) * xx - yy) * dRGB[c];
                    DSH(10) = SH_C3[1] * xy * z * dRGB[c];
                    DSH(11) = SH_C3[2] * y * (R(4.0) * zz - xx - yy) * dRGB[c];
                    DSH(12) = SH_C3[3] * z * (R(2.0) * zz - R(3.0) * xx - R(3.0) * yy) * dRGB[c];
                    DSH(13) = SH_C3[4] * x * (R(4.0) * zz - xx - yy) * dRGB[c];
                    DSH(14) = SH_C3[5] * z * (xx - yy) * dRGB[c];
                    DSH(15) = SH_C3[6] * x * (xx - R(3.0) * yy) * dRGB[c];
                    dRdx[c] += SH_C3[0] * SHc(9) * R(3.0) * R(2.0) * xy + SH_C3[1] * SHc(10) * yz +
                               SH_C3[2] * SHc(11) * -R(2.0) * xy + SH_C3[3] * SHc(12) * -R(3.0) * R(2.0) * xz +
                               SH_C3[4] * SHc(13) * (-R(3.0) * xx + R(4.0) * zz - yy) + SH_C3[5] * SHc(14) * R(2.0) * xz +
                               SH_C3[6] * SHc(15) * R(3.0) * (xx - yy);
                    dRdy[c] += SH_C3[0] * SHc(9) * R(3.0) * (xx - yy) + SH_C3[1] * SHc(10) * xz +
                               SH_C3[2] * SHc(11) * (-R(3.0) * yy + R(4.0) * zz - xx) + SH_C3[3] * SHc(12) * -R(3.0) * R(2.0) * yz +
                               SH_C3[4] * SHc(13) * -R(2.0) * xy + SH_C3[5] * SHc(14) * -R(2.0) * yz +
                               SH_C3[6] * SHc(15) * -R(3.0) * R(2.0) * xy;
                    dRdz[c] += SH_C3[1] * SHc(10) * xy + SH_C3[2] * SHc(11) * R(4.0) * R(2.0) * yz +
                               SH_C3[3] * SHc(12) * R(3.0) * (R(2.0) * zz - xx - yy) + SH_C3[4] * SHc(13) * R(4.0) * R(2.0) * xz +
                               SH_C3[5] * SHc(14) * (xx - yy);
                }
            }
        }
#undef SHc
#undef DSH
    }
    /* dL/ddir (dot over colour channels), then through the normalisation (dnormvdv) */
    const real dLdx = dRdx[0] * dRGB[0] + dRdx[1] * dRGB[1] + dRdx[2] * dRGB[2];
    const real dLdy = dRdy[0] * dRGB[0] + dRdy[1] * dRGB[1] + dRdy[2] * dRGB[2];
    const real dLdz = dRdz[0] * dRGB[0] + dRdz[1] * dRGB[1] + dRdz[2] * dRGB[2];
    const real sum2 = dir_orig[0] * dir_orig[0] + dir_orig[1] * dir_orig[1] + dir_orig[2] * dir_orig[2];
    const real invsum32 = R(1.0) / RSQRT(sum2 * sum2 * sum2);
    dL_dmean[0] += ((sum2 - dir_orig[0] * dir_orig[0]) * dLdx - dir_orig[1] * dir_orig[0] * dLdy - dir_orig[2] * dir_orig[0] * dLdz) * invsum32;
    dL_dmean[1] += (-dir_orig[0] * dir_orig[1] * dLdx + (sum2 - dir_orig[1] * dir_orig[1]) * dLdy - dir_orig[2] * dir_orig[1] * dLdz) * invsum32;
    dL_dmean[2] += (-dir_orig[0] * dir_orig[2] * dLdx - dir_orig[1] * dir_orig[2] * dLdy + (sum2 - dir_orig[2] * dir_orig[2]) * dLdz) * invsum32;
}

/* Conditioning mode (test infrastructure): while on, the compositing backward accumulates, for the
 * directly accumulated gradients -- dL/dlanguage, dL/dopacity and dL/dmean2D -- the sum over pixels of
 * the magnitude of every term an implementation's value is built from (dL/dalpha's channel products
 * and blended predecessors taken in absolute value, dG/dmean's two products likewise), i.e. the scale
 * relative to which any implementation's rounding of those sums is measured.  Every other output is
 * meaningless in this mode. */
static int g_abs_terms = 0;
void orc_set_abs_terms(int on) { g_abs_terms = on != 0; }
#define RABS(v) ((v) < R(0.0) ? -(v) : (v))
#define TERM(v) (g_abs_terms ? RABS(v) : (v))

/* dL_d* outputs are overwritten.  dL_ddepth_pix may be NULL (no depth gradient). */
void orc_backward(const orc_state *st, const orc_settings *s,
                  const real *means3D, const real *shs, const real *colors_precomp, const real *lang,
                  const real *opacities, const real *scales, const real *rotations, const real *cov3D_precomp,
                  const real *dL_dpix, const real *dL_dpix_lang, const real *dL_dpix_depth,
                  real *dL_dmeans3D, real *dL_dmeans2D, real *dL_dcolors, real *dL_dlang,
                  real *dL_dopacity, real *dL_dcov3D, real *dL_dsh, real *dL_dscales, real *dL_drots,
                  int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#else
    (void)nthreads;
#endif
    const int P = st->P, M = st->M, C = st->C, H = st->H, W = st->W, gx = st->tiles_x, gy = st->tiles_y;
    const size_t HW = (size_t)H * W;
    const int feat = s->include_feature && C > 0;
    (void)opacities;
    real *dL_dconic = (real *)calloc((size_t)P * 3 + 1, sizeof(real));
    real *dL_ddepth = (real *)calloc((size_t)P + 1, sizeof(real));
    memset(dL_dmeans2D, 0, sizeof(real) * 3 * (size_t)P);
    memset(dL_dcolors, 0, sizeof(real) * 3 * (size_t)P);
    memset(dL_dopacity, 0, sizeof(real) * (size_t)P);
    if (C > 0) memset(dL_dlang, 0, sizeof(real) * (size_t)C * P);
    const real ddelx_dx = R(0.5) * (real)W, ddely_dy = R(0.5) * (real)H;

#pragma omp parallel for schedule(dynamic, 1)
    for (int tile = 0; tile < gx * gy; ++tile) {
        const int tx = tile % gx, ty = tile / gx;
        const uint32_t r0 = st->ranges[2 * tile], r1 = st->ranges[2 * tile + 1];
        real *accF = (real *)malloc(sizeof(real) * (size_t)(C > 0 ? 3 * C : 3));
        real *lastF = accF + (C > 0 ? C : 1);
        real *accFA = lastF + (C > 0 ? C : 1);   /* conditioning mode: blends of |feature| */
        for (int py = ty * BLOCK_Y; py < imin(ty * BLOCK_Y + BLOCK_Y, H); ++py)
            for (int px = tx * BLOCK_X; px < imin(tx * BLOCK_X + BLOCK_X, W); ++px) {
                const size_t pid = (size_t)py * W + px;
                const real T_final = st->final_T[pid];
                real T = T_final;
                const uint32_t last_contributor = st->n_contrib[pid];
                uint32_t contributor = r1 - r0;
                real acc[3] = {0, 0, 0}, lastc[3] = {0, 0, 0}, accD = 0, lastD = 0, last_alpha = 0;
                real accA[3] = {0, 0, 0}, accDA = 0;   /* conditioning mode: blends of |colour|, |depth| */
                for (int c = 0; c < C; ++c) { accF[c] = 0; lastF[c] = 0; accFA[c] = 0; }
                real dpix[3];
                for (int c = 0; c < 3; ++c) dpix[c] = dL_dpix[c * HW + pid];
                const real dpixD = dL_dpix_depth ? dL_dpix_depth[pid] : R(0.0);
                for (uint32_t kk = r1; kk > r0; --kk) {
                    contributor--;
                    if (contributor >= last_contributor) continue;
                    const uint32_t g = st->point_list[kk - 1];
                    const real *xy = st->xy + 2 * (size_t)g, *co = st->conic_o + 4 * (size_t)g;
                    const real dx = xy[0] - (real)px, dy = xy[1] - (real)py;
                    const real power = orc_power(co, dx, dy);
                    if (power > R(0.0)) continue;
                    const real G = orc_exp(power);
                    const real alpha = RMIN(R(0.99), co[3] * G);
                    if (alpha < R(1.0) / R(255.0)) continue;
                    T = T / (R(1.0) - alpha);
                    const real dchannel_dcolor = alpha * T;
                    real dL_dalpha = 0;
                    /* conditioning mode: the scale of dL/dalpha's terms, T sum (|c| + blend |c_prev|) |dL/dpix|
                     * (an implementation's dot(c, dL/dpix) - acc rounds relative to it, not to the difference) */
                    real dLa_abs = 0;
                    for (int c = 0; c < 3; ++c) {
                        const real col = st->rgb[3 * (size_t)g + c];
                        if (g_abs_terms) {
                            accA[c] = last_alpha * RABS(lastc[c]) + (R(1.0) - last_alpha) * accA[c];
                            dLa_abs += (RABS(col) + accA[c]) * RABS(dpix[c]);
                        }
                        acc[c] = last_alpha * lastc[c] + (R(1.0) - last_alpha) * acc[c];
                        lastc[c] = col;
                        dL_dalpha += (col - acc[c]) * dpix[c];
                        ATOMIC_ADD(dL_dcolors[3 * (size_t)g + c], dchannel_dcolor * dpix[c]);
                    }
                    if (feat) {
                        for (int c = 0; c < C; ++c) {
                            const real f = lang[(size_t)g * C + c];
                            const real dF = dL_dpix_lang[c * HW + pid];
                            if (g_abs_terms) {
                                accFA[c] = last_alpha * RABS(lastF[c]) + (R(1.0) - last_alpha) * accFA[c];
                                dLa_abs += (RABS(f) + accFA[c]) * RABS(dF);
                            }
                            accF[c] = last_alpha * lastF[c] + (R(1.0) - last_alpha) * accF[c];
                            lastF[c] = f;
                            dL_dalpha += (f - accF[c]) * dF;
                            ATOMIC_ADD(dL_dlang[(size_t)g * C + c], TERM(dchannel_dcolor * dF));
                        }
                    }
                    {
                        const real dep = st->depth[g];
                        if (g_abs_terms) {
                            accDA = last_alpha * RABS(lastD) + (R(1.0) - last_alpha) * accDA;
                            dLa_abs += (RABS(dep) + accDA) * RABS(dpixD);
                        }
                        accD = last_alpha * lastD + (R(1.0) - last_alpha) * accD;
                        lastD = dep;
                        dL_dalpha += (dep - accD) * dpixD;
                        ATOMIC_ADD(dL_ddepth[g], dchannel_dcolor * dpixD);
                    }
                    dL_dalpha *= T;
                    last_alpha = alpha;
                    const real bg_dot = s->bg[0] * dpix[0] + s->bg[1] * dpix[1] + s->bg[2] * dpix[2];
                    dL_dalpha += (-T_final / (R(1.0) - alpha)) * bg_dot;
                    const real dL_dG = co[3] * dL_dalpha;
                    const real gdx = G * dx, gdy = G * dy;
                    const real dG_ddelx = -gdx * co[0] - gdy * co[1];
                    const real dG_ddely = -gdy * co[2] - gdx * co[1];
                    if (g_abs_terms) {
                        dLa_abs = dLa_abs * T + (T_final / (R(1.0) - alpha)) *
                                  (RABS(s->bg[0] * dpix[0]) + RABS(s->bg[1] * dpix[1]) + RABS(s->bg[2] * dpix[2]));
                        const real aG = RABS(co[3]) * dLa_abs;
                        ATOMIC_ADD(dL_dmeans2D[3 * (size_t)g + 0], aG * (RABS(gdx * co[0]) + RABS(gdy * co[1])) * ddelx_dx);
                        ATOMIC_ADD(dL_dmeans2D[3 * (size_t)g + 1], aG * (RABS(gdy * co[2]) + RABS(gdx * co[1])) * ddely_dy);
                    } else {
                        ATOMIC_ADD(dL_dmeans2D[3 * (size_t)g + 0], dL_dG * dG_ddelx * ddelx_dx);
                        ATOMIC_ADD(dL_dmeans2D[3 * (size_t)g + 1], dL_dG * dG_ddely * ddely_dy);
                    }
                    ATOMIC_ADD(dL_dconic[3 * (size_t)g + 0], R(-0.5) * gdx * dx * dL_dG);
                    ATOMIC_ADD(dL_dconic[3 * (size_t)g + 1], R(-0.5) * gdx * dy * dL_dG);
                    ATOMIC_ADD(dL_dconic[3 * (size_t)g + 2], R(-0.5) * gdy * dy * dL_dG);
                    ATOMIC_ADD(dL_dopacity[g], g_abs_terms ? G * dLa_abs : G * dL_dalpha);
                }
            }
        free(accF);
    }

    /* preprocess backward, one Gaussian at a time */
    const real fx = (real)W / (R(2.0) * s->tanfovx), fy = (real)H / (R(2.0) * s->tanfovy);
#pragma omp parallel for schedule(static)
    for (int i = 0; i < P; ++i) {
        real *dm = dL_dmeans3D + 3 * (size_t)i;
        dm[0] = dm[1] = dm[2] = 0;
        real *dcov = dL_dcov3D + 6 * (size_t)i;
        for (int k = 0; k < 6; ++k) dcov[k] = 0;
        if (dL_dsh && M > 0) memset(dL_dsh + (size_t)i * M * 3, 0, sizeof(real) * (size_t)M * 3);
        if (dL_dscales) dL_dscales[3 * (size_t)i] = dL_dscales[3 * (size_t)i + 1] = dL_dscales[3 * (size_t)i + 2] = 0;
        if (dL_drots) for (int k = 0; k < 4; ++k) dL_drots[4 * (size_t)i + k] = 0;
        if (!(st->radii[i] > 0)) continue;
        const real *p = means3D + 3 * (size_t)i;
        real cov3[6];
        const real *c3;
        if (cov3D_precomp) c3 = cov3D_precomp + 6 * (size_t)i;
        else { compute_cov3d(scales + 3 * (size_t)i, s->scale_modifier, rotations + 4 * (size_t)i, cov3); c3 = cov3; }
        /* computeCov2DCUDA: conic -> cov2D -> (cov3D, mean) */
        cov2d_backward(p, c3, fx, fy, s->tanfovx, s->tanfovy, s->view, dL_dconic + 3 * (size_t)i, dm, dcov);
        /* projection of the mean: dL/dmean2D (NDC) -> dL/dmean3D */
        const real *pm = s->proj;
        real mh[4];
        xform4x4(pm, p, mh);
        const real mw = R(1.0) / (mh[3] + R(0.0000001));
        const real mul1 = (pm[0] * p[0] + pm[4] * p[1] + pm[8] * p[2] + pm[12]) * mw * mw;
        const real mul2 = (pm[1] * p[0] + pm[5] * p[1] + pm[9] * p[2] + pm[13]) * mw * mw;
        const real g2x = dL_dmeans2D[3 * (size_t)i], g2y = dL_dmeans2D[3 * (size_t)i + 1];
        dm[0] += (pm[0] * mw - pm[3] * mul1) * g2x + (pm[1] * mw - pm[3] * mul2) * g2y;
        dm[1] += (pm[4] * mw - pm[7] * mul1) * g2x + (pm[5] * mw - pm[7] * mul2) * g2y;
        dm[2] += (pm[8] * mw - pm[11] * mul1) * g2x + (pm[9] * mw - pm[11] * mul2) * g2y;
        /* depth = view row 2 . [p,1] */
        dm[0] += s->view[2] * dL_ddepth[i];
        dm[1] += s->view[6] * dL_ddepth[i];
        dm[2] += s->view[10] * dL_ddepth[i];
        if (shs)
            sh_backward(s->sh_degree, M, p, s->campos, shs + (size_t)i * M * 3, st->clamped + 3 * (size_t)i,
                        dL_dcolors + 3 * (size_t)i, dL_dsh + (size_t)i * M * 3, dm);
        if (!cov3D_precomp)
            cov3d_backward(scales + 3 * (size_t)i, s->scale_modifier, rotations + 4 * (size_t)i, dcov,
                           dL_dscales + 3 * (size_t)i, dL_drots + 4 * (size_t)i);
    }
    (void)colors_precomp;
    free(dL_dconic);
    free(dL_ddepth);
}

/* mark_visible: z_view > 0.2 */
void orc_mark_visible(int P, const real *means3D, const real *view, uint8_t *present) {
    for (int i = 0; i < P; ++i) {
        real pv[3];
        xform4x3(view, means3D + 3 * (size_t)i, pv);
        present[i] = pv[2] > R(0.2);
    }
}

/* ---- accessors for the Python test wrapper -------------------------------------------------- */
int64_t orc_num_rendered(const orc_state *st) { return st->num_rendered; }
void orc_copy_state(const orc_state *st, real *xy, real *depth, real *conic_o, real *rgb, uint8_t *clamped,
                    uint32_t *tiles, uint32_t *point_list, uint32_t *ranges, real *final_T, uint32_t *n_contrib) {
    const size_t P = (size_t)st->P, HW = (size_t)st->H * st->W, NT = (size_t)st->tiles_x * st->tiles_y;
    if (xy) memcpy(xy, st->xy, sizeof(real) * 2 * P);
    if (depth) memcpy(depth, st->depth, sizeof(real) * P);
    if (conic_o) memcpy(conic_o, st->conic_o, sizeof(real) * 4 * P);
    if (rgb) memcpy(rgb, st->rgb, sizeof(real) * 3 * P);
    if (clamped) memcpy(clamped, st->clamped, 3 * P);
    if (tiles) memcpy(tiles, st->tiles, sizeof(uint32_t) * P);
    if (point_list) memcpy(point_list, st->point_list, sizeof(uint32_t) * (size_t)st->num_rendered);
    if (ranges) memcpy(ranges, st->ranges, sizeof(uint32_t) * 2 * NT);
    if (final_T) memcpy(final_T, st->final_T, sizeof(real) * HW);
    if (n_contrib) memcpy(n_contrib, st->n_contrib, sizeof(uint32_t) * HW);
}
void orc_free(orc_state *st) {
    if (!st) return;
    free(st->xy); free(st->depth); free(st->conic_o); free(st->rgb); free(st->clamped); free(st->radii);
    free(st->tiles); free(st->point_list); free(st->tile_of); free(st->ranges); free(st->final_T);
    free(st->n_contrib); free(st);
}
int orc_real_size(void) { return (int)sizeof(real); }
/* SH helper exposed for the golden-vector test (colour of one Gaussian, before nothing else). */
void orc_sh_colors(int N, int deg, int M, const real *pos, const real *campos, const real *sh, real *rgb, uint8_t *clamped) {
    for (int i = 0; i < N; ++i) color_from_sh(deg, M, pos + 3 * (size_t)i, campos, sh + (size_t)i * M * 3, rgb + 3 * (size_t)i, clamped + 3 * (size_t)i);
}
void orc_cov3d(int N, const real *scales, real mod, const real *rots, real *cov) {
    for (int i = 0; i < N; ++i) compute_cov3d(scales + 3 * (size_t)i, mod, rots + 4 * (size_t)i, cov + 6 * (size_t)i);
}
