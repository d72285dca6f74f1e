"""CPU restatement of the 4D-LangSplat deformation network forward and backward (numpy, float64).

TEST INFRASTRUCTURE ONLY: imported by tests/ as the checker of the HIP deformation kernels
(4dlangsplat_amd/csrc/deform.hip); never part of the product path.

Parity: pinned on the reference module itself.  tests/golden/deform_golden.npz holds inputs,
parameters, outputs and autograd gradients of the reference `deform_network` (generated in the
build container by tests/golden/make_deform_golden.py), and tests/test_deform_oracle.py checks this
restatement against them.

Follows (reference file:line):
  normalize_aabb                      scene/hexplane.py:19-20
  grid_sample_wrapper (bilinear, align_corners=True, padding_mode='border')   :21-46
  interpolate_ms_features (product over the 6 planes, concat over scales)     :73-106
  HexPlaneField.get_density (pts ++ t, plane list per scale)                  :160-177
  Deformation.query_time / create_net (feature_out: max(defor_depth, 1) Linear layers with ReLU
                                      between them)  scene/deformation.py:45-86
  Deformation.forward_dynamic         :103-182 -- residual heads (each can be off: no_dx / no_ds /
                                      no_dr / no_do / no_dshs), apply_rotation (quaternion product and
                                      normalisation, utils/graphics_utils.py:109-132), and the language
                                      modes: pass-through (no_dlang), lang_deform over
                                      [lang ++ poc_fre(t)] with residual (or not: no_resnet) and
                                      re-normalisation (:164-180), or the discrete centres with the
                                      discrete_coff_generator head (use_discrete_lang_f, :156-163)
  deform_network.forward_dynamic      :232-248, poc_fre :261-267 (rays_pts_emb[:, :3] == means3D;
                                      only the time embedding feeds a computed path: lang_deform)
Layouts: plane of combo (c0, c1) is [C, res[c1], res[c0]] (x along res[c0]); Linear weights are
[out, in] as torch.
"""
import itertools

import numpy as np

HEADS = (("pos_deform", 3), ("scales_deform", 3), ("rotations_deform", 4), ("opacity_deform", 1),
         ("shs_deform", 48))
COMBOS = list(itertools.combinations(range(4), 2))   # xy, xz, xt, yz, yt, zt


def plane_key(scale, ci):
    return f"grid.grids.{scale}.{ci}"


def _sample(plane, x, y):
    """Bilinear sample of plane [C, H, W] at normalised coords x, y in [-1, 1] (align_corners,
    border).  Returns values [P, C] and the tap description for the backward."""
    C, H, W = plane.shape
    ix = np.clip((x + 1.0) * 0.5 * (W - 1), 0.0, W - 1)
    iy = np.clip((y + 1.0) * 0.5 * (H - 1), 0.0, H - 1)
    x0 = np.floor(ix).astype(np.int64)
    y0 = np.floor(iy).astype(np.int64)
    fx, fy = ix - x0, iy - y0
    x1, y1 = np.minimum(x0 + 1, W - 1), np.minimum(y0 + 1, H - 1)   # weight 0 whenever clamped
    v00, v01 = plane[:, y0, x0].T, plane[:, y0, x1].T
    v10, v11 = plane[:, y1, x0].T, plane[:, y1, x1].T
    val = (v00 * ((1 - fx) * (1 - fy))[:, None] + v01 * (fx * (1 - fy))[:, None]
           + v10 * ((1 - fx) * fy)[:, None] + v11 * (fx * fy)[:, None])
    return val, (x0, x1, y0, y1, fx, fy, v00, v01, v10, v11, x, y, W, H)


def _relu(x):
    return np.maximum(x, 0.0)


HEAD_NAMES = ("pos_deform", "scales_deform", "rotations_deform", "opacity_deform", "shs_deform")


class DeformConfig:
    """The switches of scene/deformation.py that change the computation (ModelHiddenParams plus the
    env vars the reference reads).  lang_mode: "pass" (no_dlang), "residual" (lang_deform),
    "noresnet" (lang_deform, env no_resnet=t) or "discrete" (env use_discrete_lang_f=t)."""

    def __init__(self, n_scales=2, depth=0, heads=(True, True, True, True, True), apply_rotation=False,
                 lang_mode="pass", lang_dim=3, centers=0, time_pe=4):
        self.n_scales, self.depth, self.heads = n_scales, depth, tuple(bool(h) for h in heads)
        self.apply_rotation, self.lang_mode, self.lang_dim = apply_rotation, lang_mode, lang_dim
        self.centers, self.time_pe = centers, time_pe

    @classmethod
    def from_golden(cls, cfg):
        """From the config dict of tests/golden/deform_variants.npz."""
        mode = "pass" if cfg["no_dlang"] else ("discrete" if cfg["discrete"] else
                                               ("noresnet" if cfg["no_resnet"] else "residual"))
        return cls(len(cfg["multires"]), cfg["depth"], tuple(not cfg[k] for k in ("no_dx", "no_ds", "no_dr", "no_do",
                                                                                   "no_dshs")),
                   cfg["apply_rotation"], mode, cfg["lang_dim"], cfg["centers"], cfg["time_pe"])


def poc_fre(x, n):
    """[x, sin(x 2^i), cos(x 2^i)] for i < n, as deformation.py:261-267 (x: [P, k])."""
    e = (x[:, :, None] * (2.0 ** np.arange(n))[None, None, :]).reshape(x.shape[0], -1)
    return np.concatenate([x, np.sin(e), np.cos(e)], axis=1)


def quat_mul(q1, q2):
    """batch_quaternion_multiply before its normalisation (utils/graphics_utils.py:121-124)."""
    w = q1[:, 0] * q2[:, 0] - q1[:, 1] * q2[:, 1] - q1[:, 2] * q2[:, 2] - q1[:, 3] * q2[:, 3]
    x = q1[:, 0] * q2[:, 1] + q1[:, 1] * q2[:, 0] + q1[:, 2] * q2[:, 3] - q1[:, 3] * q2[:, 2]
    y = q1[:, 0] * q2[:, 2] - q1[:, 1] * q2[:, 3] + q1[:, 2] * q2[:, 0] + q1[:, 3] * q2[:, 1]
    z = q1[:, 0] * q2[:, 3] + q1[:, 1] * q2[:, 2] - q1[:, 2] * q2[:, 1] + q1[:, 3] * q2[:, 0]
    return np.stack([w, x, y, z], axis=1)


def quat_mul_bwd(q1, q2, d):
    """Gradients of sum(quat_mul(q1, q2) * d) w.r.t. q1 and q2."""
    e = np.eye(4)
    d1 = np.stack([(quat_mul(np.broadcast_to(e[k], q1.shape), q2) * d).sum(1) for k in range(4)], axis=1)
    d2 = np.stack([(quat_mul(q1, np.broadcast_to(e[k], q2.shape)) * d).sum(1) for k in range(4)], axis=1)
    return d1, d2


def normalize_bwd(v, d, eps):
    """Gradient of sum(v / (|v| + eps) * d) w.r.t. v (rows)."""
    n = np.linalg.norm(v, axis=1, keepdims=True)
    return d / (n + eps) - v * ((v * d).sum(1, keepdims=True) / (n * (n + eps) ** 2))


class DeformOracle:
    """params: dict name -> array, names as in the reference Deformation module
    (grid.grids.{s}.{ci}, feature_out.{2k}.weight / .bias, {head}.1 / .3 weight / bias,
    discrete_coff_generator.1 / .3, lang_deform.1 / .3 / .5).  cfg: DeformConfig (default: the
    Neu3D structure, arguments/neu3d/default.py)."""

    def __init__(self, params, aabb, n_scales=2, cfg=None):
        self.p = {k: np.asarray(v, dtype=np.float64) for k, v in params.items()}
        self.aabb = np.asarray(aabb, dtype=np.float64)
        self.cfg = cfg or DeformConfig(n_scales=n_scales)
        self.n_scales = self.cfg.n_scales

    def features(self, means3D, time):
        a0, a1 = self.aabb[0], self.aabb[1]
        pn = (means3D - a0) * (2.0 / (a1 - a0)) - 1.0
        q = np.concatenate([pn, time.reshape(-1, 1)], axis=1)
        feats, taps = [], []
        for s in range(self.n_scales):
            prod = None
            vals, tp = [], []
            for ci, (c0, c1) in enumerate(COMBOS):
                plane = self.p[plane_key(s, ci)][0]
                v, t = _sample(plane, q[:, c0], q[:, c1])
                vals.append(v)
                tp.append(t)
                prod = v if prod is None else prod * v
            feats.append(prod)
            taps.append((vals, tp))
        return np.concatenate(feats, axis=1), taps

    def _lin(self, name, x):
        return x @ self.p[name + ".weight"].T + self.p[name + ".bias"]

    def _heads(self):
        c = self.cfg
        hs = [(n, w) for (n, w), on in zip(HEADS, c.heads) if on]
        if c.lang_mode == "discrete":
            hs.append(("discrete_coff_generator", c.centers))
        return hs

    def forward(self, means3D, scales, rotations, opacity, shs, lang, time):
        c = self.cfg
        P = means3D.shape[0]
        feat, taps = self.features(means3D, time)
        pre, acts = [], [feat]
        for k in range(max(c.depth, 1)):        # feature_out.{2k}, ReLU before the next layer / the heads
            pre.append(self._lin(f"feature_out.{2 * k}", acts[-1]))
            acts.append(_relu(pre[-1]))
        a = acts[-1]
        outs, cache = {}, {}
        for name, n in self._heads():
            z = self._lin(name + ".1", a)
            a2 = _relu(z)
            outs[name] = self._lin(name + ".3", a2)
            cache[name] = (z, a2)
        res = dict(means3D=means3D + outs["pos_deform"] if c.heads[0] else means3D.copy(),
                   scales=scales + outs["scales_deform"] if c.heads[1] else scales.copy(),
                   opacity=opacity + outs["opacity_deform"] if c.heads[3] else opacity.copy(),
                   shs=shs + outs["shs_deform"].reshape(-1, 16, 3) if c.heads[4] else shs.copy(), coff=None)
        rq = None
        if not c.heads[2]:
            res["rotations"] = rotations.copy()
        elif c.apply_rotation:
            rq = quat_mul(rotations, outs["rotations_deform"])
            res["rotations"] = rq / np.linalg.norm(rq, axis=1, keepdims=True)
        else:
            res["rotations"] = rotations + outs["rotations_deform"]
        lc = None
        if c.lang_mode == "pass":
            res["lang"] = None if lang is None else lang[:, :c.lang_dim].copy()
        elif c.lang_mode == "discrete":
            e = lang[:, :c.lang_dim * c.centers].reshape(P, c.centers, c.lang_dim)
            en = np.linalg.norm(e, axis=2, keepdims=True)
            u = e / en
            coff = outs["discrete_coff_generator"]
            m = (coff[:, :, None] * u).sum(1)
            res["lang"] = m / (np.linalg.norm(m, axis=1, keepdims=True) + 1e-9)
            res["coff"] = coff
            lc = (e, en, u, coff, m)
        else:
            x0 = np.concatenate([lang, poc_fre(time.reshape(-1, 1), c.time_pe)], axis=1)
            u0 = _relu(x0)
            z1 = self._lin("lang_deform.1", u0)
            u1 = _relu(z1)
            z2 = self._lin("lang_deform.3", u1)
            u2 = _relu(z2)
            dl = self._lin("lang_deform.5", u2)
            v = dl if c.lang_mode == "noresnet" else lang[:, :c.lang_dim] + dl
            res["lang"] = v / (np.linalg.norm(v, axis=1, keepdims=True) + 1e-9)
            lc = (x0, u0, z1, u1, z2, u2, v)
        self._cache = (feat, taps, pre[-1], a, cache, P)
        self._full = dict(pre=pre, acts=acts, rq=rq, rotations=rotations, outs=outs, lc=lc, lang=lang)
        return res

    def preactivations(self):
        """Every ReLU input of the last forward (for tests that avoid ReLU kinks)."""
        f = self._full
        zs = list(f["pre"]) + [z for z, _ in self._cache[4].values()]
        if self.cfg.lang_mode in ("residual", "noresnet"):
            lc = f["lc"]
            zs += [lc[0], lc[2], lc[4]]
        return zs

    def backward(self, up_means3D, up_scales, up_rotations, up_opacity, up_shs, up_lang=None, up_coff=None):
        """Gradients of sum(out * up) w.r.t. inputs and parameters (after forward)."""
        c = self.cfg
        feat, taps, h, a, cache, P = self._cache
        f = self._full
        g = {}
        g_in = dict(means3D=up_means3D.copy(), scales=up_scales.copy(), rotations=up_rotations.copy(),
                    opacity=up_opacity.copy(), shs=up_shs.copy())
        lang = f["lang"]
        if lang is None:   # pass-through with no language rows: nothing to differentiate
            lang = np.zeros((P, c.lang_dim))
        dlang_in = np.zeros_like(lang)
        ups = dict(pos_deform=up_means3D, scales_deform=up_scales, rotations_deform=up_rotations,
                   opacity_deform=up_opacity, shs_deform=up_shs.reshape(P, 48))
        if c.heads[2] and c.apply_rotation:
            dq = normalize_bwd(f["rq"], up_rotations, 0.0)
            g_in["rotations"], ups["rotations_deform"] = quat_mul_bwd(f["rotations"], f["outs"]["rotations_deform"], dq)
        up_lang = np.zeros((P, c.lang_dim)) if up_lang is None else up_lang
        if c.lang_mode == "pass":
            dlang_in[:, :c.lang_dim] += up_lang
        elif c.lang_mode == "discrete":
            e, en, u, coff, m = f["lc"]
            dm = normalize_bwd(m, up_lang, 1e-9)
            dcoff = (u * dm[:, None, :]).sum(2) + (0.0 if up_coff is None else up_coff)
            du = coff[:, :, None] * dm[:, None, :]
            de = (du - u * (u * du).sum(2, keepdims=True)) / en
            dlang_in[:, :c.lang_dim * c.centers] += de.reshape(P, -1)
            ups["discrete_coff_generator"] = dcoff
        else:
            x0, u0, z1, u1, z2, u2, v = f["lc"]
            dv = normalize_bwd(v, up_lang, 1e-9)
            if c.lang_mode == "residual":
                dlang_in[:, :c.lang_dim] += dv
            g["lang_deform.5.weight"] = dv.T @ u2
            g["lang_deform.5.bias"] = dv.sum(0)
            dz2 = (dv @ self.p["lang_deform.5.weight"]) * (z2 > 0)
            g["lang_deform.3.weight"] = dz2.T @ u1
            g["lang_deform.3.bias"] = dz2.sum(0)
            dz1 = (dz2 @ self.p["lang_deform.3.weight"]) * (z1 > 0)
            g["lang_deform.1.weight"] = dz1.T @ u0
            g["lang_deform.1.bias"] = dz1.sum(0)
            dx0 = (dz1 @ self.p["lang_deform.1.weight"]) * (x0 > 0)
            dlang_in += dx0[:, :lang.shape[1]]
        g_in["lang"] = dlang_in
        da = np.zeros_like(a)
        for name, n in self._heads():
            z, a2 = cache[name]
            u_ = ups[name]
            g[name + ".3.weight"] = u_.T @ a2
            g[name + ".3.bias"] = u_.sum(0)
            dz = (u_ @ self.p[name + ".3.weight"]) * (z > 0)
            g[name + ".1.weight"] = dz.T @ a
            g[name + ".1.bias"] = dz.sum(0)
            da += dz @ self.p[name + ".1.weight"]
        pre, acts = f["pre"], f["acts"]
        for k in reversed(range(len(pre))):
            dh = da * (pre[k] > 0)
            g[f"feature_out.{2 * k}.weight"] = dh.T @ acts[k]
            g[f"feature_out.{2 * k}.bias"] = dh.sum(0)
            da = dh @ self.p[f"feature_out.{2 * k}.weight"]
        dfeat = da
        dq = np.zeros((P, 4))
        nc = feat.shape[1] // self.n_scales
        for s in range(self.n_scales):
            vals, tp = taps[s]
            df = dfeat[:, s * nc:(s + 1) * nc]
            for ci, (c0, c1) in enumerate(COMBOS):
                others = np.ones_like(df)
                for cj in range(len(COMBOS)):
                    if cj != ci:
                        others = others * vals[cj]
                dv = df * others                                       # [P, C]
                x0_, x1_, y0_, y1_, fx, fy, v00, v01, v10, v11, x, y, W, H = tp[ci]
                key = plane_key(s, ci)
                gp = g.setdefault(key, np.zeros_like(self.p[key]))[0]
                for (yy, xx, w) in ((y0_, x0_, (1 - fx) * (1 - fy)), (y0_, x1_, fx * (1 - fy)),
                                    (y1_, x0_, (1 - fx) * fy), (y1_, x1_, fx * fy)):
                    np.add.at(gp, (slice(None), yy, xx), (dv * w[:, None]).T)
                dix = (dv * ((v01 - v00) * (1 - fy)[:, None] + (v11 - v10) * fy[:, None])).sum(1)
                diy = (dv * ((v10 - v00) * (1 - fx)[:, None] + (v11 - v01) * fx[:, None])).sum(1)
                # border padding: no gradient through a clipped coordinate (clip at <= 0, >= size-1)
                rx, ry = (x + 1.0) * 0.5 * (W - 1), (y + 1.0) * 0.5 * (H - 1)
                dq[:, c0] += dix * 0.5 * (W - 1) * ((rx > 0) & (rx < W - 1))
                dq[:, c1] += diy * 0.5 * (H - 1) * ((ry > 0) & (ry < H - 1))
        a0, a1 = self.aabb[0], self.aabb[1]
        g_in["means3D"] = g_in["means3D"] + dq[:, :3] * (2.0 / (a1 - a0))
        return g_in, g
