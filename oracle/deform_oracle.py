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
  Deformation.query_time / create_net (feature_out = one Linear at defor_depth 0)
                                      scene/deformation.py:45-86
  Deformation.forward_dynamic (residual heads; language pass-through, no_dlang)  :103-182
  deform_network.forward_dynamic      :232-248 (the poc_fre embeddings only feed the unused
                                      time / language paths; rays_pts_emb[:, :3] == means3D)
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


class DeformOracle:
    """params: dict name -> array, names as in the reference Deformation module
    (grid.grids.{s}.{ci}, feature_out.0.weight / .bias, {head}.1 / .3 weight / bias)."""

    def __init__(self, params, aabb, n_scales=2):
        self.p = {k: np.asarray(v, dtype=np.float64) for k, v in params.items()}
        self.aabb = np.asarray(aabb, dtype=np.float64)
        self.n_scales = n_scales

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

    def forward(self, means3D, scales, rotations, opacity, shs, lang, time):
        feat, taps = self.features(means3D, time)
        h = feat @ self.p["feature_out.0.weight"].T + self.p["feature_out.0.bias"]
        a = _relu(h)
        outs, cache = {}, {}
        for name, n in HEADS:
            z = a @ self.p[name + ".1.weight"].T + self.p[name + ".1.bias"]
            a2 = _relu(z)
            outs[name] = a2 @ self.p[name + ".3.weight"].T + self.p[name + ".3.bias"]
            cache[name] = (z, a2)
        self._cache = (feat, taps, h, a, cache, means3D.shape[0])
        return dict(means3D=means3D + outs["pos_deform"], scales=scales + outs["scales_deform"],
                    rotations=rotations + outs["rotations_deform"], opacity=opacity + outs["opacity_deform"],
                    shs=shs + outs["shs_deform"].reshape(-1, 16, 3), lang=lang)

    def backward(self, up_means3D, up_scales, up_rotations, up_opacity, up_shs):
        """Gradients of sum(out * up) w.r.t. inputs and parameters (after forward)."""
        feat, taps, h, a, cache, P = self._cache
        g = {}
        ups = dict(pos_deform=up_means3D, scales_deform=up_scales, rotations_deform=up_rotations,
                   opacity_deform=up_opacity, shs_deform=up_shs.reshape(P, 48))
        da = np.zeros_like(a)
        for name, n in HEADS:
            z, a2 = cache[name]
            u = ups[name]
            g[name + ".3.weight"] = u.T @ a2
            g[name + ".3.bias"] = u.sum(0)
            dz = (u @ self.p[name + ".3.weight"]) * (z > 0)
            g[name + ".1.weight"] = dz.T @ a
            g[name + ".1.bias"] = dz.sum(0)
            da += dz @ self.p[name + ".1.weight"]
        dh = da * (h > 0)
        g["feature_out.0.weight"] = dh.T @ feat
        g["feature_out.0.bias"] = dh.sum(0)
        dfeat = dh @ self.p["feature_out.0.weight"]
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
                x0, x1, y0, y1, fx, fy, v00, v01, v10, v11, x, y, W, H = tp[ci]
                key = plane_key(s, ci)
                gp = g.setdefault(key, np.zeros_like(self.p[key]))[0]
                for (yy, xx, w) in ((y0, x0, (1 - fx) * (1 - fy)), (y0, x1, fx * (1 - fy)),
                                    (y1, x0, (1 - fx) * fy), (y1, x1, fx * fy)):
                    np.add.at(gp, (slice(None), yy, xx), (dv * w[:, None]).T)
                dix = (dv * ((v01 - v00) * (1 - fy)[:, None] + (v11 - v10) * fy[:, None])).sum(1)
                diy = (dv * ((v10 - v00) * (1 - fx)[:, None] + (v11 - v01) * fx[:, None])).sum(1)
                # border padding: no gradient through a clipped coordinate (clip at <= 0, >= size-1)
                rx, ry = (x + 1.0) * 0.5 * (W - 1), (y + 1.0) * 0.5 * (H - 1)
                dq[:, c0] += dix * 0.5 * (W - 1) * ((rx > 0) & (rx < W - 1))
                dq[:, c1] += diy * 0.5 * (H - 1) * ((ry > 0) & (ry < H - 1))
        a0, a1 = self.aabb[0], self.aabb[1]
        g_in = dict(means3D=up_means3D + dq[:, :3] * (2.0 / (a1 - a0)), scales=up_scales.copy(),
                    rotations=up_rotations.copy(), opacity=up_opacity.copy(), shs=up_shs.copy())
        return g_in, g
