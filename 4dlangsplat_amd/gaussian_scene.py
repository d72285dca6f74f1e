"""Gaussian scene I/O and the per-view render() of the reference, on the MI355X rasterizer.

SURVEY.md 8(f) row 2 (and 8(a) row a1).  Restates, from the reference:
  * the parameter layout and activations of GaussianModel   scene/gaussian_model.py:31-46,168-172
  * its PLY format (attribute list, order, float32 vertex element)
                                                             scene/gaussian_model.py:331-345,370-389,396-444
  * render(): settings, stage logic, deformation, activations, rasterizer call, output dict
                                                             gaussian_renderer/__init__.py:19-248
  * render.py's per-frame loop: FPS print, renders_npy/{idx:05d}.npy as [H, W, C], PCA of
    language maps with C > 3 for the PNGs                    render.py:52-65,67-161
The reference reads and writes PLY with `plyfile` (not installed here); this module parses and
writes the same binary_little_endian vertex element itself (numpy structured arrays).  The
rasterizer is diff_gaussian_rasterization (liblsr.so) and the deformation the HIP
DeformationField (deformation.py): no CPU fallback.
"""
from __future__ import annotations

import math
import os
import time as _time
import zlib
import struct
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

_PLY_TYPES = {"float": "f4", "float32": "f4", "double": "f8", "float64": "f8", "uchar": "u1", "uint8": "u1",
              "char": "i1", "int8": "i1", "ushort": "u2", "uint16": "u2", "short": "i2", "int16": "i2",
              "uint": "u4", "uint32": "u4", "int": "i4", "int32": "i4"}


@dataclass
class GaussianScene:
    """Raw (pre-activation) Gaussian parameters, the reference's GaussianModel tensors
    (_xyz, _features_dc, _features_rest, _language_feature, _opacity, _scaling, _rotation)."""
    xyz: torch.Tensor                 # [P, 3]
    features_dc: torch.Tensor         # [P, 1, 3]
    features_rest: torch.Tensor       # [P, (deg+1)^2 - 1, 3]
    language_feature: torch.Tensor    # [P, C]
    opacity: torch.Tensor             # [P, 1] logit
    scaling: torch.Tensor             # [P, 3] log scale
    rotation: torch.Tensor            # [P, 4] unnormalised quaternion (r, x, y, z)
    max_sh_degree: int = 3
    active_sh_degree: int = 3
    deformation: Optional[object] = None   # deformation.DeformationField for the 'fine' stages
    extra: Dict[str, np.ndarray] = field(default_factory=dict)

    @property
    def P(self) -> int:
        return self.xyz.shape[0]

    # activations: gaussian_model.py:38-46 (exp, normalize, sigmoid)
    @property
    def get_xyz(self):
        return self.xyz

    @property
    def get_features(self):
        return torch.cat((self.features_dc, self.features_rest), dim=1)

    @property
    def get_scaling(self):
        return torch.exp(self.scaling)

    @property
    def get_rotation(self):
        return torch.nn.functional.normalize(self.rotation)

    @property
    def get_opacity(self):
        return torch.sigmoid(self.opacity)

    @property
    def get_language_feature(self):
        return self.language_feature

    def to(self, device):
        t = lambda x: x.to(device)   # noqa: E731
        return GaussianScene(t(self.xyz), t(self.features_dc), t(self.features_rest), t(self.language_feature),
                             t(self.opacity), t(self.scaling), t(self.rotation), self.max_sh_degree,
                             self.active_sh_degree, self.deformation,
                             {k: (v.to(device) if torch.is_tensor(v) else v) for k, v in self.extra.items()})

    # ---- PLY (gaussian_model.py:331-345 attribute list, :370-389 save, :396-444 load) ---------
    def attribute_names(self) -> List[str]:
        names = ["x", "y", "z", "nx", "ny", "nz"]
        names += [f"f_dc_{i}" for i in range(self.features_dc.shape[1] * self.features_dc.shape[2])]
        names += [f"f_rest_{i}" for i in range(self.features_rest.shape[1] * self.features_rest.shape[2])]
        names += [f"f_lang_{i}" for i in range(self.language_feature.shape[1])]
        names += ["opacity"]
        names += [f"scale_{i}" for i in range(self.scaling.shape[1])]
        names += [f"rot_{i}" for i in range(self.rotation.shape[1])]
        return names

    def save_ply(self, path: str) -> None:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
        c = lambda x: x.detach().float().cpu().numpy()   # noqa: E731
        xyz = c(self.xyz)
        # features are stored channel-major: transpose(1, 2).flatten (gaussian_model.py:375-376)
        f_dc = c(self.features_dc.transpose(1, 2).flatten(start_dim=1))
        f_rest = c(self.features_rest.transpose(1, 2).flatten(start_dim=1))
        cols = np.concatenate([xyz, np.zeros_like(xyz), f_dc, f_rest, c(self.language_feature), c(self.opacity),
                               c(self.scaling), c(self.rotation)], axis=1).astype(np.float32)
        write_ply_vertices(path, self.attribute_names(), cols)

    @classmethod
    def load_ply(cls, path: str, max_sh_degree: int = 3, device="cpu") -> "GaussianScene":
        v = read_ply_vertices(path)
        P = len(v["x"])
        col = lambda n: np.asarray(v[n], dtype=np.float32)   # noqa: E731

        def group(prefix):
            names = sorted((n for n in v if n.startswith(prefix)), key=lambda n: int(n.split("_")[-1]))
            return np.stack([col(n) for n in names], axis=1) if names else np.zeros((P, 0), np.float32)

        xyz = np.stack([col("x"), col("y"), col("z")], axis=1)
        f_dc = np.stack([col("f_dc_0"), col("f_dc_1"), col("f_dc_2")], axis=1)[:, :, None]      # [P, 3, 1]
        rest = group("f_rest_")
        n_rest = 3 * (max_sh_degree + 1) ** 2 - 3
        if rest.shape[1] != n_rest:
            raise ValueError(f"{path}: {rest.shape[1]} f_rest_* attributes, expected {n_rest} for SH degree "
                             f"{max_sh_degree}")
        rest = rest.reshape(P, 3, (max_sh_degree + 1) ** 2 - 1)
        t = lambda a: torch.tensor(a, dtype=torch.float32, device=device)   # noqa: E731
        return cls(xyz=t(xyz), features_dc=t(f_dc).transpose(1, 2).contiguous(),
                   features_rest=t(rest).transpose(1, 2).contiguous(), language_feature=t(group("f_lang_")),
                   opacity=t(col("opacity"))[:, None], scaling=t(group("scale_")), rotation=t(group("rot")),
                   max_sh_degree=max_sh_degree, active_sh_degree=max_sh_degree)


# ---- trained model directories (scene/__init__.py:35-37,85-101; gaussian_model.py:352-370) -------
def search_for_max_iteration(folder: str, stage: str) -> int:
    """utils/system_utils.py:26-28: the largest N of the `{stage}_iteration_N` entries in folder."""
    iters = [int(f.split("_")[-1]) for f in os.listdir(folder) if f.split("_")[0] == stage]
    if not iters:
        raise FileNotFoundError(f"no {stage}_iteration_* in {folder}")
    return max(iters)


def _load_pth(path: str, device):
    """torch.load of a tensor file the reference wrote, without unpickling code (weights_only)."""
    return torch.load(path, map_location=device, weights_only=True)


def read_model_dir(model_path: str, load_iteration: int = -1, load_stage: str = "fine-lang", max_sh_degree: int = 3,
                   device="cpu"):
    """What Scene(load_iteration=...) reads (scene/__init__.py:35-37,85-93; gaussian_model.py:352-364):
    model_path/point_cloud/{load_stage}_iteration_{N}/point_cloud.ply (N = the largest if -1),
    deformation.pth (the deform_network state dict), deformation_table.pth (default all True) and
    deformation_accum.pth (default zeros [P, 3]).  Returns (scene, deformation state dict, iteration);
    the scene's `extra` holds the table and accumulator.  CPU; build the field with load_model_dir."""
    root = os.path.join(model_path, "point_cloud")
    it = search_for_max_iteration(root, load_stage) if load_iteration == -1 else int(load_iteration)
    d = os.path.join(root, f"{load_stage}_iteration_{it}")
    scene = GaussianScene.load_ply(os.path.join(d, "point_cloud.ply"), max_sh_degree=max_sh_degree, device=device)
    state = _load_pth(os.path.join(d, "deformation.pth"), device)
    P = scene.P
    table = os.path.join(d, "deformation_table.pth")
    accum = os.path.join(d, "deformation_accum.pth")
    scene.extra["deformation_table"] = _load_pth(table, device) if os.path.exists(table) else \
        torch.ones(P, dtype=torch.bool, device=device)
    scene.extra["deformation_accum"] = _load_pth(accum, device) if os.path.exists(accum) else \
        torch.zeros(P, 3, device=device)
    return scene, state, it


DEFORM_CONFIG = "deformation_config.json"   # this build's sidecar next to deformation.pth


def load_model_dir(model_path: str, hidden=None, env=None, load_iteration: int = -1, load_stage: str = "fine-lang",
                   max_sh_degree: int = 3, device="cuda"):
    """read_model_dir + the deformation field on the GPU (DeformationField.from_reference with the
    ModelHiddenParams and env the model was trained with).  Returns (scene, iteration).

    The reference keeps the language mode in environment variables (no_dlang aside), which a
    deformation.pth does not record: a model directory written by save_model_dir carries them in
    `deformation_config.json` ({"hidden": ..., "env": ...}), which fills `hidden` / `env` when they are
    None, and an explicit `env` whose language mode contradicts it raises.  Without the sidecar (a
    directory the reference wrote) `hidden` is required and `env` defaults to os.environ."""
    import json

    from deformation import DeformationField
    scene, state, it = read_model_dir(model_path, load_iteration, load_stage, max_sh_degree, device="cpu")
    side = os.path.join(model_path, "point_cloud", f"{load_stage}_iteration_{it}", DEFORM_CONFIG)
    if os.path.exists(side):
        with open(side) as f:
            rec = json.load(f)
        if hidden is None:
            hidden = rec["hidden"]
        if env is None:
            env = rec["env"]
        else:
            for k, v in rec["env"].items():
                default = {"use_discrete_lang_f": "f", "no_resnet": "f", "language_feature_hiddendim": "3",
                           "centers_num": "3"}[k]
                if str(env.get(k, default)) != v:
                    raise ValueError(f"env {k}={env.get(k, default)!r} contradicts the model's {DEFORM_CONFIG} ({v!r})")
    elif hidden is None:
        raise ValueError(f"{model_path}: no {DEFORM_CONFIG}; pass the ModelHiddenParams the model was trained with")
    scene = scene.to(device)
    scene.deformation = DeformationField.from_reference(state, hidden, env=env, device=device)
    return scene, it


def save_model_dir(scene: "GaussianScene", model_path: str, iteration: int, stage: str) -> str:
    """Scene.save (scene/__init__.py:98-101): point_cloud.ply + deformation.pth (+ the table and
    accumulator when the scene carries them) under model_path/point_cloud/{stage}_iteration_{N},
    plus deformation_config.json (the field's ModelHiddenParams and language-mode env switches,
    which the reference keeps outside the checkpoint; load_model_dir reads it back)."""
    d = os.path.join(model_path, "point_cloud", f"{stage}_iteration_{iteration}")
    os.makedirs(d, exist_ok=True)
    scene.save_ply(os.path.join(d, "point_cloud.ply"))
    if scene.deformation is not None:
        import json
        torch.save({k: v.cpu() for k, v in scene.deformation.state_dict().items()}, os.path.join(d, "deformation.pth"))
        with open(os.path.join(d, DEFORM_CONFIG), "w") as f:
            json.dump({"hidden": scene.deformation.hidden_params(), "env": scene.deformation.env_params()}, f)
    for k in ("deformation_table", "deformation_accum"):
        if k in scene.extra:
            torch.save(torch.as_tensor(scene.extra[k]).cpu(), os.path.join(d, f"{k}.pth"))
    return d


def write_ply_vertices(path: str, names: List[str], cols: np.ndarray) -> None:
    """binary_little_endian PLY with one float32 `vertex` element (what plyfile writes for the
    reference's save_ply)."""
    cols = np.ascontiguousarray(cols, dtype="<f4")
    if cols.ndim != 2 or cols.shape[1] != len(names):
        raise ValueError("one column per attribute name")
    header = ["ply", "format binary_little_endian 1.0", f"element vertex {cols.shape[0]}"]
    header += [f"property float {n}" for n in names]
    header += ["end_header"]
    with open(path, "wb") as f:
        f.write(("\n".join(header) + "\n").encode("ascii"))
        f.write(cols.tobytes())


def read_ply_vertices(path: str) -> Dict[str, np.ndarray]:
    """The `vertex` element of a PLY file (binary little/big endian or ascii; scalar properties)."""
    with open(path, "rb") as f:
        if f.readline().strip() != b"ply":
            raise ValueError(f"{path}: not a PLY file")
        fmt, elements, cur = None, [], None
        while True:
            line = f.readline()
            if not line:
                raise ValueError(f"{path}: no end_header")
            tok = line.decode("ascii", "replace").split()
            if not tok or tok[0] in ("comment", "obj_info"):
                continue
            if tok[0] == "end_header":
                break
            if tok[0] == "format":
                fmt = tok[1]
            elif tok[0] == "element":
                cur = [tok[1], int(tok[2]), []]
                elements.append(cur)
            elif tok[0] == "property":
                if tok[1] == "list":
                    raise ValueError(f"{path}: list properties are not supported")
                cur[2].append((tok[2], _PLY_TYPES[tok[1]]))
        out = None
        for name, count, props in elements:
            if fmt == "ascii":
                rows = [f.readline().split() for _ in range(count)]
                arr = np.array(rows, dtype=np.float64).reshape(count, len(props)) if count else \
                    np.zeros((0, len(props)))
                data = {p: arr[:, i].astype(t) for i, (p, t) in enumerate(props)}
            else:
                end = "<" if fmt == "binary_little_endian" else ">"
                dt = np.dtype([(p, end + t) for p, t in props])
                rec = np.frombuffer(f.read(dt.itemsize * count), dtype=dt, count=count)
                data = {p: rec[p].astype(rec[p].dtype.newbyteorder("=")) for p, _ in props}
            if name == "vertex":
                out = data
                break
        if out is None:
            raise ValueError(f"{path}: no vertex element")
        return out


# ---- render(): gaussian_renderer/__init__.py:19-248 -----------------------------------------------
class _Activate(torch.autograd.Function):
    """exp(scales), normalize(rotations), sigmoid(opacity) (gaussian_renderer/__init__.py:191-193) in one
    launch forward and one backward (lsr_activate / lsr_activate_backward, include/lsr_train.h)
    instead of about five PyTorch kernels forward and eight backward."""

    @staticmethod
    def forward(ctx, s_raw, r_raw, o_raw):
        from diff_gaussian_rasterization import _lib
        L = _lib.load()
        s_raw, r_raw, o_raw = s_raw.contiguous(), r_raw.contiguous(), o_raw.contiguous()
        if s_raw.dtype != torch.float32 or r_raw.shape[-1] != 4 or s_raw.shape[-1] != 3 \
                or not (s_raw.shape[0] == r_raw.shape[0] == o_raw.shape[0]) or o_raw.numel() != o_raw.shape[0]:
            raise ValueError("activate: float32 scales [N,3], rotations [N,4], opacity [N,1]")
        s, r, o = torch.empty_like(s_raw), torch.empty_like(r_raw), torch.empty_like(o_raw)
        p = lambda t: t.data_ptr()   # noqa: E731
        st = torch.cuda.current_stream(s_raw.device).cuda_stream
        _lib.check(L.lsr_activate(s_raw.shape[0], p(s_raw), p(r_raw), p(o_raw), p(s), p(r), p(o), st), "lsr_activate")
        ctx.save_for_backward(s, r_raw, o)
        return s, r, o

    @staticmethod
    def backward(ctx, ds, dr, do):
        from diff_gaussian_rasterization import _lib
        L = _lib.load()
        s, r_raw, o = ctx.saved_tensors
        need = ctx.needs_input_grad
        outs = [torch.empty_like(x) if need[k] else None for k, x in enumerate((s, r_raw, o))]
        g = [None if x is None else x.contiguous() for x in (ds, dr, do)]
        p = lambda t: None if t is None else t.data_ptr()   # noqa: E731
        st = torch.cuda.current_stream(s.device).cuda_stream
        _lib.check(L.lsr_activate_backward(s.shape[0], p(s), p(r_raw), p(o), p(g[0]), p(g[1]), p(g[2]),
                                           p(outs[0]), p(outs[1]), p(outs[2]), st), "lsr_activate_backward")
        return tuple(outs)


class _RepeatViews(torch.autograd.Function):
    """x.repeat(V, 1, ...) of several tensors in one launch, and their backward (the V row blocks
    summed) in one (lsr_repeat_rows / lsr_sum_row_blocks, include/lsr_train.h)."""

    @staticmethod
    def _jobs(pairs):
        from diff_gaussian_rasterization import _lib
        rows = (_lib.RowTensor * len(pairs))()
        for k, (src, dst) in enumerate(pairs):
            rows[k].src, rows[k].dst = src.data_ptr(), dst.data_ptr()
            rows[k].row_bytes, rows[k].zero_from = src[0].numel() * 4 if src.shape[0] else 4, 0
        return rows

    @staticmethod
    def forward(ctx, V, *xs):
        from diff_gaussian_rasterization import _lib
        xs = [x.contiguous() for x in xs]
        P = xs[0].shape[0]
        if any(x.dtype != torch.float32 or x.shape[0] != P for x in xs):
            raise ValueError("repeat_views: float32 tensors of the same row count")
        outs = [x.new_empty((V * P,) + tuple(x.shape[1:])) for x in xs]
        ctx.V, ctx.P, ctx.shapes = V, P, [tuple(x.shape) for x in xs]
        st = torch.cuda.current_stream(xs[0].device).cuda_stream
        _lib.check(_lib.load().lsr_repeat_rows(len(xs), _RepeatViews._jobs(list(zip(xs, outs))), P, V, st),
                   "lsr_repeat_rows")
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        from diff_gaussian_rasterization import _lib
        need = ctx.needs_input_grad[1:]
        grads, pairs = [], []
        for k, g in enumerate(gs):
            if not need[k] or g is None:
                grads.append(None)
                continue
            d = g.new_empty(ctx.shapes[k])
            pairs.append((g.contiguous(), d))
            grads.append(d)
        if pairs:
            st = torch.cuda.current_stream(pairs[0][0].device).cuda_stream
            _lib.check(_lib.load().lsr_sum_row_blocks(len(pairs), _RepeatViews._jobs(pairs), ctx.P, ctx.V, st),
                       "lsr_sum_row_blocks")
        return (None,) + tuple(grads)


_ZEROS = {}   # device -> a zero float buffer (the source of the absent views' gradient rows)


def _zeros_source(device, nbytes):
    z = _ZEROS.get(device)
    if z is None or z.numel() * 4 < nbytes:
        z = _ZEROS[device] = torch.zeros((nbytes + 3) // 4, device=device)
    return z


class _SplitViews(torch.autograd.Function):
    """The field's outputs over V * P rows split into the V views' row blocks (views, no copy), whose
    backward assembles every output's gradient from the views' in one launch (lsr_repeat_rows with
    one block: a multi-tensor copy) instead of one concatenation per output; absent view gradients
    read zeros."""

    @staticmethod
    def forward(ctx, V, *xs):
        P = xs[0].shape[0] // V
        ctx.V, ctx.P, ctx.shapes = V, P, [tuple(x.shape) for x in xs]
        ctx.set_materialize_grads(False)   # absent view gradients stay None (no zero tensors made)
        outs = []
        for x in xs:
            outs.extend(x.split(P))
        return tuple(outs)

    @staticmethod
    def backward(ctx, *gs):
        from diff_gaussian_rasterization import _lib
        V, P = ctx.V, ctx.P
        res, jobs, keep = [], [], []
        for k, shp in enumerate(ctx.shapes):
            part = gs[k * V:(k + 1) * V]
            if not ctx.needs_input_grad[1 + k] or all(g is None for g in part):
                res.append(None)
                continue
            ref = next(g for g in part if g is not None)
            out = ref.new_empty(shp)
            res.append(out)
            row = out[0].numel() * 4
            for b, g in enumerate(part):
                src = _zeros_source(out.device, P * row) if g is None else g.contiguous()
                keep.append(src)
                jobs.append((src.data_ptr(), out.data_ptr() + b * P * row, row))
        if not jobs:
            return (None,) + tuple(res)
        st = torch.cuda.current_stream(next(r for r in res if r is not None).device).cuda_stream
        L = _lib.load()
        for i in range(0, len(jobs), 32):
            chunk = jobs[i:i + 32]
            rows = (_lib.RowTensor * len(chunk))()
            for k, (src, dst, row) in enumerate(chunk):
                rows[k].src, rows[k].dst, rows[k].row_bytes, rows[k].zero_from = src, dst, row, 0
            _lib.check(L.lsr_repeat_rows(len(chunk), rows, P, 1, st), "lsr_repeat_rows")
        return (None,) + tuple(res)


def split_views(V, *xs):
    """xs' row blocks per view (tuples of V views each); on the GPU the backward is one launch."""
    live = [x for x in xs if x is not None]
    if not live or not live[0].is_cuda or live[0].shape[0] == 0:
        return [x.split(x.shape[0] // V) if x is not None else (None,) * V for x in xs]
    parts = iter(_SplitViews.apply(V, *live))
    return [tuple(next(parts) for _ in range(V)) if x is not None else (None,) * V for x in xs]


def repeat_views(V, *xs):
    """The tensors' rows repeated V times (render_views): one native launch each way on the GPU."""
    if xs[0].is_cuda and xs[0].shape[0] > 0:
        return _RepeatViews.apply(V, *xs)
    return tuple(x.repeat(V, *([1] * (x.dim() - 1))) for x in xs)


def activate(scales, rotations, opacity):
    """The render path's activations: one native launch each way on the GPU (_Activate); the PyTorch
    ops for host tensors or a missing input."""
    if scales is not None and rotations is not None and scales.is_cuda:
        return _Activate.apply(scales, rotations, opacity)
    return (torch.exp(scales) if scales is not None else None,
            torch.nn.functional.normalize(rotations) if rotations is not None else None, torch.sigmoid(opacity))


def _screenspace(pc):
    """The screen-space gradient carrier (gaussian_renderer/__init__.py:30-35): zeros + 0, grad retained."""
    sp = torch.zeros_like(pc.get_xyz, requires_grad=True, device=pc.xyz.device) + 0
    try:
        sp.retain_grad()
    except RuntimeError:
        pass
    return sp


def _raster_settings(viewpoint_camera, pc, bg_color, scaling_modifier, debug, include_feature, cam_type):
    """render()'s GaussianRasterizationSettings (gaussian_renderer/__init__.py:49-63, 74-76) and the
    view's time."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    dev = pc.xyz.device
    if cam_type != "PanopticSports":
        rs = GaussianRasterizationSettings(
            image_height=int(viewpoint_camera.image_height), image_width=int(viewpoint_camera.image_width),
            tanfovx=math.tan(viewpoint_camera.FoVx * 0.5), tanfovy=math.tan(viewpoint_camera.FoVy * 0.5),
            bg=bg_color, scale_modifier=scaling_modifier, viewmatrix=viewpoint_camera.world_view_transform.to(dev),
            projmatrix=viewpoint_camera.full_proj_transform.to(dev), sh_degree=pc.active_sh_degree,
            campos=viewpoint_camera.camera_center.to(dev), prefiltered=False, debug=debug,
            include_feature=include_feature)
        return rs, viewpoint_camera.time
    # the Panoptic reader's prebuilt settings, taken as they are (their include_feature, bg and
    # sh_degree included), and the frame time from the dict
    return viewpoint_camera["camera"], viewpoint_camera["time"]


def render(viewpoint_camera, pc: GaussianScene, bg_color: torch.Tensor, scaling_modifier: float = 1.0,
           override_color=None, stage: str = "fine-lang", compute_cov3D_python: bool = False,
           convert_SHs_python: bool = False, debug: bool = False, nonormalized: bool = False,
           language_feature_hiddendim: int = 3, cam_type: Optional[str] = None, _deformed=None):
    """The reference's render() on this build's rasterizer.  viewpoint_camera: FoVx, FoVy,
    image_width, image_height, world_view_transform, full_proj_transform, camera_center, time
    (synthetic.Camera or the reference Camera); with cam_type == "PanopticSports" a dict
    {"camera": GaussianRasterizationSettings, "time": t} as the Panoptic reader builds it
    (scene/dataset_readers.py:491-516, `panoptic_camera` here), whose settings are used as they are
    (gaussian_renderer/__init__.py:46, 74-76).  Environment switches of the reference
    (nonormalized, language_feature_hiddendim) are arguments here.  _deformed: this view's
    deformation outputs, already evaluated and activated (render_views); the field is then not
    called.

    One deliberate divergence: with override_color (or convert_SHs_python) the reference passes
    both shs_final and colors_precomp to the rasterizer (gaussian_renderer/__init__.py:219-228),
    and the upstream GaussianRasterizer raises "Please provide excatly one of either SHs or
    precomputed colors!" on that, so the reference's override path cannot run.  Here the SHs are
    dropped when colours are precomputed, so the path renders the given colours; the rasterizer
    itself (GaussianRasterizer.forward) keeps upstream's error for callers that pass both."""
    from diff_gaussian_rasterization import GaussianRasterizer

    dev = pc.xyz.device
    screenspace_points = _screenspace(pc)
    means3D = pc.get_xyz
    include_feature = "base" not in stage
    raster_settings, cam_time = _raster_settings(viewpoint_camera, pc, bg_color, scaling_modifier, debug,
                                                 include_feature, cam_type)
    rasterizer = GaussianRasterizer(raster_settings=raster_settings)
    opacity = pc.opacity
    scales = rotations = cov3D_precomp = None
    coff = None
    activated = False
    if _deformed is not None:   # render_views: the field's outputs for this view, activated there
        m3, s3, r3, o3, sh3, l3, coff = _deformed
        activated = True
    else:
        # the reference builds this with torch.tensor(time).to(device).repeat (a host-to-device copy,
        # which synchronises the stream): a fill gives the same values without the wait
        t = torch.full((means3D.shape[0], 1), float(cam_time), device=dev)
        shs = pc.get_features
        if include_feature:
            lang = pc.get_language_feature
            if not nonormalized:
                lang = lang / (lang.norm(dim=-1, keepdim=True) + 1e-9)
        else:
            lang = torch.zeros((pc.P, language_feature_hiddendim), dtype=opacity.dtype, device=dev)
        if compute_cov3D_python:
            cov3D_precomp = _covariance(pc.get_scaling, scaling_modifier, pc.rotation)
        else:
            scales, rotations = pc.scaling, pc.rotation
        if "coarse" in stage:
            m3, s3, r3, o3, sh3, l3 = means3D, scales, rotations, opacity, shs, lang
        elif "fine" in stage:
            if pc.deformation is None:
                raise ValueError("a 'fine' stage needs the scene's deformation field")
            if cov3D_precomp is not None:
                raise ValueError("compute_cov3D_python with a deformation field is not supported")
            # inside autograd (training) the field's backward runs (DeformationField.apply)
            deform = pc.deformation.apply if (torch.is_grad_enabled() and hasattr(pc.deformation, "apply")) \
                else pc.deformation
            # 'base' stages pass the language through (the reference sets no_dlang = 1 there,
            # gaussian_renderer/__init__.py:121-124)
            m3, s3, r3, o3, sh3, l3, coff = deform(means3D, scales, rotations, opacity, shs, lang, t,
                                                   no_dlang=True if "base" in stage else None)
        else:
            raise NotImplementedError(stage)
    if not activated:
        s3, r3, o3 = activate(s3, r3, o3)
    colors_precomp = None
    if override_color is not None:
        colors_precomp = override_color
    elif convert_SHs_python:
        # as the reference (gaussian_renderer/__init__.py:200-205): undeformed means and features
        shs_view = pc.get_features.transpose(1, 2).view(-1, 3, (pc.max_sh_degree + 1) ** 2)
        campos = raster_settings.campos.to(dev).reshape(1, 3) if cam_type == "PanopticSports" \
            else viewpoint_camera.camera_center.to(dev)
        dir_pp = pc.get_xyz - campos.repeat(pc.P, 1)
        dirs = dir_pp / dir_pp.norm(dim=1, keepdim=True)
        colors_precomp = torch.clamp_min(eval_sh(pc.active_sh_degree, shs_view, dirs) + 0.5, 0.0)
    image, lang_img, radii, depth = rasterizer(
        means3D=m3, means2D=screenspace_points, shs=None if colors_precomp is not None else sh3,
        colors_precomp=colors_precomp, language_feature_precomp=l3, opacities=o3, scales=s3, rotations=r3,
        cov3D_precomp=cov3D_precomp)
    if "base" in stage:
        lang_img = None
    return {"render": image, "language_feature_image": lang_img, "viewspace_points": screenspace_points,
            "visibility_filter": radii > 0, "radii": radii, "depth": depth, "coff": coff}


def render_views(cams: Sequence, pc: GaussianScene, bg_color: torch.Tensor, stage: str = "fine-lang",
                 nonormalized: bool = False, language_feature_hiddendim: int = 3, **kw):
    """render() for each camera of a batch, the deformation field evaluated ONCE for all of them.
    train.py:242-268 renders the batch's views one after the other, each with its own
    deform_network call at that view's time; here the Gaussians are repeated once per view and
    the field runs one launch over V * P rows (row block v at cams[v].time), then each view
    rasterizes its block.  Same values as the per-view loop (the field is per-row); the
    field's backward then runs once per iteration, not once per view (its plane-gradient
    replicas are cleared and folded once).  Falls back to per-view render() outside the 'fine'
    stages or for one view."""
    if "fine" not in stage or pc.deformation is None or len(cams) < 2 or kw.get("compute_cov3D_python"):
        return [render(c, pc, bg_color, stage=stage, nonormalized=nonormalized,
                       language_feature_hiddendim=language_feature_hiddendim, **kw) for c in cams]
    dev = pc.xyz.device
    V, P = len(cams), pc.P
    t = torch.cat([torch.full((P,), float(c.time), device=dev) for c in cams])
    deform = pc.deformation.apply if (torch.is_grad_enabled() and hasattr(pc.deformation, "apply")) \
        else pc.deformation
    ins = [pc.get_xyz, pc.scaling, pc.rotation, pc.opacity, pc.get_features]
    if "base" not in stage:
        lang = pc.get_language_feature
        if not nonormalized:
            lang = lang / (lang.norm(dim=-1, keepdim=True) + 1e-9)
        ins = list(repeat_views(V, *ins, lang))
    else:   # the passed-through zeros, made at the batch's size
        ins = list(repeat_views(V, *ins)) + [torch.zeros((V * P, language_feature_hiddendim), dtype=pc.opacity.dtype,
                                                          device=dev)]
    outs = list(deform(*ins, t, no_dlang=True if "base" in stage else None))
    # the activations (render(), gaussian_renderer/__init__.py:131-133) once over the V * P rows: the
    # same values row by row, a third of the launches forward and backward
    outs[1], outs[2], outs[3] = activate(outs[1], outs[2], outs[3])
    parts = split_views(V, *outs)
    if set(kw) - {"scaling_modifier", "debug"}:   # override / python paths: render() per view
        return [render(c, pc, bg_color, stage=stage, nonormalized=nonormalized,
                       language_feature_hiddendim=language_feature_hiddendim,
                       _deformed=tuple(p[v] for p in parts), **kw) for v, c in enumerate(cams)]
    # the views rasterized as one batch (their preprocesses ahead of their count waits), each
    # exactly as render() rasterizes it
    from diff_gaussian_rasterization import rasterize_views
    include_feature = "base" not in stage
    rss, sps, ins = [], [], []
    for v, c in enumerate(cams):
        rs, _ = _raster_settings(c, pc, bg_color, kw.get("scaling_modifier", 1.0), kw.get("debug", False),
                                 include_feature, None)
        m3, s3, r3, o3, sh3, l3, _ = (p[v] for p in parts)
        sp = _screenspace(pc)
        rss.append(rs)
        sps.append(sp)
        ins.append(dict(means3D=m3, means2D=sp, shs=sh3, language_feature_precomp=l3, opacities=o3, scales=s3,
                        rotations=r3))
    res = []
    for v, (image, lang_img, radii, depth) in enumerate(rasterize_views(rss, ins)):
        res.append({"render": image, "language_feature_image": None if "base" in stage else lang_img,
                    "viewspace_points": sps[v], "visibility_filter": radii > 0, "radii": radii, "depth": depth,
                    "coff": parts[6][v]})
    return res


def panoptic_camera(w: int, h: int, k, w2c, time: float, near: float = 0.01, far: float = 100.0,
                    device="cuda") -> dict:
    """The Panoptic Sports reader's camera (scene/dataset_readers.py:491-516 setup_camera): raster
    settings built from intrinsics k [3,3] and world-to-camera w2c [4,4] (OpenGL-style projection,
    black background, sh_degree 0, debug on), with the frame time, as render(cam_type="PanopticSports")
    takes it."""
    from diff_gaussian_rasterization import GaussianRasterizationSettings
    fx, fy, cx, cy = k[0][0], k[1][1], k[0][2], k[1][2]
    w2c = torch.as_tensor(w2c, dtype=torch.float32, device=device)
    cam_center = torch.inverse(w2c)[:3, 3]
    w2c = w2c.unsqueeze(0).transpose(1, 2)
    opengl_proj = torch.tensor([[2 * fx / w, 0.0, -(w - 2 * cx) / w, 0.0],
                                [0.0, 2 * fy / h, -(h - 2 * cy) / h, 0.0],
                                [0.0, 0.0, far / (far - near), -(far * near) / (far - near)],
                                [0.0, 0.0, 1.0, 0.0]], dtype=torch.float32, device=device).unsqueeze(0).transpose(1, 2)
    settings = GaussianRasterizationSettings(
        image_height=h, image_width=w, tanfovx=w / (2 * fx), tanfovy=h / (2 * fy),
        bg=torch.zeros(3, dtype=torch.float32, device=device), scale_modifier=1.0, viewmatrix=w2c,
        projmatrix=w2c.bmm(opengl_proj), sh_degree=0, campos=cam_center, prefiltered=False, debug=True)
    return {"camera": settings, "time": time}

_SH_C0 = 0.28209479177387814
_SH_C1 = 0.4886025119029199
_SH_C2 = (1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396)
_SH_C3 = (-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
          1.445305721320277, -0.5900435899266435)


def eval_sh(deg: int, sh: torch.Tensor, dirs: torch.Tensor) -> torch.Tensor:
    """SH -> colour for degree <= 3 (utils/sh_utils.py:57-112): sh [..., C, (deg+1)^2], dirs
    [..., 3] unit."""
    result = _SH_C0 * sh[..., 0]
    if deg > 0:
        x, y, z = dirs[..., 0:1], dirs[..., 1:2], dirs[..., 2:3]
        result = result - _SH_C1 * y * sh[..., 1] + _SH_C1 * z * sh[..., 2] - _SH_C1 * x * sh[..., 3]
        if deg > 1:
            xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
            result = (result + _SH_C2[0] * xy * sh[..., 4] + _SH_C2[1] * yz * sh[..., 5]
                      + _SH_C2[2] * (2.0 * zz - xx - yy) * sh[..., 6] + _SH_C2[3] * xz * sh[..., 7]
                      + _SH_C2[4] * (xx - yy) * sh[..., 8])
            if deg > 2:
                result = (result + _SH_C3[0] * y * (3 * xx - yy) * sh[..., 9] + _SH_C3[1] * xy * z * sh[..., 10]
                          + _SH_C3[2] * y * (4 * zz - xx - yy) * sh[..., 11]
                          + _SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[..., 12]
                          + _SH_C3[4] * x * (4 * zz - xx - yy) * sh[..., 13] + _SH_C3[5] * z * (xx - yy) * sh[..., 14]
                          + _SH_C3[6] * x * (xx - 3 * yy) * sh[..., 15])
    return result


def _covariance(scaling, scaling_modifier, rotation):
    """build_scaling_rotation + strip_symmetric (utils/general_utils.py:70-116)."""
    r = torch.nn.functional.normalize(rotation)
    w, x, y, z = r[:, 0], r[:, 1], r[:, 2], r[:, 3]
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
                     2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
                     2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], dim=1).view(-1, 3, 3)
    L = R @ torch.diag_embed(scaling_modifier * scaling)
    S = L @ L.transpose(1, 2)
    return torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], dim=1)


# ---- render.py's render_set -----------------------------------------------------------------------
def pca_compress(feature_map: torch.Tensor) -> torch.Tensor:
    """[C, H, W] -> [H, W, 3] in [0, 1] (render.py:52-65: sklearn PCA over pixels, min-max)."""
    from sklearn.decomposition import PCA
    C, H, W = feature_map.shape
    x = feature_map.permute(1, 2, 0).reshape(-1, C).detach().cpu().numpy()
    y = PCA(n_components=3).fit_transform(x).reshape(H, W, 3)
    y = (y - y.min()) / (y.max() - y.min())
    return torch.from_numpy(y)


def write_png(path: str, rgb: np.ndarray) -> None:
    """8-bit RGB PNG (zlib, no external imaging library)."""
    rgb = np.ascontiguousarray(rgb, dtype=np.uint8)
    H, W, _ = rgb.shape
    raw = b"".join(b"\x00" + rgb[y].tobytes() for y in range(H))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", W, H, 8, 2, 0, 0, 0))
                + chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))


def to8b(x: np.ndarray) -> np.ndarray:
    return (255 * np.clip(x, 0, 1)).astype(np.uint8)


def render_set(model_path: str, name: str, iteration, views, scene: GaussianScene, background: torch.Tensor,
               output_channel: str = "rgb", stage: str = "fine-lang", save_images: bool = True,
               save_npy: bool = True, **render_kw) -> float:
    """render.py:67-161 without ground truth (ONLY_EVAL): renders every view, writes
    {model_path}/{name}_{output_channel}/ours_{iteration}/renders_npy/{idx:05d}.npy ([H, W, C], the
    files eval/eval.py reads) and renders/{idx:05d}.png; returns the FPS as render.py prints it."""
    key = "render" if output_channel == "rgb" else "language_feature_image"
    base = os.path.join(model_path, f"{name}_{output_channel}", f"ours_{iteration}")
    render_path, npy_path = os.path.join(base, "renders"), os.path.join(base, "renders_npy")
    os.makedirs(render_path, exist_ok=True)
    os.makedirs(npy_path, exist_ok=True)
    outs, t1 = [], None
    with torch.no_grad():
        for idx, view in enumerate(views):
            if idx == 0:
                torch.cuda.synchronize()
                t1 = _time.time()
            outs.append(render(view, scene, background, stage=stage, **render_kw)[key])
        torch.cuda.synchronize()
        t2 = _time.time()
    fps = (len(views) - 1) / (t2 - t1) if len(views) > 1 else float("nan")
    print("FPS:", fps)
    for idx, r in enumerate(outs):
        if save_npy:
            np.save(os.path.join(npy_path, f"{idx:05d}.npy"), r.permute(1, 2, 0).cpu().numpy())
        if save_images:
            img = r if output_channel == "rgb" else (r + 1.0) / 2
            img = pca_compress(img).numpy() if img.shape[0] > 3 else img.permute(1, 2, 0).cpu().numpy()
            write_png(os.path.join(render_path, f"{idx:05d}.png"), to8b(img))
    return fps
