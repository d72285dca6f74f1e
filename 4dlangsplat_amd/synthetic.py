"""Synthetic scenes and cameras for the rasterizer benchmark and parity tests.

Camera matrices restate the reference's convention (scene/cameras.py:56-67,
utils/graphics_utils.py:38-71): world_view_transform = getWorld2View2(R, T).T,
projection = getProjectionMatrix(znear, zfar, fovX, fovY).T, full_proj = view @ proj,
camera_center = inverse(view)[3, :3].  The restatement is pinned against the reference's own
functions by tests/golden/cameras.npz (tests/golden/make_golden.py).

The S2M scene follows SURVEY.md section 8(d): camera at the origin looking down +z,
W x H = 1352 x 1014, tanfov 0.6 / 0.45, z ~ U(2, 10), x, y inside 1.1x the frustum, log-scales
~ N(-5, 0.5) with 1 % of Gaussians +ln 10, quaternions ~ N(0, I4) normalised,
opacity = sigmoid(N(0, 1.5)), SH DC ~ N(0, 0.5), rest ~ N(0, 0.1) (degree 3), language
features ~ N(0, I_C) L2-normalised, bg = (1, 1, 1).  Seeded torch.Generator on the CPU.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np
import torch


def get_world2view2(R, t, translate=np.array([0.0, 0.0, 0.0]), scale=1.0):
    """utils/graphics_utils.py:38-49 restated (float64 math, float32 result)."""
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = np.asarray(R).transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    cam_center = (C2W[:3, 3] + translate) * scale
    C2W[:3, 3] = cam_center
    return np.float32(np.linalg.inv(C2W))


def get_projection_matrix(znear, zfar, fovX, fovY):
    """utils/graphics_utils.py:51-71 restated."""
    tan_y, tan_x = math.tan(fovY / 2), math.tan(fovX / 2)
    top, right = tan_y * znear, tan_x * znear
    bottom, left = -top, -right
    P = torch.zeros(4, 4)
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


@dataclass
class Camera:
    image_width: int
    image_height: int
    FoVx: float
    FoVy: float
    world_view_transform: torch.Tensor  # [4,4] float32
    projection_matrix: torch.Tensor
    full_proj_transform: torch.Tensor
    camera_center: torch.Tensor         # [3]
    time: float = 0.0

    @property
    def tanfovx(self):
        return math.tan(self.FoVx * 0.5)

    @property
    def tanfovy(self):
        return math.tan(self.FoVy * 0.5)


def make_camera(R, T, FoVx, FoVy, width, height, znear=0.01, zfar=100.0, time=0.0) -> Camera:
    """scene/cameras.py:56-67 restated."""
    wv = torch.tensor(get_world2view2(np.asarray(R, dtype=np.float64), np.asarray(T, dtype=np.float64))).transpose(0, 1)
    pr = get_projection_matrix(znear, zfar, FoVx, FoVy).transpose(0, 1)
    full = wv.unsqueeze(0).bmm(pr.unsqueeze(0)).squeeze(0)
    center = wv.inverse()[3, :3]
    return Camera(width, height, FoVx, FoVy, wv.contiguous(), pr.contiguous(), full.contiguous(),
                  center.contiguous(), time)


def yaw_matrix(deg):
    a = math.radians(deg)
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, 0.0, s], [0.0, 1.0, 0.0], [-s, 0.0, c]])


def origin_camera(width=1352, height=1014, tanfovx=0.6, tanfovy=None) -> Camera:
    if tanfovy is None:
        tanfovy = tanfovx * height / width
    return make_camera(np.eye(3), np.zeros(3), 2 * math.atan(tanfovx), 2 * math.atan(tanfovy), width, height)


def camera_batch(n, width=1352, height=1014, tanfovx=0.6, seed=1, max_yaw=15.0, sigma_t=0.05):
    """cfg4 camera batch: origin camera yawed U(-15, 15) deg and translated N(0, 0.05^2)."""
    g = torch.Generator().manual_seed(seed)
    yaws = (torch.rand(n, generator=g, dtype=torch.float64) * 2 - 1) * max_yaw
    trans = torch.randn(n, 3, generator=g, dtype=torch.float64) * sigma_t
    tanfovy = tanfovx * height / width
    cams = []
    for i in range(n):
        cams.append(make_camera(yaw_matrix(float(yaws[i])), trans[i].numpy(), 2 * math.atan(tanfovx),
                                2 * math.atan(tanfovy), width, height))
    return cams


@dataclass
class Scene:
    means3D: torch.Tensor     # [P,3]
    scales: torch.Tensor      # [P,3] activated (exp)
    rotations: torch.Tensor   # [P,4] activated (normalised)
    opacities: torch.Tensor   # [P,1] activated (sigmoid)
    shs: torch.Tensor         # [P,16,3]
    lang: torch.Tensor        # [P,C] L2-normalised
    sh_degree: int = 3

    @property
    def P(self):
        return self.means3D.shape[0]

    def to(self, device):
        return Scene(*(t.to(device) for t in (self.means3D, self.scales, self.rotations, self.opacities,
                                              self.shs, self.lang)), self.sh_degree)


def make_scene(P, C=32, tanfovx=0.6, tanfovy=0.45, seed=0, z_range=(2.0, 10.0), logscale_mean=-5.0,
               logscale_std=0.5, big_frac=0.01, sh_degree=3) -> Scene:
    """Seeded S2M-style scene; generated on the CPU for reproducibility."""
    g = torch.Generator().manual_seed(seed)
    z = torch.rand(P, generator=g) * (z_range[1] - z_range[0]) + z_range[0]
    u = torch.rand(P, generator=g) * 2 - 1
    v = torch.rand(P, generator=g) * 2 - 1
    means = torch.stack([u * z * tanfovx * 1.1, v * z * tanfovy * 1.1, z], dim=1)
    logs = torch.randn(P, 3, generator=g) * logscale_std + logscale_mean
    big = torch.rand(P, generator=g) < big_frac
    logs[big] += math.log(10.0)
    scales = torch.exp(logs)
    q = torch.randn(P, 4, generator=g)
    rots = q / q.norm(dim=1, keepdim=True)
    opac = torch.sigmoid(torch.randn(P, 1, generator=g) * 1.5)
    M = (sh_degree + 1) ** 2
    shs = torch.randn(P, M, 3, generator=g) * 0.1
    shs[:, 0, :] = torch.randn(P, 3, generator=g) * 0.5
    if C > 0:
        lang = torch.randn(P, C, generator=g)
        lang = lang / (lang.norm(dim=-1, keepdim=True) + 1e-9)
    else:
        lang = torch.zeros(P, 0)
    return Scene(means.contiguous(), scales.contiguous(), rots.contiguous(), opac.contiguous(),
                 shs.contiguous(), lang.contiguous(), sh_degree)
