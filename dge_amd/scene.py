"""Gaussian parameter container with the reference's activation getters.

Restates the part of gaussiansplatting/scene/gaussian_model.py that feeds the
rasterizer (:42-57 activations, :221-258 getters incl. ``localize``/``mask``):
raw tensors _xyz [P,3], _features_dc [P,1,3], _features_rest [P,(D+1)^2-1,3],
_opacity [P,1], _scaling [P,3], _rotation [P,4] (w,x,y,z) and
  get_xyz = _xyz, get_features = cat(dc, rest), get_opacity = sigmoid,
  get_scaling = exp, get_rotation = F.normalize.
Also the seeded synthetic scene of SURVEY.md §8(d) used by tests and bench.py
(there is no network, hence no checkpoints; ``data: synthetic``).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


class GaussianScene:
    def __init__(self, xyz, features_dc, features_rest, opacity, scaling, rotation, sh_degree: int = 3):
        self._xyz = xyz
        self._features_dc = features_dc
        self._features_rest = features_rest
        self._opacity = opacity
        self._scaling = scaling
        self._rotation = rotation
        self.max_sh_degree = sh_degree
        self.active_sh_degree = sh_degree  # load_ply sets it from the file (gaussian_model.py:480, 534)
        self.localize = False
        self.mask = None

    # -- activation getters (gaussian_model.py:221-258) --------------------
    def _sel(self, t):
        return t[self.mask] if self.localize else t

    @property
    def get_xyz(self):
        return self._sel(self._xyz)

    @property
    def get_features(self):
        return torch.cat((self._sel(self._features_dc), self._sel(self._features_rest)), dim=1)

    @property
    def get_opacity(self):
        return torch.sigmoid(self._sel(self._opacity))

    @property
    def get_scaling(self):
        return torch.exp(self._sel(self._scaling))

    @property
    def get_rotation(self):
        return F.normalize(self._sel(self._rotation))

    def get_covariance(self, scaling_modifier=1.0):
        return build_covariance(self.get_scaling * scaling_modifier, self.get_rotation)

    def parameters(self):
        return [self._xyz, self._features_dc, self._features_rest, self._opacity, self._scaling, self._rotation]

    def num_points(self) -> int:
        return int(self._xyz.shape[0])

    def requires_grad_(self, flag: bool = True):
        for p in self.parameters():
            p.requires_grad_(flag)
        return self


def build_rotation(r):
    """general_utils.py:64-86 (normalised quaternion -> rotation matrix)."""
    norm = torch.sqrt(r[:, 0] * r[:, 0] + r[:, 1] * r[:, 1] + r[:, 2] * r[:, 2] + r[:, 3] * r[:, 3])
    q = r / norm[:, None]
    w, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([
        1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y),
        2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x),
        2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)], dim=-1).reshape(-1, 3, 3)
    return R


def build_covariance(scaling, rotation):
    """gaussian_model.py:42-46 + general_utils.py:88-110: strip_symmetric(L L^T), L = R S."""
    L = build_rotation(rotation) * scaling[:, None, :]
    cov = L @ L.transpose(1, 2)
    return torch.stack([cov[:, 0, 0], cov[:, 0, 1], cov[:, 0, 2], cov[:, 1, 1], cov[:, 1, 2], cov[:, 2, 2]], dim=-1)


def synthetic_scene(P: int, sh_degree: int = 3, seed: int = 0, radius: float = 2.0, scale: float = 0.02,
                    device="cpu", opacity_mean: float = 0.0, opacity_std: float = 1.5) -> GaussianScene:
    """Seeded scene of SURVEY.md §8(d): uniform ball, log-normal scales, random quaternions; raw opacity
    N(opacity_mean, opacity_std) (the survey's N(0, 1.5) by default; N(-2, 1) is the bench's high-live
    side config: mostly translucent Gaussians, so most of them reach the backward)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    d = torch.randn(P, 3, generator=g, dtype=torch.float64)
    d = d / d.norm(dim=1, keepdim=True).clamp_min(1e-12)
    r = radius * torch.rand(P, 1, generator=g, dtype=torch.float64) ** (1.0 / 3.0)
    xyz = (d * r).float()
    scaling = (math.log(scale) + 0.3 * torch.randn(P, 3, generator=g)).float()
    rotation = torch.randn(P, 4, generator=g).float()
    opacity = (opacity_mean + opacity_std * torch.randn(P, 1, generator=g)).float()
    n_rest = (sh_degree + 1) ** 2 - 1
    features_dc = (0.5 * torch.randn(P, 1, 3, generator=g)).float()
    features_rest = (0.1 * torch.randn(P, n_rest, 3, generator=g)).float()
    t = [x.to(device).contiguous() for x in (xyz, features_dc, features_rest, opacity, scaling, rotation)]
    return GaussianScene(*t, sh_degree=sh_degree)
