"""Camera -> rasterizer matrices (the input contract of the hot path).

Restates gaussiansplatting/utils/graphics_utils.py:40-93 (getWorld2View2,
getProjectionMatrix, fov2focal, focal2fov) and the matrix construction of
Simple_Camera (gaussiansplatting/scene/cameras.py:59-96):
  world_view_transform = getWorld2View2(R, T).T          (column-major view)
  full_proj_transform  = world_view_transform @ getProjectionMatrix(...).T
  camera_center        = inverse(world_view_transform)[3, :3]
``R`` is the camera-to-world rotation as stored by the COLMAP loaders (its
transpose rotates world into camera), ``T`` the world-to-camera translation;
camera +z looks forward, +y points down.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def get_world2view2(R, t, translate=np.array([0.0, 0.0, 0.0]), scale=1.0) -> np.ndarray:
    Rt = np.zeros((4, 4))
    Rt[:3, :3] = np.asarray(R).transpose()
    Rt[:3, 3] = t
    Rt[3, 3] = 1.0
    C2W = np.linalg.inv(Rt)
    C2W[:3, 3] = (C2W[:3, 3] + translate) * scale
    return np.float32(np.linalg.inv(C2W))


def get_projection_matrix(znear: float, zfar: float, fovX: float, fovY: float) -> torch.Tensor:
    tan_y, tan_x = math.tan(fovY / 2), math.tan(fovX / 2)
    top, right = tan_y * znear, tan_x * znear
    bottom, left = -top, -right
    P = torch.zeros(4, 4, dtype=torch.float32)
    P[0, 0] = 2.0 * znear / (right - left)
    P[1, 1] = 2.0 * znear / (top - bottom)
    P[0, 2] = (right + left) / (right - left)
    P[1, 2] = (top + bottom) / (top - bottom)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def fov2focal(fov: float, pixels: int) -> float:
    return pixels / (2 * math.tan(fov / 2))


def focal2fov(focal: float, pixels: int) -> float:
    return 2 * math.atan(pixels / (2 * focal))


class Camera:
    """The attributes render() reads from a Simple_Camera (cameras.py:59-96)."""

    def __init__(self, R, T, FoVx, FoVy, height, width, device="cuda", znear=0.01, zfar=100.0, uid=0,
                 trans=np.array([0.0, 0.0, 0.0]), scale=1.0):
        self.R, self.T = np.asarray(R, np.float64), np.asarray(T, np.float64)
        self.trans, self.scale = np.asarray(trans, np.float64), float(scale)
        self.FoVx, self.FoVy = float(FoVx), float(FoVy)
        self.image_height, self.image_width = int(height), int(width)
        self.znear, self.zfar = znear, zfar
        self.uid = uid
        self.world_view_transform = torch.tensor(get_world2view2(self.R, self.T, self.trans, self.scale)).transpose(
            0, 1).to(device)
        self.projection_matrix = get_projection_matrix(znear, zfar, self.FoVx, self.FoVy).transpose(0, 1).to(device)
        self.full_proj_transform = (self.world_view_transform.unsqueeze(0).bmm(
            self.projection_matrix.unsqueeze(0))).squeeze(0).float()
        self.camera_center = self.world_view_transform.inverse()[3, :3]

    def to(self, device):
        return Camera(self.R, self.T, self.FoVx, self.FoVy, self.image_height, self.image_width, device, self.znear,
                      self.zfar, self.uid, self.trans, self.scale)


def look_at_R_T(position, target=(0.0, 0.0, 0.0), world_up=(0.0, 0.0, 1.0)):
    """COLMAP-convention (R = camera-to-world rotation, T = world-to-camera translation)."""
    C = np.asarray(position, np.float64)
    f = np.asarray(target, np.float64) - C
    f /= np.linalg.norm(f)
    x = np.cross(f, np.asarray(world_up, np.float64))
    if np.linalg.norm(x) < 1e-8:
        x = np.cross(f, np.array([0.0, 1.0, 0.0]))
    x /= np.linalg.norm(x)
    y = np.cross(f, x)  # points "down" relative to world_up
    R = np.stack([x, y, f], axis=1)
    T = -R.T @ C
    return R, T


def orbit_camera(k: int, n: int, width: int = 512, height: int = 512, distance: float = 5.0,
                 elevation_deg: float = 15.0, fovx_deg: float = 60.0, device="cuda") -> Camera:
    """Camera k of n on an orbit around the origin (SURVEY.md §8(d) bench cameras)."""
    az = 2.0 * math.pi * k / max(n, 1)
    el = math.radians(elevation_deg)
    pos = distance * np.array([math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el)])
    R, T = look_at_R_T(pos)
    fovx = math.radians(fovx_deg)
    fovy = 2.0 * math.atan(math.tan(fovx / 2) * height / width)
    return Camera(R, T, fovx, fovy, height, width, device=device, uid=k)
