"""Kernel trace target: 50 backward C calls on a tiny scene (dev probe, GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd import _C  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import _settings  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
sc = synthetic_scene(2000, seed=0, device=dev).requires_grad_(True)
cam = orbit_camera(0, 3, 64, 64, device=dev)
bg = torch.zeros(3, device=dev)
s = _settings(cam, bg, 1.0, 3)
g = torch.randn(3, 64, 64, device=dev)
e = torch.empty(0, device=dev)
args = (s.bg, sc._xyz, sc._features_dc, sc._features_rest, e, sc._opacity, sc._scaling, sc._rotation, 1.0,
        s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, 64, 64, 3, s.campos, False, False)
K, color, depth, radii, geom, binning, img = _C.rasterize_gaussians_fused(*args)
bargs = (s.bg, sc._xyz, sc._features_dc, sc._features_rest, e, sc._opacity, sc._scaling, sc._rotation, radii, 1.0,
         s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, g, 3, s.campos, geom, K, binning, img, False)
torch.cuda.synchronize()
for _ in range(50):
    _C.rasterize_gaussians_fused_backward(*bargs)
torch.cuda.synchronize()
print("done")
