"""Fraction of Gaussians with a nonzero gradient over the union of k views (dev probe, GPU):
the share of the gradient bucket a sparse all-reduce would move."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
P = 1_000_000
sc = synthetic_scene(P, seed=0, device=dev).requires_grad_(True)
bg = torch.zeros(3, device=dev)
union = torch.zeros(P, dtype=torch.bool, device=dev)
for n_views in (24,):
    for k in range(n_views):
        for p in sc.parameters():
            p.grad = None
        cam = orbit_camera(k, n_views, 512, 512, device=dev)
        render(cam, sc, PipelineParams(), bg)["render"].backward(torch.randn(3, 512, 512, device=dev) * 1e-3)
        nz = (sc._xyz.grad != 0).any(1) | (sc._opacity.grad != 0).any(1)
        union |= nz
        if k + 1 in (1, 3, 6, 12, 24):
            print(f"views {k + 1:2d}: live this view {nz.float().mean():.3f}, union {union.float().mean():.3f}")
