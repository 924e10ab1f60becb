"""Host cost of the pieces of one render fwd+bwd on a tiny scene (dev probe, GPU)."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd import _C, _native  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, _settings, render  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
sc = synthetic_scene(2000, seed=0, device=dev).requires_grad_(True)
cam = orbit_camera(0, 3, 64, 64, device=dev)
bg = torch.zeros(3, device=dev)
s = _settings(cam, bg, 1.0, 3)
g = torch.randn(3, 64, 64, device=dev)


def timeit(name, fn, n=300):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    t2 = time.perf_counter()
    print(f"{name:48s} host {1e6 * (t1 - t0) / n:8.1f} us/call   (incl. final sync {1e6 * (t2 - t0) / n:8.1f})")


args = (s.bg, sc._xyz, sc._features_dc, sc._features_rest, torch.empty(0, device=dev), sc._opacity, sc._scaling,
        sc._rotation, 1.0, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, 64, 64, 3, s.campos, False, False)
fw = _C.rasterize_gaussians_fused(*args)
K, color, depth, radii, geom, binning, img = fw
bargs = (s.bg, sc._xyz, sc._features_dc, sc._features_rest, torch.empty(0, device=dev), sc._opacity, sc._scaling,
         sc._rotation, radii, 1.0, s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, g, 3, s.campos, geom, K, binning,
         img, False)
L = _native.lib()
timeit("ctypes gs_abi_version", lambda: L.gs_abi_version())
timeit("torch.empty x1", lambda: torch.empty(16, device=dev))
timeit("torch.zeros_like(xyz)", lambda: torch.zeros_like(sc._xyz))
timeit("with torch.cuda.device(dev)", lambda: torch.cuda.device(dev).__enter__())
timeit("_C.rasterize_gaussians_fused (fwd C call)", lambda: _C.rasterize_gaussians_fused(*args))
timeit("_C.rasterize_gaussians_fused_backward", lambda: _C.rasterize_gaussians_fused_backward(*bargs))
with torch.no_grad():
    timeit("render() no_grad", lambda: render(cam, sc, PipelineParams(), bg))
timeit("render() with grad (fwd only)", lambda: render(cam, sc, PipelineParams(), bg))


def fb():
    render(cam, sc, PipelineParams(), bg)["render"].backward(g)


timeit("render() + backward", fb)
for p in sc.parameters():
    p.grad = None
_native.profile_enable(False)
