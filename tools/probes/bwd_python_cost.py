"""Where the host time of the autograd backward goes (dev probe, GPU, tiny scene)."""
import collections
import functools
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import dge_amd.diff_gaussian_rasterization as R  # noqa: E402
from dge_amd import _C  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.defaultdict(int)


def wrap(mod, name):
    f = getattr(mod, name)

    @functools.wraps(f)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[name] += time.perf_counter() - t0
            cnt[name] += 1
    setattr(mod, name, w)


for n in ("_accumulation_mode", "_into_target", "_mask_owner", "_order_grad_writes_begin", "_order_grad_writes_end",
          "_call_with_snapshot"):
    wrap(R, n)
wrap(_C, "rasterize_gaussians_fused_backward")
orig_bwd = R._RasterizeGaussiansFused.backward


def bwd(ctx, *g):
    t0 = time.perf_counter()
    try:
        return orig_bwd(ctx, *g)
    finally:
        acc["Function.backward"] += time.perf_counter() - t0
        cnt["Function.backward"] += 1


R._RasterizeGaussiansFused.backward = staticmethod(bwd)
dev = torch.device("cuda", 0)
sc = synthetic_scene(2000, seed=0, device=dev).requires_grad_(True)
cam = orbit_camera(0, 3, 64, 64, device=dev)
bg = torch.zeros(3, device=dev)
g = torch.randn(3, 64, 64, device=dev)
for _ in range(30):
    render(cam, sc, PipelineParams(), bg)["render"].backward(g)
torch.cuda.synchronize()
acc.clear()
cnt.clear()
n = 300
t0 = time.perf_counter()
tb = 0.0
for _ in range(n):
    out = render(cam, sc, PipelineParams(), bg)["render"]
    t1 = time.perf_counter()
    out.backward(g)
    tb += time.perf_counter() - t1
torch.cuda.synchronize()
print(f"total {1e6 * (time.perf_counter() - t0) / n:.1f} us/iter, out.backward() {1e6 * tb / n:.1f} us")
for k in sorted(acc, key=lambda k: -acc[k]):
    print(f"  {k:40s} {1e6 * acc[k] / n:8.1f} us/iter ({cnt[k] / n:.1f} calls)")
