"""Host-side cost of one render() forward + backward (dev tool, GPU): a tiny scene makes the
GPU time negligible, so the step rate is the CPU path (Python, autograd, ctypes, launches).
Also a cProfile of the hottest Python functions."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.multiview import GradBucket  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
sc = synthetic_scene(2000, seed=0, device=dev).requires_grad_(True)
cam = orbit_camera(0, 3, 64, 64, device=dev)
g = torch.randn(3, 64, 64, device=dev)
bg = torch.zeros(3, device=dev)
bucket = GradBucket(sc.parameters())
pipe = PipelineParams()


def step():
    bucket.zero()
    render(cam, sc, pipe, bg)["render"].backward(g)


for _ in range(20):
    step()
torch.cuda.synchronize()
n = 300
t0 = time.perf_counter()
for _ in range(n):
    step()
torch.cuda.synchronize()
print(f"host-bound render fwd+bwd: {1e6 * (time.perf_counter() - t0) / n:.1f} us per render (tiny scene)")
pr = cProfile.Profile()
pr.enable()
for _ in range(100):
    step()
torch.cuda.synchronize()
pr.disable()
pstats.Stats(pr).sort_stats("tottime").print_stats(25)
