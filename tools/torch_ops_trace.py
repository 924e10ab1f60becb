"""Which torch ops launch kernels around one c2 render step (dev tool, GPU)."""
import os
import sys

import torch
from torch.profiler import ProfilerActivity, profile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.multiview import GradBucket  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
sc = synthetic_scene(1_000_000, seed=0, device=dev).requires_grad_(True)
cam = orbit_camera(0, 3, 512, 512, device=dev)
g = torch.randn(3, 512, 512, device=dev) * 1e-3
bg = torch.zeros(3, device=dev)
bucket = GradBucket(sc.parameters())


def step():
    bucket.zero()
    out = render(cam, sc, PipelineParams(), bg)["render"]
    out.backward(g)


for _ in range(3):
    step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA]) as prof:
    step()
    torch.cuda.synchronize()
print(prof.key_averages(group_by_input_shape=True).table(sort_by="cuda_time_total", row_limit=40))
