"""cProfile of the host side of the c2 view loop on 2 streams (dev probe, GPU)."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams  # noqa: E402
from dge_amd.multiview import GradBucket, render_backward_views  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
P = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
sc = synthetic_scene(P, seed=0, device=dev).requires_grad_(True)
cams = [orbit_camera(k, 3, 512, 512, device=dev) for k in range(3)]
G = [torch.randn(3, 512, 512, device=dev) * 1e-3 for _ in range(3)]
bg = torch.zeros(3, device=dev)
pipe = PipelineParams()
bucket = GradBucket(sc.parameters())


def step():
    bucket.zero()
    render_backward_views(cams, sc, pipe, bg, G, streams=2)


for _ in range(10):
    step()
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(30):
    step()
torch.cuda.synchronize()
pr.disable()
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
