"""Host-side profile of the default bench step (dev probe, GPU): cProfile over 30 steps of bench.run_views
(c2, 3 views on 3 streams, one backward), top functions by own time and by cumulative time."""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import bench  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams  # noqa: E402
from dge_amd.multiview import GradBucket  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

sys.argv = ["bench.py"]
args = bench.parse()
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
P, W, H, V = args.points, args.width, args.height, args.views_per_rank
scene = synthetic_scene(P, sh_degree=args.sh_degree, seed=0, device=dev).requires_grad_(True)
cams = [orbit_camera(k, V, W, H, device=dev) for k in range(V)]
gen = torch.Generator(device="cpu").manual_seed(1)
seeds = [(torch.randn(3, H, W, generator=gen) * 1e-3).to(dev) for _ in range(V)]
bg = torch.zeros(3, device=dev)
pipe = PipelineParams()
bucket = GradBucket(scene.parameters())


def step():
    bench.run_views(args, cams, scene, pipe, bg, seeds, bucket)


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
st.sort_stats("tottime").print_stats(25)
st.sort_stats("cumulative").print_stats(30)
