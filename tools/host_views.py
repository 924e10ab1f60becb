"""Host-side cost of the bench's batched 3-view step (dev tool, GPU): a tiny scene makes the GPU time
negligible, so the step rate is the issuing thread's cost (Python, autograd, ctypes, HIP calls) of
render_views (speculated) + one backward + the batch check + the bucket zero beside the forwards.
Prints ms/step and a cProfile of the hottest functions."""
import cProfile
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams  # noqa: E402
from dge_amd.multiview import GradBucket, render_views, view_streams  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
V = 3
sc = synthetic_scene(2000, seed=0, device=dev).requires_grad_(True)
cams = [orbit_camera(k, V, 64, 64, device=dev) for k in range(V)]
seeds = [torch.randn(3, 64, 64, device=dev) for _ in range(V)]
bg = torch.zeros(3, device=dev)
bucket = GradBucket(sc.parameters())
pipe = PipelineParams()


def step():
    main = torch.cuda.current_stream()
    ready = main.record_event()
    outs = render_views(cams, sc, pipe, bg, streams=V, speculate=True)
    bucket.zero(stream=view_streams(dev, V)[1], after=ready)
    torch.autograd.backward([o["render"] for o in outs], seeds)
    assert outs.check()


for _ in range(20):
    step()
torch.cuda.synchronize()
N = 300
t0 = time.perf_counter()
for _ in range(N):
    step()
t1 = time.perf_counter()
torch.cuda.synchronize()
print(f"host issue {1e3 * (t1 - t0) / N:.3f} ms/step (GPU drained {1e3 * (time.perf_counter() - t0) / N:.3f})")
pr = cProfile.Profile()
pr.enable()
for _ in range(100):
    step()
pr.disable()
torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(30)
