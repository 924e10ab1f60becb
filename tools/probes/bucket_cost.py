"""Cost of GradBucket.allreduce's sparse-row bookkeeping on the GPU, collectives stubbed out
(dev probe): live-row mask, union agreement, pack, unpack, for a bucket holding the gradients of
24 views (the c3 union, ~24% of the rows)."""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.multiview import GradBucket  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
P = 1_000_000
sc = synthetic_scene(P, seed=0, device=dev).requires_grad_(True)
bg = torch.zeros(3, device=dev)
bucket = GradBucket(list(sc.parameters()))
for k in range(24):
    cam = orbit_camera(k, 24, 512, 512, device=dev)
    render(cam, sc, PipelineParams(), bg)["render"].backward(torch.randn(3, 512, 512, device=dev) * 1e-3)
torch.cuda.synchronize()
saved = bucket.flat.clone()
dist.is_available = lambda: True
dist.is_initialized = lambda: True
dist.get_world_size = lambda group=None: 8
dist.all_reduce = lambda t, op=None, group=None, async_op=False: None
for it in range(8):
    bucket.flat.copy_(saved)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    bucket.allreduce()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if it >= 3:
        print(f"sparse allreduce bookkeeping (collectives stubbed): {dt * 1e6:.0f} us")
assert torch.equal(bucket.flat, saved)
live = (bucket.flat[:P * 3].view(P, 3) != 0).any(1)
print(f"rows live in the bucket: {live.float().mean():.3f}")
