"""Host-side timeline of the multi-stream view loop (dev probe, GPU): where does the host block?"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.multiview import GradBucket, stream_pool  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
sc = synthetic_scene(1_000_000, seed=0, device=dev).requires_grad_(True)
cams = [orbit_camera(k, 3, 512, 512, device=dev) for k in range(3)]
G = [torch.randn(3, 512, 512, device=dev) * 1e-3 for _ in range(3)]
bg = torch.zeros(3, device=dev)
pipe = PipelineParams()
bucket = GradBucket(sc.parameters())


def step(nstreams, log=None):
    bucket.zero()
    main = torch.cuda.current_stream()
    pool = stream_pool(dev, nstreams) if nstreams > 1 else [main]
    ready = main.record_event()
    t0 = time.perf_counter()
    for i, (cam, g) in enumerate(zip(cams, G)):
        s = pool[i % len(pool)]
        if s != main:
            s.wait_event(ready)
        with torch.cuda.stream(s):
            ta = time.perf_counter()
            out = render(cam, sc, pipe, bg)
            tb = time.perf_counter()
            out["render"].backward(g)
            tc = time.perf_counter()
        if log is not None:
            log.append((i, (ta - t0) * 1e6, (tb - t0) * 1e6, (tc - t0) * 1e6))
    for s in pool:
        if s != main:
            main.wait_stream(s)


for n in (1, 2):
    for _ in range(8):
        step(n)
    torch.cuda.synchronize()
    st0 = torch.cuda.memory_stats().get("num_device_alloc", -1)
    log = []
    t0 = time.perf_counter()
    for _ in range(10):
        step(n, log)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    st1 = torch.cuda.memory_stats().get("num_device_alloc", -1)
    print(f"streams={n}: {dt * 1e6:.0f} us/step, device allocs during timing {st1 - st0}")
    for rec in log[-3:]:
        print("   view %d: render start %.0f, fwd returned %.0f, bwd returned %.0f us" % rec)
