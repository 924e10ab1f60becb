"""Does running views on separate HIP streams overlap their kernels? (dev probe, GPU)
c2 scene, 3 views: forward-only renders on one stream vs round-robin over 2/3 streams."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
sc = synthetic_scene(1_000_000, seed=0, device=dev)
cams = [orbit_camera(k, 3, 512, 512, device=dev) for k in range(3)]
bg = torch.zeros(3, device=dev)
pipe = PipelineParams()


def run(nstreams, iters=20):
    streams = [torch.cuda.Stream() for _ in range(nstreams)] if nstreams > 1 else [torch.cuda.current_stream()]
    main = torch.cuda.current_stream()

    def once():
        ev = main.record_event()
        for i, cam in enumerate(cams):
            s = streams[i % len(streams)]
            s.wait_event(ev)
            with torch.cuda.stream(s), torch.no_grad():
                render(cam, sc, pipe, bg)
        for s in streams:
            main.wait_stream(s)

    for _ in range(5):
        once()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters):
        once()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / iters / len(cams) * 1e6


for n in (1, 2, 3, 1):
    print(f"{n} stream(s): {run(n):.1f} us per forward render")
