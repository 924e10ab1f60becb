"""Host time per phase of the bench's distributed step on a one-rank RCCL group (dev probe, GPU):
RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=... python tools/probes/dist_phases.py"""
import os
import sys
import time

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams  # noqa: E402
from dge_amd.multiview import GradBucket, render_views, view_streams  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    P, W, H, V = 1_000_000, 512, 512, 3
    sc = synthetic_scene(P, seed=0, device=dev).requires_grad_(True)
    cams = [orbit_camera(k, V, W, H, device=dev) for k in range(V)]
    g = torch.Generator().manual_seed(1)
    seeds = [(torch.randn(3, H, W, generator=g) * 1e-3).to(dev) for _ in range(V)]
    bg = torch.zeros(3, device=dev)
    bucket = GradBucket(sc.parameters())
    pipe = PipelineParams()
    names = ["zero+render", "allreduce_begin", "backward", "check", "allreduce_end"]
    tot = {k: 0.0 for k in names}

    def step(rec):
        t = [time.perf_counter()]
        main = torch.cuda.current_stream()
        ready = main.record_event()
        outs = render_views(cams, sc, pipe, bg, streams=3, speculate=True)
        bucket.zero(stream=view_streams(dev, 3)[1], after=ready)
        t.append(time.perf_counter())
        bucket.allreduce_begin([o.get("_live_rows") for o in outs], min_world=1)
        t.append(time.perf_counter())
        torch.autograd.backward([o["render"] for o in outs], seeds)
        t.append(time.perf_counter())
        assert outs.check()
        t.append(time.perf_counter())
        bucket.allreduce_end()
        t.append(time.perf_counter())
        if rec:
            for i, k in enumerate(names):
                tot[k] += t[i + 1] - t[i]

    # allreduce_end's own parts: the wait for the union, then the pack / SUM / unpack issue
    import dge_amd.multiview as MV
    orig_sync = torch.cuda.Event.synchronize
    sub = {"union wait": 0.0}

    def timed_sync(self):
        t = time.perf_counter()
        orig_sync(self)
        sub["union wait"] += time.perf_counter() - t
    torch.cuda.Event.synchronize = timed_sync
    for _ in range(10):
        step(False)
    sub["union wait"] = 0.0
    torch.cuda.synchronize()
    n = 50
    t0 = time.perf_counter()
    for _ in range(n):
        step(True)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(f"step {1e3 * dt / n:.3f} ms; host per phase (ms):", {k: round(1e3 * v / n, 3) for k, v in tot.items()},
          {k: round(1e3 * v / n, 3) for k, v in sub.items()})
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
