"""Side measurements for the non-headline BASELINE configs (dev tool, GPU).

One JSON line per workload:
  c4    configs[3]: 2.5M Gaussians, 1920x1080, forward only (tile-sort stress)
  c5    configs[4]: 1.0M scene, localize on a 200k mask (sorted by x), fp16 SH, 512x512 fwd+bwd
  adam  SURVEY.md §8(f) F3: the optimizer step over a 1.0M-Gaussian model (59 floats / Gaussian):
        FusedAdam (one gfx950 kernel) vs torch.optim.Adam (foreach) on the same tensors
bench.py stays the headline (c2) measurement.
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dge_amd import _native  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)


def timed(fn, steps, warmup):
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / steps


def stages(fn, n=3):
    _native.profile_stages(None)
    _native.profile_enable(True)
    _native.profile_collect()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    prof = _native.profile_collect()
    _native.profile_enable(False)
    return {k: round(ms / c, 4) for k, (ms, c) in prof.items() if c}


def c4(steps, warmup):
    P, W, H = 2_500_000, 1920, 1080
    sc = synthetic_scene(P, seed=2, device=dev)
    cam = orbit_camera(0, 1, W, H, device=dev)
    bg = torch.zeros(3, device=dev)

    def fwd():
        with torch.no_grad():
            render(cam, sc, PipelineParams(), bg)

    dt = timed(fwd, steps, warmup)
    return {"workload": "c4: 2.5M Gaussians, 1920x1080, fp32 forward only", "value": round(1.0 / dt, 2),
            "unit": "renders/s", "ms_per_render": round(1e3 * dt, 3), "stages_ms": stages(fwd)}


def c5(steps, warmup):
    P, Psub, W, H = 1_000_000, 200_000, 512, 512
    sc = synthetic_scene(P, seed=0, device=dev)
    sc._features_dc = sc._features_dc.half()
    sc._features_rest = sc._features_rest.half()
    mask = torch.zeros(P, dtype=torch.bool, device=dev)
    mask[torch.argsort(sc._xyz[:, 0])[:Psub]] = True
    sc.mask, sc.localize = mask, True
    sc.requires_grad_(True)
    cam = orbit_camera(0, 1, W, H, device=dev)
    g = torch.randn(3, H, W, device=dev) * 1e-3
    bg = torch.zeros(3, device=dev)

    def step():
        for p in sc.parameters():
            p.grad = None
        (render(cam, sc, PipelineParams(), bg)["render"] * g).sum().backward()

    dt = timed(step, steps, warmup)
    return {"workload": "c5: 1.0M scene, localize 200k (x-sorted 20%), fp16 SH, 512x512 fwd+bwd",
            "value": round(1.0 / dt, 2), "unit": "renders/s", "ms_per_render": round(1e3 * dt, 3),
            "stages_ms": stages(step)}


def adam(steps, warmup):
    from dge_amd.optim import FusedAdam

    P = 1_000_000
    shapes = [(P, 3), (P, 1, 3), (P, 15, 3), (P, 1), (P, 3), (P, 4)]
    lrs = [1.6e-4, 0.0125, 0.0125 / 20, 0.05, 0.005, 0.001]
    out = {"workload": "F3: Adam step over 1.0M Gaussians (59 floats each)"}
    for name, cls in (("fused", FusedAdam), ("torch_foreach", torch.optim.Adam)):
        ps = [torch.nn.Parameter(torch.randn(s, device=dev)) for s in shapes]
        for p in ps:
            p.grad = torch.randn_like(p) * 1e-3
        opt = cls([{"params": [p], "lr": lr} for p, lr in zip(ps, lrs)], lr=0.0, eps=1e-15)
        dt = timed(opt.step, steps, warmup)
        bytes_ = 59 * P * 28  # read p, g, m, v; write p, m, v
        out[name] = {"ms": round(1e3 * dt, 4), "algorithmic_GBps": round(bytes_ / dt / 1e9, 1)}
    out["speedup"] = round(out["torch_foreach"]["ms"] / out["fused"]["ms"], 2)
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="*", default=["c4", "c5", "adam"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    for w in a.workloads:
        print(json.dumps({"c4": c4, "c5": c5, "adam": adam}[w](a.steps, a.warmup)), flush=True)
