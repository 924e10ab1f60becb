"""Blend-kernel timeline diagnostics (dev tool, GPU).

Renders the c2 workload once (forward + backward) with the library's per-wave
timestamps on and prints, for each blend kernel: the kernel span, the
distribution of per-wave/per-tile durations, the correlation with kept entries
and rounds, and how many waves are still running over time (tail shape).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dge_amd import _native  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402


def summarize(name, d):
    if d.size == 0:
        print(name, "no data")
        return
    start, end = d[:, 0].astype(np.int64), d[:, 1].astype(np.int64)
    live = end > 0
    start, end, kept, rounds = start[live], end[live], d[live, 2].astype(np.int64), d[live, 3].astype(np.int64)
    t0 = start.min()
    dur = (end - start) * 10e-3  # us (100 MHz)
    span = (end.max() - t0) * 10e-3
    print(f"== {name}: {live.sum()} items, span {span:.1f} us, start spread {(start.max() - t0) * 10e-3:.1f} us")
    for q in (50, 90, 99, 99.9, 100):
        print(f"   dur p{q}: {np.percentile(dur, q):.2f} us")
    print(f"   kept mean {kept.mean():.1f} max {kept.max()}  rounds mean {rounds.mean():.2f} max {rounds.max()}")
    if kept.std() > 0:
        A = np.stack([kept, rounds, np.ones_like(kept)], 1).astype(np.float64)
        coef, *_ = np.linalg.lstsq(A, dur, rcond=None)
        print(f"   fit dur ~ {coef[0] * 1e3:.2f} ns/kept + {coef[1]:.3f} us/round + {coef[2]:.2f} us")
    order = np.argsort(-dur)[:5]
    for i in order:
        print(f"   slowest: item {i} dur {dur[i]:.1f} kept {kept[i]} rounds {rounds[i]} start {(start[i] - t0) * 10e-3:.1f}")
    ts = np.linspace(0, span, 11)
    alive = [int(((start - t0) * 10e-3 <= t).sum() - ((end - t0) * 10e-3 <= t).sum()) for t in ts]
    print("   running over time:", " ".join(f"{t:.0f}:{a}" for t, a in zip(ts, alive)))


def main():
    dev = torch.device("cuda", 0)
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    W = H = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    scene = synthetic_scene(P, sh_degree=3, seed=0, device=dev).requires_grad_(True)
    cam = orbit_camera(0, 3, W, H, device=dev)
    g = (torch.randn(3, H, W, generator=torch.Generator().manual_seed(1)) * 1e-3).to(dev)
    bg = torch.zeros(3, device=dev)
    for _ in range(3):
        render(cam, scene, PipelineParams(), bg)["render"].backward(g)
    torch.cuda.synchronize()
    _native.diag_enable(True)
    render(cam, scene, PipelineParams(), bg)["render"].backward(g)
    torch.cuda.synchronize()
    _native.diag_enable(False)
    summarize("render_fwd (per wave)", _native.diag_read(0))
    summarize("render_bwd (per tile)", _native.diag_read(1))


if __name__ == "__main__":
    main()
