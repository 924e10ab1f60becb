"""Side measurements for the non-headline BASELINE configs (dev tool, GPU).

One JSON line per workload:
  c4    configs[3]: 2.5M Gaussians, 1920x1080, forward only (tile-sort stress)
  c5    configs[4]: 1.0M scene, localize on a 200k mask (sorted by x), fp16 SH, 512x512 fwd+bwd
  adam  SURVEY.md §8(f) F3: the optimizer step over a 1.0M-Gaussian model (59 floats / Gaussian):
        FusedAdam (one gfx950 kernel) vs torch.optim.Adam (foreach) on the same tensors
bench.py stays the headline (c2) measurement; its line carries these same legs (legs.c4_hd_forward, c5_local_edit,
f3_adam).
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import leg_adam, leg_c4, leg_c5  # noqa: E402  (the same legs bench.py's line carries)

dev = torch.device("cuda", 0)


def c4(steps, warmup):
    return leg_c4(dev, steps, warmup)


def c5(steps, warmup):
    return leg_c5(dev, steps, warmup)


def adam(steps, warmup):
    return leg_adam(dev, steps, warmup)


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("workloads", nargs="*", default=["c4", "c5", "adam"])
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    for w in a.workloads:
        print(json.dumps({"c4": c4, "c5": c5, "adam": adam}[w](a.steps, a.warmup)), flush=True)
