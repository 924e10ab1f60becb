"""Which case / parameter of test_fused_gradient_accumulation differs, with and without the speculated
training render (dev probe, GPU)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd import gaussian_renderer as GR  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.diff_gaussian_rasterization import set_fused_grad_accumulation  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda")
cams = [orbit_camera(k, 4, 160, 120, device=dev) for k in range(2)]
Gs = [torch.randn(3, 120, 160, generator=torch.Generator().manual_seed(30 + k)).to(dev) for k in range(2)]
bg = torch.zeros(3, device=dev)
names = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]


def run(fused, pre_grad, batched):
    prev = set_fused_grad_accumulation(fused)
    try:
        sc = synthetic_scene(15_000, seed=5, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
        if pre_grad:
            for p in sc.parameters():
                p.grad = torch.full_like(p, 0.25)
        outs = [render(c, sc, PipelineParams(), bg)["render"] for c in cams]
        if batched:
            sum((o * g).sum() for o, g in zip(outs, Gs)).backward()
        else:
            for o, g in zip(outs, Gs):
                (o * g).sum().backward()
        return [p.grad.clone() for p in sc.parameters()]
    finally:
        set_fused_grad_accumulation(prev)


if __name__ == "__main__":
    for spec in (False, True):
      GR._SPEC_RENDER = spec
      for pre_grad in (False, True):
          for batched in (False, True):
              a, b = run(True, pre_grad, batched), run(False, pre_grad, batched)
              bad = [(n, int((x != y).sum()), float((x - y).abs().max())) for n, x, y in zip(names, a, b)
                     if not torch.equal(x, y)]
              print(f"spec {spec} pre_grad {pre_grad} batched {batched}: {bad}")
  # the speculated render against the exact one, per view, forward and per-view backward alone
  for spec in (True, False):
      GR._SPEC_RENDER = spec
      sc = synthetic_scene(15_000, seed=5, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
      res = []
      for c, g in zip(cams, Gs):
          pkg = render(c, sc, PipelineParams(), bg)
          (pkg["render"] * g).sum().backward()
          res.append((pkg["render"].detach().clone(), [p.grad.clone() for p in sc.parameters()]))
          for p in sc.parameters():
              p.grad = None
      if spec:
          got = res
      else:
          for v, ((ia, ga), (ib, gb)) in enumerate(zip(got, res)):
              print(f"view {v}: image equal {torch.equal(ia, ib)}",
                    [(n, int((x != y).sum())) for n, x, y in zip(names, ga, gb) if not torch.equal(x, y)])
