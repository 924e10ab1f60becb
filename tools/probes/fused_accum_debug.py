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


def diff(a, b):
    return [(n, int((x != y).sum())) for n, x, y in zip(names, a, b) if not torch.equal(x, y)]


if __name__ == "__main__" and not os.environ.get("PROBE3"):
    GR._SPEC_RENDER = False
    ref = run(True, False, True)
    ref_sep = run(True, False, False)
    GR._SPEC_RENDER = True
    a = run(True, False, True)
    b = run(False, False, True)
    print("spec fused vs exact:", diff(a, ref))
    print("spec autograd vs exact:", diff(b, ref))
    print("exact joint vs separate:", diff(ref, ref_sep))
    c = run(True, False, False)
    print("spec separate fused vs exact joint:", diff(c, ref))


def per_view(spec, views, order=None, joint=False):
    GR._SPEC_RENDER = spec
    sc = synthetic_scene(15_000, seed=5, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
    outs = [render(cams[v], sc, PipelineParams(), bg)["render"] for v in views]
    losses = [(o * Gs[v]).sum() for o, v in zip(outs, views)]
    if joint:
        sum(losses).backward()
    else:
        for i in (order or range(len(losses))):
            losses[i].backward()
    return [p.grad.clone() for p in sc.parameters()]


def probe3():
    e0, e1 = per_view(False, [0]), per_view(False, [1])
    s0, s1 = per_view(True, [0]), per_view(True, [1])
    print("single view 0 spec vs exact:", diff(s0, e0), " view 1:", diff(s1, e1))
    j = per_view(True, [0, 1], joint=True)
    print("spec joint vs view0 alone:", diff(j, s0))
    print("spec joint vs view1 alone:", diff(j, s1))
    r = per_view(True, [0, 1], order=[1, 0])
    ej = per_view(False, [0, 1], joint=True)
    print("spec separate reversed vs exact joint:", diff(r, ej))
    print("spec joint vs exact joint:", diff(j, ej))
    # view 1's render after view 0's: does it disturb view 0's saved state?  view 0's backward first, jointly
    GR._SPEC_RENDER = True
    sc = synthetic_scene(15_000, seed=5, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
    o0 = render(cams[0], sc, PipelineParams(), bg)["render"]
    o1 = render(cams[1], sc, PipelineParams(), bg)["render"]
    (o0 * Gs[0]).sum().backward()
    g0 = [p.grad.clone() for p in sc.parameters()]
    print("spec: view 0 backward after view 1's forward vs view 0 alone:", diff(g0, s0))


if __name__ == "__main__" and os.environ.get("PROBE3"):
    probe3()
