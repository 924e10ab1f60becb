"""Debug: render_views (batched) vs the per-view render() loop, per parameter and view count."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from dge_amd.cameras import orbit_camera
from dge_amd.gaussian_renderer import PipelineParams, render
from dge_amd.multiview import render_views
from dge_amd.scene import synthetic_scene

dev = torch.device("cuda")
W, H = 160, 128
for V, streams in ((1, 1), (2, 1), (2, 2), (4, 2)):
    cams = [orbit_camera(k, 4, W, H, device=dev) for k in range(V)]
    G = [torch.randn(3, H, W, generator=torch.Generator().manual_seed(30 + k)).to(dev) * 1e-2 for k in range(V)]
    bg = torch.zeros(3, device=dev)
    res = {}
    for mode in ("loop", "views"):
        sc = synthetic_scene(20_000, seed=4, device=dev).requires_grad_(True)
        if mode == "loop":
            vs = []
            for c, g in zip(cams, G):
                o = render(c, sc, PipelineParams(), bg)
                o["render"].backward(g)
                vs.append(o["viewspace_points"].grad)
        else:
            outs = render_views(cams, sc, PipelineParams(), bg, streams=streams)
            torch.autograd.backward([o["render"] for o in outs], G)
            vs = [o["viewspace_points"].grad for o in outs]
        torch.cuda.synchronize()
        res[mode] = ([p.grad.clone() for p in sc.parameters()], [v.clone() for v in vs])
    names = ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]
    for n, a, b in zip(names, res["loop"][0], res["views"][0]):
        d = (a - b).abs()
        print(V, streams, n, "max diff", float(d.max()), "frac", float((d > 1e-6 * a.abs().max()).float().mean()),
              "norms", float(a.norm()), float(b.norm()))
    for i, (a, b) in enumerate(zip(res["loop"][1], res["views"][1])):
        print(V, streams, "vs", i, float((a - b).abs().max()), float(a.norm()), float(b.norm()))
