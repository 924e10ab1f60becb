"""Compiled binding vs ctypes (dev probe, GPU): render()'s pre-launch host time (render() entry -> the native
forward's first half returned, per training render) and DGE's unchanged loop (bench.py's dge_loop_unchanged
shape: per view a training render, the semantic render with the edit mask, the boolean-mask visualisation; the
masked l1 and one backward), alternating the two paths (dge_amd._C._GT set / None) on one box."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd import _C  # noqa: E402
from dge_amd import gaussian_renderer as GR  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

assert _C._GT is not None, "the compiled binding is not built / loaded"
GT = _C._GT
dev = torch.device("cuda", 0)
P, W, H, V = 1_000_000, 512, 512, 3
sc = synthetic_scene(P, seed=0, device=dev).requires_grad_(True)
cams = [orbit_camera(k, V, W, H, device=dev) for k in range(V)]
bg = torch.zeros(3, device=dev)
pipe = GR.PipelineParams()
mask = (torch.rand(P, generator=torch.Generator().manual_seed(5)) < 0.2).to(dev)
gts = [torch.rand(H, W, 3, generator=torch.Generator().manual_seed(50 + i)).to(dev) for i in range(V)]
pre, native = [], []
_begin = _C.rasterize_gaussians_fused_begin
_entry = [0.0]


def begin_timed(*a, **k):
    r = _begin(*a, **k)
    if _entry[0]:
        pre.append(time.perf_counter() - _entry[0])
    return r


_C.rasterize_gaussians_fused_begin = begin_timed


class _Proxy:
    """the binding with its fused_begin timed: the Python before the native call (render() entry -> the call)
    and the call itself (structs, allocations and the native first half's HIP calls)"""

    def __getattr__(self, n):
        return getattr(GT, n)

    def fused_begin(self, *a):
        t = time.perf_counter()
        if _entry[0]:
            native.append(t - _entry[0])  # (replaced by the call's own time below)
        r = GT.fused_begin(*a)
        if _entry[0]:
            native[-1] = (t - _entry[0], time.perf_counter() - t)
        return r


PROXY = _Proxy()


def render(*a, **k):
    _entry[0] = time.perf_counter() if k.get("override_color") is None else 0.0
    return GR.render(*a, **k)


def loop():
    for p in sc.parameters():
        p.grad = None
    sc.mask = mask
    images, masks, radii = [], [], None
    for i, cam in enumerate(cams):
        pkg = render(cam, sc, pipe, bg)
        image, r = pkg["render"], pkg["radii"]
        radii = r if i == 0 else torch.max(r, radii)
        sm = render(cam, sc, pipe, bg, override_color=sc.mask[..., None].float().repeat(1, 3))["render"]
        sm = torch.norm(sm, dim=0) > 0.8
        viz = image.detach().clone().permute(1, 2, 0)
        viz[sm] = 0.40 * viz[sm] + 0.60 * torch.tensor([1.0, 0.0, 0.0], device=dev)
        masks.append(sm)
        images.append(image.permute(1, 2, 0))
    images = torch.stack(images, 0)
    m = torch.stack(masks, 0)[..., None].float()
    torch.nn.functional.l1_loss(images * m, torch.stack(gts, 0) * m).backward()


res = {"torch": [], "ctypes": []}
pres = {"torch": [], "ctypes": []}
split = []
for rnd in range(4):
    for mode in ("torch", "ctypes"):
        _C._GT = PROXY if mode == "torch" else None
        for _ in range(3):
            loop()
        torch.cuda.synchronize()
        pre.clear()
        native.clear()
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            loop()
        torch.cuda.synchronize()
        res[mode].append(n * V / (time.perf_counter() - t0))
        pres[mode].append(statistics.median(pre) * 1e6)
        if mode == "torch":
            split.append((statistics.median(x[0] for x in native) * 1e6, statistics.median(x[1] for x in native) * 1e6))
_C._GT = GT
print(json.dumps({"dge_loop_views_per_s": {k: [round(x, 1) for x in v] for k, v in res.items()},
                  "render_entry_to_first_half_enqueued_us_median": {k: [round(x, 1) for x in v] for k, v in pres.items()},
                  "binding_python_before_native_call_us": [round(a, 1) for a, _ in split],
                  "binding_native_first_half_call_us": [round(b, 1) for _, b in split]}))
