"""Host time of DGE's loop split by our functions (dev probe, GPU): the loop of dge_loop_profile.py with
perf_counter wrappers around render(), the autograd node's backward, the deferred passes and the _C calls.
A wrapper's time includes any wait for the GPU inside it (the count read after the preprocess)."""
import collections
import functools
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import dge_amd.diff_gaussian_rasterization as R  # noqa: E402
from dge_amd import _C  # noqa: E402
from dge_amd import gaussian_renderer as GR  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

acc = collections.defaultdict(float)
cnt = collections.defaultdict(int)


def timed(name, f):
    @functools.wraps(f)
    def w(*a, **k):
        t0 = time.perf_counter()
        try:
            return f(*a, **k)
        finally:
            acc[name] += time.perf_counter() - t0
            cnt[name] += 1
    return w


for n in ("rasterize_gaussians_fused_begin", "rasterize_gaussians_fused_end", "render_recolor",
          "rasterize_gaussians_fused_backward", "rasterize_backward_passes"):
    setattr(_C, n, timed("_C." + n, getattr(_C, n)))
R._run_deferred_passes = timed("deferred_passes", R._run_deferred_passes)
_bwd = R._RasterizeGaussiansFused.backward
R._RasterizeGaussiansFused.backward = staticmethod(timed("node.backward", _bwd))
render = timed("render()", GR.render)
# the pre-launch part of a training render: render() entry -> the native begin call
from dge_amd import _native as N  # noqa: E402
_lib = N.lib()
_begin = _lib.gs_rasterize_forward_begin
_t_entry = [0.0]


def _render_marked(*a, **k):
    _t_entry[0] = time.perf_counter()
    try:
        return render(*a, **k)
    finally:
        _t_entry[0] = 0.0


def _begin_marked(*a):
    t = time.perf_counter()
    _t_entry[0] = 0.0
    acc["render() entry -> native begin"] += t - _t_entry[0]
    cnt["render() entry -> native begin"] += 1
    try:
        return _begin(*a)
    finally:
        acc["native begin"] += time.perf_counter() - t
        cnt["native begin"] += 1


_lib.gs_rasterize_forward_begin = _begin_marked
# the timeline of the pre-launch path: time since render() entry at the entry of each step (training renders)
_marks = collections.defaultdict(float)
_mark_n = collections.defaultdict(int)


def _marked(name, mod, attr):
    f = getattr(mod, attr)

    def w(*a, **k):
        if _t_entry[0]:
            _marks[name] += time.perf_counter() - _t_entry[0]
            _mark_n[name] += 1
        return f(*a, **k)
    setattr(mod, attr, w)


for _name, _mod, _attr in (("GR._fused_ok", GR, "_fused_ok"), ("GR._render_fused", GR, "_render_fused"),
                           ("GR._settings", GR, "_settings"), ("GR._may_backward", GR, "_may_backward"),
                           ("_C._index32", _C, "_index32"), ("_C._params", _C, "_params"),
                           ("_C._settings", _C, "_settings"), ("_C._stream", _C, "_stream")):
    _marked(_name, _mod, _attr)

dev = torch.device("cuda", 0)
P, W, H, V = 1_000_000, 512, 512, 3
sc = synthetic_scene(P, seed=0, device=dev).requires_grad_(True)
cams = [orbit_camera(k, V, W, H, device=dev) for k in range(V)]
bg = torch.zeros(3, device=dev)
pipe = GR.PipelineParams()
sc.mask = (torch.rand(P, generator=torch.Generator().manual_seed(5)) < 0.2).to(dev)
gts = [torch.rand(H, W, 3, generator=torch.Generator().manual_seed(50 + i)).to(dev) for i in range(V)]


def loop(t):
    for p in sc.parameters():
        p.grad = None
    images, masks, radii = [], [], None
    for i, cam in enumerate(cams):
        pkg = _render_marked(cam, sc, pipe, bg)
        image, r = pkg["render"], pkg["radii"]
        radii = r if i == 0 else torch.max(r, radii)
        sm = render(cam, sc, pipe, bg, override_color=sc.mask[..., None].float().repeat(1, 3))["render"]
        sm = torch.norm(sm, dim=0) > 0.8
        viz = image.detach().clone().permute(1, 2, 0)
        t0 = time.perf_counter()
        viz[sm] = 0.40 * viz[sm] + 0.60 * torch.tensor([1.0, 0.0, 0.0], device=dev)
        t["viz (host sync)"] += time.perf_counter() - t0
        masks.append(sm)
        images.append(image.permute(1, 2, 0))
    images = torch.stack(images, 0)
    m = torch.stack(masks, 0)[..., None].float()
    loss = torch.nn.functional.l1_loss(images * m, torch.stack(gts, 0) * m)
    t0 = time.perf_counter()
    loss.backward()
    t["loss.backward()"] += time.perf_counter() - t0


extra = collections.defaultdict(float)
for _ in range(5):
    loop(extra)
torch.cuda.synchronize()
acc.clear()
cnt.clear()
extra.clear()
n = 30
t0 = time.perf_counter()
for _ in range(n):
    loop(extra)
torch.cuda.synchronize()
dt = time.perf_counter() - t0
print(f"dge loop: {n * V / dt:.1f} views/s, {dt / n * 1e6:.0f} us per iteration of {V} views")
for k in sorted(acc, key=lambda k: -acc[k]):
    print(f"  {k:42s} {acc[k] / n * 1e6:8.0f} us per iteration, {acc[k] / cnt[k] * 1e6:7.1f} us per call x {cnt[k] // n}")
for k, v in extra.items():
    print(f"  {k:42s} {v / n * 1e6:8.0f} us per iteration")
print("  pre-launch timeline (us since render() entry, training renders):")
for k in sorted(_marks, key=lambda k: _marks[k] / max(1, _mark_n[k])):
    print(f"    {k:40s} {_marks[k] / max(1, _mark_n[k]) * 1e6:8.1f}")

if os.environ.get("PROFILE"):
    import cProfile
    import pstats
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(n):
        loop(extra)
    torch.cuda.synchronize()
    pr.disable()
    st = pstats.Stats(pr)
    st.sort_stats("tottime").print_stats(30)
