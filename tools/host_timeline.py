"""Host-side timeline of the bench step (dev tool, GPU): wall time of each phase of the default c2
step (3 views on 3 streams, one backward) as the host sees it — each render() call (split at the
instance-count wait inside the C forward via the stage profiler being off: we time the whole call),
the bucket zero and the autograd backward — against the GPU step time, to show where the host waits."""
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dge_amd import gaussian_renderer as GR  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.multiview import GradBucket, render_views  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
DIST = os.environ.get("DIST") == "1"  # run the bucket's sparse all-reduce protocol on a one-rank RCCL group
if DIST:
    import torch.distributed as dist

    dist.init_process_group("nccl", device_id=dev)
P, W, H, V = 1_000_000, 512, 512, 3
scene = synthetic_scene(P, sh_degree=3, seed=0, device=dev).requires_grad_(True)
cams = [orbit_camera(k, V, W, H, device=dev) for k in range(V)]
gen = torch.Generator(device="cpu").manual_seed(1)
seeds = [(torch.randn(3, H, W, generator=gen) * 1e-3).to(dev) for _ in range(V)]
bg = torch.zeros(3, device=dev)
pipe = GR.PipelineParams()
bucket = GradBucket(scene.parameters())
streams = int(os.environ.get("STREAMS", "3"))

stamps = []
_render = GR.render


def timed_render(*a, **k):
    t0 = time.perf_counter()
    out = _render(*a, **k)
    stamps.append(("render", time.perf_counter() - t0))
    return out


GR.render = timed_render

from dge_amd import _C  # noqa: E402
from dge_amd import diff_gaussian_rasterization as DR  # noqa: E402


def _wrap(mod, name, tag):
    f = getattr(mod, name)

    def w(*a, **k):
        t0 = time.perf_counter()
        r = f(*a, **k)
        stamps.append((tag, time.perf_counter() - t0))
        return r
    setattr(mod, name, w)


_wrap(_C, "rasterize_gaussians_fused", "C fwd")
_wrap(_C, "rasterize_gaussians_fused_begin", "C begin")
_wrap(_C, "rasterize_gaussians_fused_end", "C end")
_wrap(GR, "_fused_begin", "py begin")
_wrap(GR, "_fused_end", "py end")
_wrap(_C, "rasterize_gaussians_fused_backward", "C bwd")
_bw = DR._RasterizeGaussiansFused.backward


def _timed_bw(ctx, *g):
    t0 = time.perf_counter()
    r = _bw(ctx, *g)
    stamps.append(("py bwd", time.perf_counter() - t0))
    return r


DR._RasterizeGaussiansFused.backward = staticmethod(_timed_bw)


def step():
    t0 = time.perf_counter()
    outs = render_views(cams, scene, pipe, bg, streams=streams)
    t1 = time.perf_counter()
    bucket.zero(overlap=streams > 1 and not os.environ.get("SERIAL_ZERO"))
    t2 = time.perf_counter()
    torch.autograd.backward([o["render"] for o in outs], seeds)
    t3 = time.perf_counter()
    if DIST:
        bucket.allreduce(min_world=1)
        stamps.append(("allreduce", time.perf_counter() - t3))
    stamps.append(("views", t1 - t0))
    stamps.append(("zero", t2 - t1))
    stamps.append(("backward", t3 - t2))


for _ in range(5):
    step()
torch.cuda.synchronize()
stamps.clear()
n = 40
t0 = time.perf_counter()
for _ in range(n):
    step()
th = time.perf_counter() - t0
torch.cuda.synchronize()
tw = time.perf_counter() - t0
print(f"streams {streams}: host loop {1e3 * th / n:.3f} ms/step, wall {1e3 * tw / n:.3f} ms/step "
      f"({n * V / tw:.0f} renders/s)")
for name in ("render", "C fwd", "py begin", "C begin", "py end", "C end", "views", "zero", "backward", "py bwd",
             "C bwd", "allreduce", "ar live", "ar max", "ar nonzero", "ar gather", "ar sum", "ar scatter"):
    v = [d for k, d in stamps if k == name]
    if not v:
        continue
    print(f"  {name:9s} median {1e6 * statistics.median(v):8.1f} us  p90 {1e6 * sorted(v)[int(0.9 * len(v))]:8.1f} us"
          f"  x{len(v) / n:.0f}/step")

if DIST:
    import dge_amd.multiview as MV

    _wrap(MV, "_rows_live", "ar live")
    _wrap(MV, "_rows_gather", "ar gather")
    _wrap(MV, "_rows_scatter", "ar scatter")
    _nz = torch.nonzero
    _ar = dist.all_reduce

    def nz(*a, **k):
        t0 = time.perf_counter()
        r = _nz(*a, **k)
        stamps.append(("ar nonzero", time.perf_counter() - t0))
        return r

    def ar(t, *a, **k):
        t0 = time.perf_counter()
        r = _ar(t, *a, **k)
        stamps.append(("ar max" if t.dtype == torch.uint8 else "ar sum", time.perf_counter() - t0))
        return r
    torch.nonzero = nz
    MV.dist.all_reduce = ar
    stamps.clear()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    tw = time.perf_counter() - t0
    print(f"DIST phases: wall {1e3 * tw / n:.3f} ms/step")
    for name in ("views", "backward", "allreduce", "ar live", "ar max", "ar nonzero", "ar gather", "ar sum",
                 "ar scatter"):
        v = [d for k, d in stamps if k == name]
        if v:
            print(f"  {name:10s} median {1e6 * statistics.median(v):8.1f} us")
    dist.destroy_process_group()

if os.environ.get("CPROFILE"):
    import cProfile
    import pstats

    GR.render = _render
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        step()
    torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(30)
