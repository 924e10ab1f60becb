"""Host cost of the pieces of render()'s path before its first kernel launch (dev probe, GPU)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd import _C, _native as N  # noqa: E402
from dge_amd import gaussian_renderer as GR  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
sc = synthetic_scene(20000, seed=0, device=dev).requires_grad_(True)
sc.mask = torch.rand(20000, device=dev) < 0.2
cam = orbit_camera(0, 3, 64, 64, device=dev)
bg = torch.zeros(3, device=dev)
pipe = GR.PipelineParams()
rs = GR._settings(cam, bg, 1.0, 3)


def timeit(name, fn, n=2000):
    for _ in range(50):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{name:52s} {1e6 * (t1 - t0) / n:8.2f} us/call")


def dev_ctx():
    with torch.cuda.device(dev):
        pass


vis = torch.empty(20000, dtype=torch.bool, device=dev)
timeit("_fused_ok", lambda: GR._fused_ok(sc, pipe))
timeit("gaussian_renderer._settings", lambda: GR._settings(cam, bg, 1.0, 3))
timeit("torch.empty(bool)", lambda: torch.empty(20000, dtype=torch.bool, device=dev))
timeit("_may_backward", lambda: GR._may_backward(sc._xyz, sc._features_dc, sc._features_rest, None, sc._opacity,
                                                sc._scaling, sc._rotation))
timeit("N.require_gpu", lambda: N.require_gpu(sc._xyz))
timeit("with torch.cuda.device(dev)", dev_ctx)
timeit("_C._f32(xyz)", lambda: _C._f32(sc._xyz, "xyz"))
timeit("_C._features(f_rest)", lambda: _C._features(sc._features_rest, "f"))
timeit("_C._params", lambda: _C._params(20000, sc._xyz, sc._features_dc, sc._features_rest, None, sc._opacity,
                                        sc._scaling, sc._rotation, None, vis, False, None))
timeit("_C._settings", lambda: _C._settings(rs.bg, rs.viewmatrix, rs.projmatrix, rs.campos, rs.tanfovx, rs.tanfovy,
                                            64, 64, 3, 1.0, False, False))
timeit("_C._Allocator", lambda: _C._Allocator(dev))
timeit("_C._stream", lambda: _C._stream(dev))
timeit("ctypes call (gs_abi_version)", lambda: N.lib().gs_abi_version())
timeit("aux contiguous().view(uint8)", lambda: sc.mask.contiguous().view(torch.uint8))
timeit("_viewspace_zeros", lambda: GR._viewspace_zeros(20000, torch.float32, dev))
timeit("torch.cuda.current_stream", lambda: torch.cuda.current_stream(dev))
with torch.no_grad():
    timeit("render() no_grad (whole)", lambda: GR.render(cam, sc, pipe, bg), n=500)
timeit("render() grad, aux (whole)", lambda: GR.render(cam, sc, pipe, bg), n=500)
