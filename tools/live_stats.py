"""Live-set statistics of the c2 backward (dev tool, GPU): how many Gaussians
get records, their tiles_touched / record counts (gauss_bwd_live's loop trips)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dge_amd import _C, _native  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import _settings  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
P, W, H = 1_000_000, 512, 512
sc = synthetic_scene(P, seed=0, device=dev)
cam = orbit_camera(0, 3, W, H, device=dev)
bg = torch.zeros(3, device=dev)
s = _settings(cam, bg, 1.0, 3)
e = torch.empty(0, device=dev)
K, color, depth, radii, geom, binning, img = _C.rasterize_gaussians(
    bg, sc.get_xyz, e, sc.get_opacity, sc.get_scaling, sc.get_rotation, 1.0, e, s.viewmatrix, s.projmatrix,
    s.tanfovx, s.tanfovy, H, W, sc.get_features, 3, s.campos, False, False)
g = torch.randn(3, H, W, device=dev) * 1e-3
_C.rasterize_gaussians_backward(bg, sc.get_xyz, radii, e, sc.get_scaling, sc.get_rotation, 1.0, e, s.viewmatrix,
                                s.projmatrix, s.tanfovx, s.tanfovy, g, sc.get_features, 3, s.campos, geom, K, binning,
                                img, False)
torch.cuda.synchronize()
L = _native.lib()
off = lambda b, f: L.gs_buffer_offset(b, f, P, W, H, K)  # noqa: E731
touched = geom[off(b"geometry", b"touched"):][:P].cpu().numpy() != 0
tt = geom[off(b"geometry", b"tiles_touched"):][:4 * P].view(torch.int32).cpu().numpy()
fs = geom[off(b"geometry", b"first_slot"):][:4 * P].view(torch.int32).cpu().numpy()
fl = binning[off(b"binning", b"rec_flags"):][:4 * K].cpu().numpy().reshape(K, 4) != 0
live = touched & (radii.cpu().numpy() > 0)
n = tt[live]
recs = np.array([fl[f:f + c].sum() for f, c in zip(fs[live], n)])
print("K", K, "visible", int((radii > 0).sum()), "live", int(live.sum()))
for name, v in (("tiles_touched(live)", n), ("records(live)", recs), ("tiles_touched(all vis)", tt[tt > 0])):
    print(name, "mean %.2f" % v.mean(), "p50", np.percentile(v, 50), "p90", np.percentile(v, 90),
          "p99", np.percentile(v, 99), "max", v.max())
# per 2048-Gaussian group (one k_gauss_bwd_live block): live count and max n
grp = np.arange(P)[live] // 2048
for q in (50, 90, 99, 100):
    pass
cnt = np.bincount(grp, minlength=(P + 2047) // 2048)
mx = np.zeros_like(cnt)
np.maximum.at(mx, grp, n)
print("per block: live mean %.1f max %d; max n per block p50 %d p90 %d max %d" %
      (cnt.mean(), cnt.max(), np.percentile(mx, 50), np.percentile(mx, 90), mx.max()))

# records whose nine sums are all zero (kept by the quadrant cull, no pixel contributed)
roff = off(b"binning", b"records")
rec = binning[roff:roff + 4 * K * 48].view(torch.float32).view(4 * K, 12)
flags = binning[off(b"binning", b"rec_flags"):][:4 * K] != 0
r = rec[flags]
nz = (r[:, :9].abs().sum(dim=1) != 0)
print("records", int(flags.sum()), "all-zero", int((~nz).sum()), "frac %.3f" % float((~nz).float().mean()))
