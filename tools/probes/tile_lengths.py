"""c2 scene statistics (dev probe, GPU): visible Gaussians, tile list lengths."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from dge_amd import _C, _native  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import _settings  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

dev = torch.device("cuda", 0)
for P, W, H, name in ((1_000_000, 512, 512, "c2"), (2_500_000, 1920, 1080, "c4")):
    sc = synthetic_scene(P, seed=0 if name == "c2" else 2, device=dev)
    s = _settings(orbit_camera(0, 1, W, H, device=dev), torch.zeros(3, device=dev), 1.0, 3)
    shs = torch.cat([sc._features_dc, sc._features_rest], 1).contiguous()
    fw = _C.rasterize_gaussians(s.bg, sc._xyz, torch.empty(0, device=dev), torch.sigmoid(sc._opacity),
                                torch.exp(sc._scaling), torch.nn.functional.normalize(sc._rotation), 1.0,
                                torch.empty(0, device=dev), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, H, W,
                                shs, 3, s.campos, False, False)
    K, color, depth, radii, geom, binning, img = fw
    torch.cuda.synchronize()
    L = _native.lib()
    off = L.gs_buffer_offset(b"image", b"ranges", P, W, H, K)
    tiles = ((W + 15) // 16) * ((H + 15) // 16)
    r = img[off:off + 8 * tiles].cpu().numpy().view(np.uint32).reshape(-1, 2)
    n = (r[:, 1] - r[:, 0]).astype(np.int64)
    vis = int((radii > 0).sum())
    q = np.percentile(n, [50, 90, 99, 100])
    print(f"{name}: P={P} visible={vis} ({vis / P:.2%}) K={K} tiles={tiles} list len p50/p90/p99/max={q} "
          f"frac>4096={np.mean(n > 4096):.3f} entries in lists>4096={n[n > 4096].sum() / max(K, 1):.3f}")
