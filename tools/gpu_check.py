"""Quick end-to-end check: HIP path vs oracle on a small scene (dev tool)."""
import sys, time, os
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O
from dge_amd.scene import synthetic_scene
from dge_amd.cameras import orbit_camera
from dge_amd.gaussian_renderer import _settings
from dge_amd import _C

def rel(a, b, floor=1e-6):
    a = np.asarray(a, np.float64); b = np.asarray(b, np.float64)
    return float(np.max(np.abs(a - b) / np.maximum(np.maximum(np.abs(a), np.abs(b)), floor))) if a.size else 0.0

def main(P=10000, W=256, H=256):
    dev = 'cuda'
    sc = synthetic_scene(P, device='cpu')
    cam = orbit_camera(0, 1, W, H, device='cpu')
    s = _settings(cam, torch.zeros(3), 1.0, 3)
    xyz, op, sh, scl, rot = sc.get_xyz, sc.get_opacity, sc.get_features, sc.get_scaling, sc.get_rotation
    nr, color, depth, radii, st = O.forward(s, xyz, op, shs=sh, scales=scl, rotations=rot)
    g = np.random.default_rng(1).standard_normal((3, H, W)).astype(np.float32) * 1e-3
    og = O.backward(st, g)
    camd = orbit_camera(0, 1, W, H, device=dev)
    bg = torch.zeros(3, device=dev)
    args = (bg, xyz.to(dev), torch.empty(0, device=dev), op.to(dev), scl.to(dev), rot.to(dev), 1.0, torch.empty(0, device=dev),
            camd.world_view_transform, camd.full_proj_transform, s.tanfovx, s.tanfovy, H, W, sh.to(dev), 3, camd.camera_center, False, True)
    K, c2, d2, r2, geom, binning, img = _C.rasterize_gaussians(*args)
    torch.cuda.synchronize()
    print('K', K, nr, 'radii equal', bool((r2.cpu().numpy() == radii).all()))
    print('color maxabs', float((c2.cpu() - torch.from_numpy(color)).abs().max()), 'depth', float((d2.cpu() - torch.from_numpy(depth)).abs().max()))
    gr = _C.rasterize_gaussians_backward(bg, xyz.to(dev), r2, torch.empty(0, device=dev), scl.to(dev), rot.to(dev), 1.0, torch.empty(0, device=dev),
            camd.world_view_transform, camd.full_proj_transform, s.tanfovx, s.tanfovy, torch.from_numpy(g).to(dev), sh.to(dev), 3, camd.camera_center,
            geom, K, binning, img, True)
    torch.cuda.synchronize()
    names = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales", "dL_drotations"]
    for n, t in zip(names, gr):
        a = t.cpu().numpy(); b = og[n]
        print(n, 'maxabs', float(np.abs(a - b).max()), 'ref max', float(np.abs(b).max()), 'rel(floor=1e-3*max)', rel(a, b, 1e-3 * float(np.abs(b).max()) + 1e-12))

if __name__ == '__main__':
    main(*[int(x) for x in sys.argv[1:]])
