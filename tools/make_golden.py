#!/usr/bin/env python
"""Generate the committed golden fixtures under tests/golden/.

  sh_eval_ref.npz   inputs/outputs of the REFERENCE's own eval_sh
                    (gaussiansplatting/utils/sh_utils.py:57-112), imported read-only
                    from /root/reference with bytecode writing disabled.  Pins the
                    oracle's and the kernels' SH->RGB (forward.cu:20-71 restates it).
  cameras_ref.npz   the REFERENCE's getWorld2View2 / getProjectionMatrix outputs (and the
                    Simple_Camera composition) for the c1-c5 cameras and random poses, generated
                    in round 2 from the reference functions; now checked against restatements
                    (camera_fixture), which no longer import the reference.
  lr_schedule_ref.npz  the REFERENCE's get_expon_lr_func schedules (the optimizer's position
                    learning rate, gaussian_model.py:373-380) and inverse_sigmoid
                    (gaussiansplatting/utils/general_utils.py:18-19, 29-62), imported read-only.
  multiview_3views.npz  the oracle's 3-view step reductions (summed parameter and view-space
                    gradients, max radii) for the F1 multi-view step test.
  scene_*.npz       seeded scenes (inputs) with the oracle's outputs and gradients:
                    the GPU parity tests compare the HIP path against them.

Only data is written (no reference source).  Run from the repo root:
    python tools/make_golden.py            (all fixtures)
    python tools/make_golden.py lr sh ...  (only those)
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OUT = os.path.join(ROOT, "tests", "golden")


def sh_fixture():
    sys.dont_write_bytecode = True
    sys.path.insert(0, "/root/reference")
    from gaussiansplatting.utils.sh_utils import eval_sh  # the reference function itself

    g = torch.Generator().manual_seed(7)
    N = 512
    sh = torch.randn(N, 3, 16, generator=g)
    d = torch.randn(N, 3, generator=g)
    d = d / d.norm(dim=1, keepdim=True)
    out = {"sh": sh.numpy(), "dirs": d.numpy()}
    for deg in range(4):
        out[f"rgb_deg{deg}"] = eval_sh(deg, sh, d).numpy()
    np.savez_compressed(os.path.join(OUT, "sh_eval_ref.npz"), **out)
    sys.path.remove("/root/reference")


def _world_to_view(R, t, translate, scale):
    """graphics_utils.py:40-51 (getWorld2View2) restated: the camera-to-world inverse of [R^T | t],
    its centre moved by `translate` and scaled, inverted back; float32 like the reference."""
    w2c = np.eye(4)
    w2c[:3, :3] = np.asarray(R).T
    w2c[:3, 3] = t
    c2w = np.linalg.inv(w2c)
    c2w[:3, 3] = (c2w[:3, 3] + translate) * scale
    return np.float32(np.linalg.inv(c2w))


def _projection(znear, zfar, fovx, fovy):
    """graphics_utils.py:67-87 (getProjectionMatrix) restated: a symmetric frustum (left = -right,
    bottom = -top), z_sign = +1, built in float32 like the reference's torch.zeros(4, 4)."""
    import math

    tx, ty = math.tan(fovx / 2), math.tan(fovy / 2)
    top, right = ty * znear, tx * znear
    P = torch.zeros(4, 4, dtype=torch.float32)
    P[0, 0] = 2.0 * znear / (right - -right)
    P[1, 1] = 2.0 * znear / (top - -top)
    P[0, 2] = (right + -right) / (right - -right)
    P[1, 2] = (top + -top) / (top - -top)
    P[3, 2] = 1.0
    P[2, 2] = zfar / (zfar - znear)
    P[2, 3] = -(zfar * znear) / (zfar - znear)
    return P


def camera_fixture(write: bool = False):
    """cameras_ref.npz holds the REFERENCE's camera matrices (graphics_utils.py:40-51 getWorld2View2,
    :67-87 getProjectionMatrix) and the Simple_Camera composition (scene/cameras.py:90-94) for the
    c1-c5 orbit cameras and seeded random poses with trans/scale — generated in round 2 by calling the
    reference functions themselves.  This tool no longer imports the reference: it recomputes the
    fixture with the restatements above and checks it against the committed file, element for element
    (write=True — `python tools/make_golden.py cameras-write` — rewrites it from them instead)."""
    import math

    from dge_amd.cameras import look_at_R_T

    cams = []
    for (k, n, W, H) in [(0, 1, 256, 256), (0, 1, 512, 512), (5, 24, 512, 512), (17, 24, 512, 512),
                         (0, 1, 1920, 1080)]:
        az, el = 2.0 * math.pi * k / n, math.radians(15.0)
        pos = 5.0 * np.array([math.cos(el) * math.cos(az), math.cos(el) * math.sin(az), math.sin(el)])
        R, T = look_at_R_T(pos)
        fx = math.radians(60.0)
        cams.append((R, T, np.zeros(3), 1.0, fx, 2.0 * math.atan(math.tan(fx / 2) * H / W)))
    rng = np.random.default_rng(3)
    for _ in range(4):
        q = rng.standard_normal(4)
        q /= np.linalg.norm(q)
        w, x, y, z = q
        R = np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - w * z), 2 * (x * z + w * y)],
                      [2 * (x * y + w * z), 1 - 2 * (x * x + z * z), 2 * (y * z - w * x)],
                      [2 * (x * z - w * y), 2 * (y * z + w * x), 1 - 2 * (x * x + y * y)]])
        cams.append((R, rng.uniform(-3, 3, 3), rng.uniform(-1, 1, 3), float(rng.uniform(0.5, 2.0)),
                     float(rng.uniform(0.6, 1.6)), float(rng.uniform(0.6, 1.6))))
    out = {"n": len(cams)}
    for i, (R, T, trans, scale, fovx, fovy) in enumerate(cams):
        w2v = _world_to_view(R, T, trans, scale)
        proj = _projection(0.01, 100.0, fovx, fovy)
        wv = torch.tensor(w2v).transpose(0, 1)
        pt = proj.transpose(0, 1)
        full = wv.unsqueeze(0).bmm(pt.unsqueeze(0)).squeeze(0).float()
        out.update({f"R{i}": R, f"T{i}": T, f"trans{i}": trans, f"scale{i}": scale, f"fovx{i}": fovx,
                    f"fovy{i}": fovy, f"w2v{i}": w2v, f"proj{i}": proj.numpy(),
                    f"world_view{i}": wv.numpy(), f"full_proj{i}": full.numpy(),
                    f"center{i}": wv.inverse()[3, :3].numpy()})
    path = os.path.join(OUT, "cameras_ref.npz")
    if write or not os.path.exists(path):
        np.savez_compressed(path, **out)
        print("cameras written", len(cams))
        return
    ref = np.load(path)
    bad = [k for k in out if not np.array_equal(np.asarray(out[k]), ref[k])]
    assert not bad, f"restated camera matrices differ from the reference's fixture: {bad}"
    print("cameras: restatement equals the committed reference fixture,", len(cams), "cameras")


def scene_fixture(name, P, W, H, seed, radius=1.5, scale=0.05, sh_degree=3, bg=(0.0, 0.0, 0.0), mode="sh",
                  scale_modifier=1.0, view=0, nviews=1):
    from oracle import oracle as O
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import _settings
    from dge_amd.scene import synthetic_scene

    sc = synthetic_scene(P, sh_degree=sh_degree, seed=seed, radius=radius, scale=scale)
    cam = orbit_camera(view, nviews, W, H, device="cpu")
    s = _settings(cam, torch.tensor(bg, dtype=torch.float32), scale_modifier, sh_degree)
    with torch.no_grad():
        xyz, op = sc.get_xyz.numpy(), sc.get_opacity.numpy()
        shs, scl, rot = sc.get_features.numpy(), sc.get_scaling.numpy(), sc.get_rotation.numpy()
        cov = sc.get_covariance(scale_modifier).numpy()
    g = np.random.default_rng(seed + 100).standard_normal((3, H, W)).astype(np.float32) * 1e-2
    kw = dict(shs=shs, scales=scl, rotations=rot)
    colors = None
    if mode == "colors":
        colors = np.random.default_rng(seed + 5).random((P, 3)).astype(np.float32)
        kw = dict(colors_precomp=colors, scales=scl, rotations=rot)
    elif mode == "cov3d":
        kw = dict(shs=shs, cov3D_precomp=cov)
    nr, color, depth, radii, st = O.forward(s, xyz, op, **kw)
    grads = O.backward(st, g)
    rec = dict(
        P=P, W=W, H=H, sh_degree=sh_degree, mode=mode, scale_modifier=scale_modifier,
        tanfovx=s.tanfovx, tanfovy=s.tanfovy, bg=np.asarray(bg, np.float32),
        viewmatrix=s.viewmatrix.numpy(), projmatrix=s.projmatrix.numpy(), campos=s.campos.numpy(),
        means3D=xyz, opacities=op, shs=shs, scales=scl, rotations=rot, cov3D=cov,
        colors=colors if colors is not None else np.zeros((0, 3), np.float32), dL_dpix=g,
        num_rendered=nr, color=color, depth=depth, radii=radii,
        n_contrib=st.get("n_contrib"), final_T=st.get("final_T"), point_list=st.get("point_list"),
        ranges=st.get("ranges"), means2D=st.get("means2D"), conic_opacity=st.get("conic_opacity"),
        rgb=st.get("rgb"), depths=st.get("depths"), tiles_touched=st.get("tiles_touched"),
        clamped=st.get("clamped"),
        **grads)
    np.savez_compressed(os.path.join(OUT, f"scene_{name}.npz"), **rec)
    print(name, "P", P, "K", nr, "bytes", os.path.getsize(os.path.join(OUT, f"scene_{name}.npz")))


def multiview_fixture():
    """F1: DGE's per-step reductions over a 3-view batch, from the oracle: the
    parameter gradients summed over the views (one backward of the summed loss, DGE.py:617-699), the
    view-space gradient sum and the radii max (DGE.py:190-193, 269-281), with each view's oracle
    magnitudes (mag9) summed for the view-space tolerance."""
    from oracle import oracle as O
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import _settings
    from dge_amd.scene import synthetic_scene

    P, W, H, V = 2500, 112, 96, 3
    sc = synthetic_scene(P, sh_degree=3, seed=21, radius=1.5, scale=0.04)
    with torch.no_grad():
        kw = dict(shs=sc.get_features.numpy(), scales=sc.get_scaling.numpy(), rotations=sc.get_rotation.numpy())
        xyz, op = sc.get_xyz.numpy(), sc.get_opacity.numpy()
    rng = np.random.default_rng(31)
    acc = {k: np.zeros(v.shape, np.float64) for k, v in dict(means3D=xyz, opacity=op, sh=kw["shs"],
                                                              scales=kw["scales"], rotations=kw["rotations"]).items()}
    vs = np.zeros((P, 3), np.float64)
    mag = np.zeros((P, 9), np.float64)
    rmax = np.zeros(P, np.int32)
    seeds = []
    for k in range(V):
        s = _settings(orbit_camera(k, V, W, H, device="cpu"), torch.zeros(3), 1.0, 3)
        g = (rng.standard_normal((3, H, W)) * 1e-2).astype(np.float32)
        seeds.append(g)
        nr, color, depth, radii, st = O.forward(s, xyz, op, **kw)
        gr = O.backward(st, g)
        acc["means3D"] += gr["dL_dmeans3D"]
        acc["opacity"] += gr["dL_dopacity"]
        acc["sh"] += gr["dL_dsh"]
        acc["scales"] += gr["dL_dscales"]
        acc["rotations"] += gr["dL_drotations"]
        vs += gr["dL_dmeans2D"]
        mag += gr["mag9"]
        rmax = np.maximum(rmax, radii)
    rec = dict(P=P, W=W, H=H, V=V, means3D=xyz, opacities=op, **kw, dL_dpix=np.stack(seeds),
               viewspace_grad_sum=vs.astype(np.float32), mag9_sum=mag.astype(np.float32), radii_max=rmax,
               **{f"dL_d{k}_sum": v.astype(np.float32) for k, v in acc.items()})
    np.savez_compressed(os.path.join(OUT, "multiview_3views.npz"), **rec)
    print("multiview_3views", os.path.getsize(os.path.join(OUT, "multiview_3views.npz")))


# (lr_init, lr_final, lr_delay_steps, lr_delay_mult, max_steps): DGE's position schedule (the optimizer
# defaults of arguments/__init__.py:71-89 x spatial_lr_scale, gaussian_model.py:373-380), a delayed one,
# a disabled one (both rates 0) and a short one
LR_CASES = [(0.00016 * 2.5, 0.000016 * 2.5, 0, 0.01, 30_000), (1e-3, 1e-5, 500, 0.01, 10_000),
            (0.0, 0.0, 0, 1.0, 1000), (5e-2, 5e-4, 10, 0.1, 100)]
LR_STEPS = [-1, 0, 1, 2, 5, 9, 10, 11, 50, 99, 100, 101, 499, 500, 501, 1000, 5000, 9999, 10000, 10001, 15000,
            29_999, 30_000, 30_001, 100_000]


def lr_fixture():
    sys.dont_write_bytecode = True
    sys.path.insert(0, "/root/reference")
    from gaussiansplatting.utils.general_utils import get_expon_lr_func, inverse_sigmoid  # the reference's own

    out = {"cases": np.array(LR_CASES, dtype=np.float64), "steps": np.array(LR_STEPS, dtype=np.int64)}
    for i, c in enumerate(LR_CASES):
        f = get_expon_lr_func(lr_init=c[0], lr_final=c[1], lr_delay_steps=int(c[2]), lr_delay_mult=c[3],
                              max_steps=int(c[4]))
        out[f"lr_{i}"] = np.array([float(f(s)) for s in LR_STEPS], dtype=np.float64)
    x = torch.linspace(0.001, 0.999, 257)
    out["inv_sigmoid_x"] = x.numpy()
    out["inv_sigmoid"] = inverse_sigmoid(x).numpy()
    np.savez_compressed(os.path.join(OUT, "lr_schedule_ref.npz"), **out)
    sys.path.remove("/root/reference")


FIXTURES = {
    "sh": sh_fixture,
    "cameras": camera_fixture,
    "cameras-write": lambda: camera_fixture(write=True),
    "lr": lr_fixture,
    "scenes": lambda: [
        scene_fixture("sh3_96x80", 1500, 96, 80, seed=11),
        scene_fixture("sh1_bg_64", 800, 64, 64, seed=12, sh_degree=1, bg=(0.2, 0.5, 0.9), scale=0.08),
        scene_fixture("colors_120x72", 1000, 120, 72, seed=13, mode="colors", scale=0.06, view=1, nviews=3),
        scene_fixture("cov3d_mod_80", 900, 80, 80, seed=14, mode="cov3d", scale_modifier=0.8, scale=0.07)],
    "multiview": lambda: multiview_fixture(),
}


def main():
    os.makedirs(OUT, exist_ok=True)
    for name in sys.argv[1:] or list(FIXTURES):
        FIXTURES[name]()


if __name__ == "__main__":
    main()
