#!/usr/bin/env python
"""Generate the committed golden fixtures under tests/golden/.

  sh_eval_ref.npz   inputs/outputs of the REFERENCE's own eval_sh
                    (gaussiansplatting/utils/sh_utils.py:57-112), imported read-only
                    from /root/reference with bytecode writing disabled.  Pins the
                    oracle's and the kernels' SH->RGB (forward.cu:20-71 restates it).
  scene_*.npz       seeded scenes (inputs) with the oracle's outputs and gradients:
                    the GPU parity tests compare the HIP path against them.

Only data is written (no reference source).  Run from the repo root:
    python tools/make_golden.py
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


def main():
    os.makedirs(OUT, exist_ok=True)
    sh_fixture()
    scene_fixture("sh3_96x80", 1500, 96, 80, seed=11)
    scene_fixture("sh1_bg_64", 800, 64, 64, seed=12, sh_degree=1, bg=(0.2, 0.5, 0.9), scale=0.08)
    scene_fixture("colors_120x72", 1000, 120, 72, seed=13, mode="colors", scale=0.06, view=1, nviews=3)
    scene_fixture("cov3d_mod_80", 900, 80, 80, seed=14, mode="cov3d", scale_modifier=0.8, scale=0.07)


if __name__ == "__main__":
    main()
