"""Blend-exp A/B (dev probe, GPU): the forward of the in-tree library (DGE_AMD_LIB picks another build, e.g.
dge_amd/lib/var/hwexp.so built with -DGS_HW_EXP: v_exp_f32) against the oracle at c2 and c4: pixels whose
n_contrib differs (a skip / stop decision of the blend flipped), image elements that differ and by how much, and
the backward's rasterizer sums against the oracle's (max err / (1e-4 x magnitude)).  One JSON line per config."""
import json
import os
import sys

import numpy as np
import torch

root = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, root)
sys.path.insert(0, os.path.join(root, "tests"))
from helpers import camera_settings, raster_grad_mismatches, run_gpu, run_oracle, scene_arrays  # noqa: E402
from oracle import oracle as O  # noqa: E402

O.build()
O.set_threads(16)
for name, P, W, H, bwd in (("c2", 1_000_000, 512, 512, True), ("c4", 2_500_000, 1920, 1080, False)):
    a = scene_arrays(P, seed=0 if name == "c2" else 2, radius=2.0, scale=0.02)
    kw = dict(means3D=a["means3D"], opacities=a["opacities"], shs=a["shs"], scales=a["scales"],
              rotations=a["rotations"])
    g = np.random.default_rng(1).standard_normal((3, H, W)).astype(np.float32) * 1e-3 if bwd else None
    ref = run_oracle(O, camera_settings(W, H), g, **kw)
    got = run_gpu(camera_settings(W, H, device="cuda"), g, **kw)
    nc = got["n_contrib"].reshape(-1) != ref["n_contrib"].reshape(-1)
    dc = np.abs(got["color"] - ref["color"])
    rec = {"config": name, "lib": os.environ.get("DGE_AMD_LIB") or "in-tree", "pixels": int(W * H),
           "n_contrib_flips": int(nc.sum()), "color_elements_differ": int((dc > 0).sum()),
           "color_max_abs_diff": float(dc.max()), "color_max": float(np.abs(ref["color"]).max()),
           "final_T_differ": int((got["final_T"] != ref["final_T"]).sum())}
    if bwd:
        rec["raster_sums_max_err_over_1e-4_mag"] = {k: round(v[1], 4) for k, v in raster_grad_mismatches(got, ref).items()}
    print(json.dumps(rec), flush=True)
