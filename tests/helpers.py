"""Shared helpers: scene/settings construction, the parity metric, and a
driver that runs the HIP path through the C ABI and extracts intermediates.

Parity metric (north_star: "within 1e-4 relative fp32"): for a tensor pair
(got, ref), |got - ref| <= rtol * (|ref| + max|ref|) element-wise, i.e.
1e-4 relative for large elements and 1e-4 of the tensor's scale for small
ones (gradient sums differ only in summation order).  Integer/index outputs
(radii, num_rendered, tiles_touched, point lists, ranges) must be identical.
"""
from __future__ import annotations

import math
from types import SimpleNamespace

import numpy as np
import torch

RTOL = 1e-4
GRAD_NAMES = ["dL_dmeans2D", "dL_dcolors", "dL_dopacity", "dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales",
              "dL_drotations"]


def close_report(got, ref, rtol=RTOL):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    if ref.size == 0:
        return 0.0, 0.0
    scale = float(np.abs(ref).max())
    err = np.abs(got - ref)
    tol = rtol * (np.abs(ref) + scale) + 1e-30
    return float((err / tol).max()), float(err.max() / max(scale, 1e-30))


def assert_close(got, ref, name, rtol=RTOL, allow_frac=0.0):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    assert got.shape == ref.shape, f"{name}: shape {got.shape} vs {ref.shape}"
    if ref.size == 0:
        return
    scale = float(np.abs(ref).max())
    tol = rtol * (np.abs(ref) + scale)
    bad = np.abs(got - ref) > tol
    nbad = int(bad.sum())
    if nbad > allow_frac * ref.size:
        i = np.unravel_index(np.argmax(np.abs(got - ref) - tol), ref.shape)
        raise AssertionError(f"{name}: {nbad}/{ref.size} elements beyond {rtol} rel (scale {scale:.3e}); "
                             f"worst at {i}: got {got[i]!r} ref {ref[i]!r}")


def settings_from(W, H, tanfovx, tanfovy, bg, viewmatrix, projmatrix, campos, sh_degree, scale_modifier=1.0,
                  prefiltered=False, debug=False, device="cpu"):
    t = lambda a: torch.as_tensor(np.asarray(a, np.float32)).to(device)
    return SimpleNamespace(image_height=H, image_width=W, tanfovx=float(tanfovx), tanfovy=float(tanfovy), bg=t(bg),
                           scale_modifier=float(scale_modifier), viewmatrix=t(viewmatrix).reshape(4, 4),
                           projmatrix=t(projmatrix).reshape(4, 4), sh_degree=int(sh_degree), campos=t(campos),
                           prefiltered=prefiltered, debug=debug)


def settings_from_golden(rec, device="cpu"):
    return settings_from(int(rec["W"]), int(rec["H"]), float(rec["tanfovx"]), float(rec["tanfovy"]), rec["bg"],
                         rec["viewmatrix"], rec["projmatrix"], rec["campos"], int(rec["sh_degree"]),
                         float(rec["scale_modifier"]), device=device)


def golden_inputs(rec):
    mode = str(rec["mode"])
    kw = dict(means3D=rec["means3D"], opacities=rec["opacities"])
    if mode == "sh":
        kw.update(shs=rec["shs"], scales=rec["scales"], rotations=rec["rotations"])
    elif mode == "colors":
        kw.update(colors_precomp=rec["colors"], scales=rec["scales"], rotations=rec["rotations"])
    elif mode == "cov3d":
        kw.update(shs=rec["shs"], cov3D_precomp=rec["cov3D"])
    return kw


def camera_settings(W, H, fovx_deg=60.0, bg=(0.0, 0.0, 0.0), sh_degree=3, view=0, nviews=1, distance=5.0,
                    device="cpu", scale_modifier=1.0):
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import _settings

    cam = orbit_camera(view, nviews, W, H, distance=distance, fovx_deg=fovx_deg, device=device)
    return _settings(cam, torch.tensor(bg, dtype=torch.float32, device=device), scale_modifier, sh_degree)


def scene_arrays(P, seed=0, sh_degree=3, radius=1.5, scale=0.05):
    from dge_amd.scene import synthetic_scene

    sc = synthetic_scene(P, sh_degree=sh_degree, seed=seed, radius=radius, scale=scale)
    with torch.no_grad():
        return dict(means3D=sc.get_xyz.numpy(), opacities=sc.get_opacity.numpy(), shs=sc.get_features.numpy(),
                    scales=sc.get_scaling.numpy(), rotations=sc.get_rotation.numpy(),
                    cov3D=sc.get_covariance().numpy())


# ---------------------------------------------------------------------------
# GPU driver (C ABI through dge_amd._C) + intermediates
# ---------------------------------------------------------------------------
def run_gpu(settings, dL_dpix=None, means3D=None, opacities=None, shs=None, colors_precomp=None, scales=None,
            rotations=None, cov3D_precomp=None, device="cuda", intermediates=True):
    from dge_amd import _C, _native

    dev = torch.device(device)
    T = lambda a: torch.empty(0, device=dev) if a is None else torch.as_tensor(np.asarray(a, np.float32)).to(dev)
    s = settings
    m = T(means3D)
    P = m.shape[0]
    H, W = int(s.image_height), int(s.image_width)
    fw = _C.rasterize_gaussians(s.bg.to(dev), m, T(colors_precomp), T(opacities), T(scales), T(rotations),
                                float(s.scale_modifier), T(cov3D_precomp), s.viewmatrix.to(dev), s.projmatrix.to(dev),
                                s.tanfovx, s.tanfovy, H, W, T(shs), int(s.sh_degree), s.campos.to(dev),
                                bool(s.prefiltered), bool(s.debug))
    K, color, depth, radii, geom, binning, img = fw
    torch.cuda.synchronize()
    out = dict(num_rendered=K, color=color.cpu().numpy(), depth=depth.cpu().numpy(), radii=radii.cpu().numpy())
    if intermediates and P > 0:
        L = _native.lib()

        def view(buf, which, field, dtype, count):
            off = L.gs_buffer_offset(which.encode(), field.encode(), P, W, H, K)
            assert off >= 0, field
            nbytes = np.dtype(dtype).itemsize * count
            return buf[off:off + nbytes].cpu().numpy().view(dtype).copy()

        tiles = ((W + 15) // 16) * ((H + 15) // 16)
        sp = view(geom, "geometry", "splat", np.float32, 16 * P).reshape(P, 16)  # 64-B records
        out["means2D"] = np.ascontiguousarray(sp[:, 0:2])
        out["conic_opacity"] = np.ascontiguousarray(sp[:, 4:8])
        out["rgbd"] = np.ascontiguousarray(sp[:, 8:12])
        out["tiles_touched"] = view(geom, "geometry", "tiles_touched", np.uint32, P)
        out["clamped"] = view(geom, "geometry", "clamped", np.uint8, P)
        out["final_T"] = view(img, "image", "final_T", np.float32, W * H)
        out["n_contrib"] = view(img, "image", "n_contrib", np.uint32, W * H)
        out["ranges"] = view(img, "image", "ranges", np.uint32, 2 * tiles)
        # per-tile lists: (Gaussian, slot) pairs; the Gaussian ids are the reference's point_list
        out["point_list"] = view(binning, "binning", "point_pairs", np.uint32, 2 * K)[0::2] if K else np.zeros(0, np.uint32)
    if dL_dpix is not None:
        g = torch.as_tensor(np.asarray(dL_dpix, np.float32)).to(dev)
        grads = _C.rasterize_gaussians_backward(s.bg.to(dev), m, radii, T(colors_precomp), T(scales), T(rotations),
                                                float(s.scale_modifier), T(cov3D_precomp), s.viewmatrix.to(dev),
                                                s.projmatrix.to(dev), s.tanfovx, s.tanfovy, g, T(shs),
                                                int(s.sh_degree), s.campos.to(dev), geom, K, binning, img,
                                                bool(s.debug))
        torch.cuda.synchronize()
        for n, t in zip(GRAD_NAMES, grads):
            out[n] = t.cpu().numpy()
    return out


def run_oracle(O, settings, dL_dpix=None, **kw):
    nr, color, depth, radii, st = O.forward(settings, **kw)
    out = dict(num_rendered=nr, color=color, depth=depth, radii=radii)
    for k in ("means2D", "conic_opacity", "rgb", "depths", "tiles_touched", "clamped", "final_T", "n_contrib",
              "ranges", "point_list"):
        out[k] = st.get(k)
    if dL_dpix is not None:
        out.update(O.backward(st, dL_dpix))
    return out


def compare_forward(got, ref, rtol=RTOL, allow_flip_frac=0.0, strict_lists=True, check_rgb=True):
    """HIP vs oracle forward, field by field."""
    assert got["num_rendered"] == ref["num_rendered"], (got["num_rendered"], ref["num_rendered"])
    np.testing.assert_array_equal(got["radii"], ref["radii"])
    vis = ref["radii"] > 0
    P = vis.shape[0]
    if P:
        np.testing.assert_array_equal(got["tiles_touched"], ref["tiles_touched"])
        assert_close(got["means2D"][vis], ref["means2D"].reshape(P, 2)[vis], "means2D", rtol)
        assert_close(got["conic_opacity"][vis], ref["conic_opacity"].reshape(P, 4)[vis], "conic_opacity", rtol)
        assert_close(got["rgbd"][vis, 3], ref["depths"][vis], "depth (per Gaussian)", rtol)
        if check_rgb and "rgb" in ref and "rgbd" in got:
            assert_close(got["rgbd"][vis, :3], ref["rgb"].reshape(P, 3)[vis], "rgb", rtol)
            cl = ref["clamped"].reshape(P, 3)
            bits = (cl[:, 0] | (cl[:, 1] << 1) | (cl[:, 2] << 2)).astype(np.uint8)
            np.testing.assert_array_equal(got["clamped"][vis], bits[vis])
        np.testing.assert_array_equal(got["ranges"], ref["ranges"])
        if strict_lists:
            np.testing.assert_array_equal(got["point_list"], ref["point_list"])
    assert_close(got["color"], ref["color"], "color", rtol, allow_flip_frac)
    assert_close(got["depth"], ref["depth"], "depth", rtol, allow_flip_frac)
    if P:
        assert_close(got["final_T"], ref["final_T"], "final_T", rtol, allow_flip_frac)
        mism = float(np.mean(got["n_contrib"] != ref["n_contrib"]))
        assert mism <= allow_flip_frac, f"n_contrib mismatch fraction {mism}"


def compare_grads(got, ref, rtol=RTOL, allow_frac=0.0):
    for n in GRAD_NAMES:
        assert_close(got[n], ref[n], n, rtol, allow_frac)
