"""CPU tests of the host-side logic around the kernels: camera matrices,
the GaussianModel-compatible getters, the Python wrapper's argument checks."""
from __future__ import annotations

import math

import numpy as np
import pytest
import torch

from dge_amd import cameras as C
from dge_amd.diff_gaussian_rasterization import GaussianRasterizationSettings, GaussianRasterizer
from dge_amd.scene import build_covariance, synthetic_scene


def test_projection_matrix_known_answer():
    # graphics_utils.py:67-87 with symmetric frustum: P[0,0] = 1/tan(fovx/2), P[1,1] = 1/tan(fovy/2)
    P = C.get_projection_matrix(0.01, 100.0, math.radians(60), math.radians(50)).numpy()
    assert abs(P[0, 0] - 1 / math.tan(math.radians(30))) < 1e-6
    assert abs(P[1, 1] - 1 / math.tan(math.radians(25))) < 1e-6
    assert P[3, 2] == 1.0 and abs(P[2, 2] - 100 / 99.99) < 1e-6 and abs(P[2, 3] + 1.0 / 99.99) < 1e-6
    assert P[0, 2] == 0 and P[1, 2] == 0 and P[3, 3] == 0


def test_world2view_and_camera_center():
    R, T = C.look_at_R_T([3.0, -4.0, 2.0])
    Wv = C.get_world2view2(R, T)
    np.testing.assert_allclose(Wv[:3, :3] @ Wv[:3, :3].T, np.eye(3), atol=1e-6)
    cam = C.Camera(R, T, math.radians(60), math.radians(60), 64, 64, device="cpu")
    np.testing.assert_allclose(cam.camera_center.numpy(), [3.0, -4.0, 2.0], atol=1e-5)
    # the origin projects to the image centre (the camera looks at it)
    p = torch.tensor([0.0, 0.0, 0.0, 1.0]) @ cam.full_proj_transform
    assert abs(p[0] / p[3]) < 1e-6 and abs(p[1] / p[3]) < 1e-6 and p[3] > 0
    # view-space z of the origin is the distance
    v = torch.tensor([0.0, 0.0, 0.0, 1.0]) @ cam.world_view_transform
    assert abs(float(v[2]) - math.sqrt(29.0)) < 1e-4


def test_orbit_cameras_distinct_and_aimed():
    cams = [C.orbit_camera(k, 8, 64, 48, device="cpu") for k in range(8)]
    centers = np.stack([c.camera_center.numpy() for c in cams])
    assert np.allclose(np.linalg.norm(centers, axis=1), 5.0, atol=1e-4)
    assert len({tuple(np.round(c, 3)) for c in centers}) == 8
    assert abs(cams[0].FoVy - 2 * math.atan(math.tan(math.radians(30)) * 48 / 64)) < 1e-9


def test_scene_getters_follow_reference_activations():
    sc = synthetic_scene(64, seed=1)
    assert torch.allclose(sc.get_opacity, torch.sigmoid(sc._opacity))
    assert torch.allclose(sc.get_scaling, torch.exp(sc._scaling))
    assert torch.allclose(sc.get_rotation.norm(dim=1), torch.ones(64), atol=1e-6)
    assert sc.get_features.shape == (64, 16, 3)
    sc.localize, sc.mask = True, torch.arange(64) < 10
    assert sc.get_xyz.shape == (10, 3) and sc.get_features.shape == (10, 16, 3)


def test_build_covariance_matches_rasterizer_convention():
    import torch_ref as TR

    sc = synthetic_scene(32, seed=2)
    cov = build_covariance(sc.get_scaling, sc.get_rotation)
    # the dense reference builds Sigma = R diag(s)^2 R^T from the (normalised) quaternion
    q = sc.get_rotation.double()
    s = sc.get_scaling.double()
    r, x, y, z = q[:, 0], q[:, 1], q[:, 2], q[:, 3]
    R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                     2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                     2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1).reshape(-1, 3, 3)
    S = R @ torch.diag_embed(s * s) @ R.transpose(1, 2)
    ref = torch.stack([S[:, 0, 0], S[:, 0, 1], S[:, 0, 2], S[:, 1, 1], S[:, 1, 2], S[:, 2, 2]], -1)
    assert torch.allclose(cov.double(), ref, rtol=1e-5, atol=1e-9)
    assert TR is not None


def _rs():
    return GaussianRasterizationSettings(16, 16, 0.5, 0.5, torch.zeros(3), 1.0, torch.eye(4), torch.eye(4), 0,
                                         torch.zeros(3), False, False)


def test_wrapper_argument_checks_match_reference():
    r = GaussianRasterizer(_rs())
    m = torch.zeros(4, 3)
    with pytest.raises(Exception, match="excatly one of either SHs or precomputed colors"):
        r(m, m, torch.ones(4, 1))
    with pytest.raises(Exception, match="excatly one of either SHs or precomputed colors"):
        r(m, m, torch.ones(4, 1), shs=torch.zeros(4, 1, 3), colors_precomp=torch.zeros(4, 3))
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(m, m, torch.ones(4, 1), shs=torch.zeros(4, 1, 3))
    with pytest.raises(Exception, match="scale/rotation pair or precomputed 3D covariance"):
        r(m, m, torch.ones(4, 1), shs=torch.zeros(4, 1, 3), scales=torch.ones(4, 3), rotations=torch.ones(4, 4),
          cov3D_precomp=torch.zeros(4, 6))


def test_wrapper_rejects_bad_means_shape():
    from dge_amd import _C

    with pytest.raises(RuntimeError, match="means3D must have dimensions"):
        _C.rasterize_gaussians(torch.zeros(3), torch.zeros(4, 2), torch.empty(0), torch.ones(4, 1), torch.ones(4, 3),
                               torch.ones(4, 4), 1.0, torch.empty(0), torch.eye(4), torch.eye(4), 0.5, 0.5, 16, 16,
                               torch.zeros(4, 1, 3), 0, torch.zeros(3), False, False)


# ---- fused gradient accumulation: the decision rules (pure autograd, CPU) ----
def _modes_seen_in_backward(params, use_autograd_grad=False):
    """Run a backward through a probe Function and record _accumulation_mode of every param."""
    from dge_amd.diff_gaussian_rasterization import _accumulation_mode

    seen = {}

    class Probe(torch.autograd.Function):
        @staticmethod
        def forward(ctx, *xs):
            ctx.xs = xs
            return sum(x.sum() for x in xs)

        @staticmethod
        def backward(ctx, g):
            for i, x in enumerate(ctx.xs):
                seen[i] = _accumulation_mode(x)
            return tuple(torch.ones_like(x) for x in ctx.xs)

    out = Probe.apply(*params)
    if use_autograd_grad:
        torch.autograd.grad(out, params)
    else:
        out.backward()
    return [seen[i] for i in range(len(params))]


@pytest.mark.filterwarnings("ignore")
def test_fused_accum_modes():
    a = torch.zeros(4, requires_grad=True)
    b = torch.zeros(4, requires_grad=True)
    b.grad = torch.zeros(4)
    c = torch.zeros(4, requires_grad=True)
    c.register_hook(lambda g: g)  # hooked: autograd keeps the gradient
    d = torch.zeros(4, requires_grad=True)
    d.grad = torch.zeros(8)[::2]  # non-contiguous .grad
    modes = _modes_seen_in_backward([a, b, c, d])
    assert [m for m, _ in modes] == ["new", "add", None, None]
    assert all(o is None for _, o in modes)


def test_fused_accum_with_model_grad_mask_hooks():
    """GaussianModel.apply_grad_mask hooks (gaussian_model.py:837-856) keep the fused path: the mask is
    applied in-kernel; a foreign hook next to them still disables it."""
    from dge_amd.gaussian_model import GaussianModel

    m = GaussianModel(1, device="cpu")
    P = 5
    m.set_parameters(torch.zeros(P, 3), torch.zeros(P, 1, 3), torch.zeros(P, 3, 3), torch.zeros(P, 1),
                     torch.zeros(P, 3), torch.zeros(P, 4))
    modes = _modes_seen_in_backward(m.parameters())
    assert [md for md, _ in modes] == ["new"] * 6
    # _xyz, _features_dc, _features_rest, _opacity, _scaling carry the hook; _rotation does not
    assert [o is m for _, o in modes] == [True, True, True, True, True, False]
    m._xyz.grad = None
    m._xyz.register_hook(lambda g: g)
    (md, o), = _modes_seen_in_backward([m._xyz])
    assert md is None and o is None


def test_fused_accum_not_under_autograd_grad():
    a = torch.zeros(4, requires_grad=True)
    assert _modes_seen_in_backward([a], use_autograd_grad=True) == [(None, None)]


def test_fused_accum_toggle():
    from dge_amd.diff_gaussian_rasterization import set_fused_grad_accumulation

    prev = set_fused_grad_accumulation(False)
    assert set_fused_grad_accumulation(prev) is False


def test_camera_matrix_contiguous_cache():
    """Transposed camera matrices are made contiguous once per (tensor, version), not per call."""
    from dge_amd._C import _f32_cached

    base = torch.arange(16, dtype=torch.float32).reshape(4, 4)
    t = base.transpose(0, 1)
    a, b = _f32_cached(t, "viewmatrix"), _f32_cached(t, "viewmatrix")
    assert a is b and a.is_contiguous() and torch.equal(a, t)
    t.mul_(2)  # in-place edit bumps the version counter: a fresh copy
    c = _f32_cached(t, "viewmatrix")
    assert c is not a and torch.equal(c, t)
    u = torch.eye(4)
    assert _f32_cached(u, "projmatrix") is u  # contiguous input: no copy, no cache entry


def test_cameras_match_reference_graphics_utils():
    """dge_amd.cameras against the reference's own getWorld2View2 / getProjectionMatrix outputs
    (tests/golden/cameras_ref.npz, tools/make_golden.py camera_fixture): the c1-c5 orbit cameras and
    random poses with trans/scale — bit-identical matrices and camera centres."""
    import os

    from dge_amd.cameras import Camera, get_projection_matrix, get_world2view2

    rec = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "cameras_ref.npz"))
    n = int(rec["n"])
    assert n >= 9
    for i in range(n):
        R, T, tr, sc = rec[f"R{i}"], rec[f"T{i}"], rec[f"trans{i}"], float(rec[f"scale{i}"])
        fx, fy = float(rec[f"fovx{i}"]), float(rec[f"fovy{i}"])
        np.testing.assert_array_equal(get_world2view2(R, T, tr, sc), rec[f"w2v{i}"])
        np.testing.assert_array_equal(get_projection_matrix(0.01, 100.0, fx, fy).numpy(), rec[f"proj{i}"])
        cam = Camera(R, T, fx, fy, 64, 64, device="cpu", trans=tr, scale=sc)
        np.testing.assert_array_equal(cam.world_view_transform.numpy(), rec[f"world_view{i}"])
        np.testing.assert_array_equal(cam.full_proj_transform.numpy(), rec[f"full_proj{i}"])
        np.testing.assert_array_equal(cam.camera_center.numpy(), rec[f"center{i}"])


def test_install_alias_rebinds_reference_render(monkeypatch):
    """install_alias(fused_render=True): DGE's `from gaussiansplatting.gaussian_renderer import render`
    (threestudio/systems/DGE.py:15) ends up calling dge_amd's render, in the renderer module and in
    modules that imported the name before the call; the rasterizer package alias is installed too.
    (Stand-in modules with the reference's module names: the reference package is not importable here.)"""
    import sys
    import types

    import dge_amd
    from dge_amd import gaussian_renderer as ours

    def ref_render(*a, **k):
        raise AssertionError("reference render called")

    pkg = types.ModuleType("gaussiansplatting")
    rend = types.ModuleType("gaussiansplatting.gaussian_renderer")
    rend.render, rend.camera2rasterizer = ref_render, lambda *a, **k: None
    pkg.gaussian_renderer = rend
    system = types.ModuleType("threestudio_dge_standin")
    system.render = ref_render  # as `from gaussiansplatting.gaussian_renderer import render` leaves it
    for name, mod in (("gaussiansplatting", pkg), ("gaussiansplatting.gaussian_renderer", rend),
                      ("threestudio_dge_standin", system)):
        monkeypatch.setitem(sys.modules, name, mod)
    monkeypatch.delitem(sys.modules, "diff_gaussian_rasterization", raising=False)
    monkeypatch.delitem(sys.modules, "diff_gaussian_rasterization._C", raising=False)
    dge_amd.install_alias(fused_render=True)
    assert rend.render is ours.render and system.render is ours.render
    assert rend.camera2rasterizer is ours.camera2rasterizer
    import diff_gaussian_rasterization

    assert diff_gaussian_rasterization is dge_amd.diff_gaussian_rasterization
