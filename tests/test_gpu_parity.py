"""GPU parity tests: the gfx950 HIP path (through the C ABI) against the
oracle and the committed golden fixtures.

Bar (helpers.py), the same at every size, nothing tolerated in counts:
  * forward: every output and intermediate bit-identical to the oracle
    (num_rendered, radii, geometry, clamp flags, ranges, per-tile lists,
    final_T, n_contrib, image, depth) — the blend exp is the same IEEE
    sequence on both sides (gs_exp / gs_expf), so every skip/stop decision is;
  * backward: the rasterizer's gradient sums within 1e-4 x the magnitude of
    their terms, and the per-Gaussian chain bit-identical to the oracle's on the
    same sums; end-to-end gradients reported and bounded.
Every comparison prints its mismatch counts ([parity ...] lines, pytest -s).
"""
from __future__ import annotations

import glob
import math
import os

import numpy as np
import pytest
import torch

from helpers import GRAD_NAMES, RTOL, assert_close, camera_settings, compare_forward, compare_grads, golden_inputs, \
    run_gpu, run_oracle, scene_arrays, settings_from_golden

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _sh_kw(a, deg=3):
    n = (deg + 1) ** 2
    return dict(means3D=a["means3D"], opacities=a["opacities"], shs=np.ascontiguousarray(a["shs"][:, :max(n, 1)]),
                scales=a["scales"], rotations=a["rotations"])


@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "scene_*.npz"))), ids=os.path.basename)
def test_golden_fixture(cuda_device, oracle, path):
    rec = np.load(path)
    s = settings_from_golden(rec, "cuda")
    got = run_gpu(s, rec["dL_dpix"], **golden_inputs(rec))
    ref = {k: rec[k] for k in rec.files}
    ref["state"] = oracle.forward(settings_from_golden(rec), **golden_inputs(rec))[4]  # (chain stage only)
    compare_forward(got, ref, check_rgb=str(rec["mode"]) != "colors", label=os.path.basename(path))
    compare_grads(got, ref, O=oracle, label=os.path.basename(path))


def test_blend_exp_bitwise_vs_oracle(cuda_device, oracle):
    """The blend's exp (gs_exp, packed as the blend loops evaluate it) against the oracle's gs_expf,
    bit for bit: the whole live range, every float of [-6, 0] near the 1/255 level, extremes, NaN/inf."""
    from dge_amd import _native

    rng = np.random.default_rng(0)
    lo = np.float32(np.log(1 / 255.0 / 0.99))
    near = np.arange(-2 ** 14, 2 ** 14, dtype=np.int64) + np.array(lo, np.float32).view(np.int32)
    xs = np.concatenate([
        rng.uniform(-12.0, 1.0, 2_000_000).astype(np.float32),
        rng.uniform(-200.0, 200.0, 200_000).astype(np.float32),
        near.astype(np.int32).view(np.float32),
        np.array([0.0, -0.0, -80.0, -87.3, -88.8, -103.9, -104.0, 88.7, 89.0, 1e30, -1e30, 3e38, -3e38,
                  np.inf, -np.inf, np.nan, 1e-30, -1e-30, 1.4e-45], np.float32)])
    x = torch.from_numpy(xs).cuda()
    y = torch.empty_like(x)
    _native.check(_native.lib().gs_blend_exp(x.numel(), x.data_ptr(), y.data_ptr(), None), "gs_blend_exp")
    got = y.cpu().numpy()
    ref = oracle.expf(xs)
    same = (got.view(np.uint32) == ref.view(np.uint32)) | (np.isnan(got) & np.isnan(ref))
    print(f"[parity] blend exp: {int((~same).sum())} of {xs.size} differ")
    assert same.all(), xs[~same][:10]
    live = (xs > -10) & (xs < 1)
    ref64 = np.exp(xs[live].astype(np.float64))
    ulps = np.abs(got[live].astype(np.float64) - ref64) / np.spacing(ref64.astype(np.float32)).astype(np.float64)
    print(f"[parity] blend exp: max {ulps.max():.3f} ulp against fp64 exp on [-10, 1]")
    assert ulps.max() <= 1.5  # (the oracle restatement: <= 0.86 ulp on every float of [-6, 0], 0.97 on [-10, 1])


def test_c1_scene_vs_oracle(cuda_device, oracle):
    """configs[0]: 10k Gaussians, 1 camera, 256x256, fwd + bwd."""
    a = scene_arrays(10_000, seed=0, radius=2.0, scale=0.02)
    s = camera_settings(256, 256)
    g = np.random.default_rng(1).standard_normal((3, 256, 256)).astype(np.float32) * 1e-3
    kw = _sh_kw(a)
    ref = run_oracle(oracle, s, g, **kw)
    got = run_gpu(camera_settings(256, 256, device="cuda"), g, **kw)
    compare_forward(got, ref, label="c1")
    compare_grads(got, ref, O=oracle, label="c1")


@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_sh_degrees_with_stride16(cuda_device, oracle, deg):
    a = scene_arrays(3000, seed=20 + deg, radius=1.5, scale=0.04)
    kw = dict(means3D=a["means3D"], opacities=a["opacities"], shs=a["shs"], scales=a["scales"],
              rotations=a["rotations"])  # M = 16 stride whatever the active degree (load_ply behaviour)
    s = camera_settings(128, 96, sh_degree=deg, bg=(0.1, 0.1, 0.3))
    g = np.random.default_rng(deg).standard_normal((3, 96, 128)).astype(np.float32)
    ref = run_oracle(oracle, s, g, **kw)
    got = run_gpu(camera_settings(128, 96, sh_degree=deg, bg=(0.1, 0.1, 0.3), device="cuda"), g, **kw)
    compare_forward(got, ref, label=f"deg{deg}")
    compare_grads(got, ref, O=oracle, label=f"deg{deg}")
    n = (deg + 1) ** 2 if deg < 3 else 16
    assert not got["dL_dsh"][:, n:].any()


def test_colors_and_cov3d_precomp(cuda_device, oracle):
    a = scene_arrays(4000, seed=31, radius=1.5, scale=0.05)
    colors = np.random.default_rng(3).random((4000, 3)).astype(np.float32)
    kw = dict(means3D=a["means3D"], opacities=a["opacities"], colors_precomp=colors, cov3D_precomp=a["cov3D"])
    g = np.random.default_rng(4).standard_normal((3, 80, 144)).astype(np.float32)
    ref = run_oracle(oracle, camera_settings(144, 80, view=2, nviews=5), g, **kw)
    got = run_gpu(camera_settings(144, 80, view=2, nviews=5, device="cuda"), g, **kw)
    compare_forward(got, ref, check_rgb=False, label="precomp")
    compare_grads(got, ref, O=oracle, label="precomp")
    assert not got["dL_dscales"].any() and not got["dL_drotations"].any()


def test_scale_modifier_and_ragged(cuda_device, oracle):
    a = scene_arrays(2500, seed=41, radius=1.2, scale=0.06)
    kw = _sh_kw(a)
    g = np.random.default_rng(5).standard_normal((3, 37, 100)).astype(np.float32)
    s = camera_settings(100, 37, scale_modifier=0.7)
    ref = run_oracle(oracle, s, g, **kw)
    got = run_gpu(camera_settings(100, 37, scale_modifier=0.7, device="cuda"), g, **kw)
    compare_forward(got, ref, label="ragged")
    compare_grads(got, ref, O=oracle, label="ragged")


def test_empty_and_all_culled(cuda_device, oracle):
    s = camera_settings(48, 40, bg=(0.3, 0.2, 0.1), device="cuda")
    z = np.zeros((0, 3), np.float32)
    got = run_gpu(s, np.ones((3, 40, 48), np.float32), means3D=z, opacities=np.zeros((0, 1), np.float32),
                  colors_precomp=z, scales=z, rotations=np.zeros((0, 4), np.float32))
    assert got["num_rendered"] == 0 and not got["color"].any() and got["radii"].shape == (0,)
    # everything behind the camera: background image, zero gradients
    a = scene_arrays(500, seed=3, radius=0.3)
    cam_pos = s.campos.cpu().numpy()
    behind = (2 * cam_pos[None, :] + a["means3D"]).astype(np.float32)  # beyond the camera, opposite side
    kw = dict(means3D=behind, opacities=a["opacities"], shs=a["shs"], scales=a["scales"], rotations=a["rotations"])
    got = run_gpu(s, np.ones((3, 40, 48), np.float32), **kw)
    assert got["num_rendered"] == 0 and not got["radii"].any()
    np.testing.assert_allclose(got["color"], np.broadcast_to(np.array([0.3, 0.2, 0.1])[:, None, None], (3, 40, 48)),
                               rtol=1e-7)
    for n in GRAD_NAMES:
        assert not got[n].any(), n


def test_known_answer_single_gaussian(cuda_device, oracle):
    from test_oracle import _analytic_single, _front_settings, _iso

    s_cpu = _front_settings(64, 64)
    s = _front_settings(64, 64)
    for k in ("bg", "viewmatrix", "projmatrix", "campos"):
        s = s._replace(**{k: getattr(s, k).cuda()})
    got = run_gpu(s, **_iso(2.0, 0.05, 0.8, (1.0, 0.5, 0.25)))
    expect, _ = _analytic_single(64, 64, 2.0, 0.05, 0.8, (1.0, 0.5, 0.25), s_cpu)
    np.testing.assert_allclose(got["color"], expect, rtol=1e-5, atol=1e-6)
    assert got["num_rendered"] == 4 and got["radii"][0] == 5


@pytest.mark.parametrize("W,H", [(16, 16), (32, 16)], ids=["one_tile", "two_tiles"])
def test_replay_lists_out_of_balance(cuda_device, oracle, W, H):
    """The replay's work lists are per forward XCD group (kItemXcds, gs_internal.h): one tile puts every
    item in one of the eight lists, so 8 x the longest list outgrows the grid (4 x checkpoint slots) and
    k_render_bwd takes the lists one after another; two tiles leave six lists empty (the XCD mapping's
    regions mostly holes).  Faint Gaussians: no pixel saturates, every quadrant's window is its whole list."""
    a = scene_arrays(3000, seed=17, radius=0.4, scale=0.05)
    kw = _sh_kw(a)
    kw["opacities"] = np.full_like(a["opacities"], 0.02)
    g = np.random.default_rng(9).standard_normal((3, H, W)).astype(np.float32)
    ref = run_oracle(oracle, camera_settings(W, H), g, **kw)
    got = run_gpu(camera_settings(W, H, device="cuda"), g, **kw)
    compare_forward(got, ref, label=f"lists {W}x{H}")
    compare_grads(got, ref, O=oracle, label=f"lists {W}x{H}")
    # the fallback's condition, from the forward's windows: a tile's items sit in one list, whose longest
    # class holds at least a quarter of them
    tiles = (W // 16) * (H // 16)
    nc = got["n_contrib"].reshape(H // 16, 2, 8, W // 16, 2, 8)
    items = np.ceil(nc.max(axis=(2, 5)) / 128).reshape(H // 16, 2, W // 16, 2).sum(axis=(1, 3)).ravel()
    grid = 4 * (got["num_rendered"] // 128 + tiles + 2)
    print(f"[parity] replay lists: items per tile {items.tolist()}, grid {grid}")
    assert (8 * np.ceil(items.max() / 4) > grid) == (tiles == 1)


def test_prefiltered_error_is_reported(cuda_device):
    from dge_amd._native import NativeError

    a = scene_arrays(50, seed=1)
    s = camera_settings(32, 32, device="cuda")
    s = s._replace(prefiltered=True)
    m = a["means3D"].copy()
    m[0] = 2 * s.campos.cpu().numpy()  # behind the camera -> culled although prefiltered
    with pytest.raises(NativeError, match="prefiltered"):
        run_gpu(s, means3D=m, opacities=a["opacities"], shs=a["shs"], scales=a["scales"], rotations=a["rotations"])


def test_mark_visible(cuda_device, oracle):
    from dge_amd.diff_gaussian_rasterization import GaussianRasterizer

    a = scene_arrays(5000, seed=5, radius=6.0)
    s = camera_settings(64, 64, device="cuda")
    got = GaussianRasterizer(s).markVisible(torch.from_numpy(a["means3D"]).cuda()).cpu().numpy()
    ref = oracle.mark_visible(a["means3D"], s.viewmatrix.cpu(), s.projmatrix.cpu())
    np.testing.assert_array_equal(got, ref)
    assert 0 < got.sum() < 5000


@pytest.mark.parametrize("C", [1, 2, 3])
def test_apply_weights(cuda_device, oracle, C):
    from dge_amd.diff_gaussian_rasterization import GaussianRasterizer

    P, W, H = 3000, 96, 64
    a = scene_arrays(P, seed=60 + C, radius=1.2, scale=0.05)
    iw = np.random.default_rng(C).random((C, H, W)).astype(np.float32)
    w0 = np.zeros((P, C), np.float32)
    c0 = np.zeros((P, 1), np.int32)
    s = camera_settings(W, H, device="cuda")
    w_ref, c_ref = oracle.apply_weights(s, a["means3D"], a["opacities"], w0, c0, iw, scales=a["scales"],
                                        rotations=a["rotations"])
    dev = torch.device("cuda")
    wt, ct = torch.zeros(P, C, device=dev), torch.zeros(P, 1, dtype=torch.int32, device=dev)
    GaussianRasterizer(s).apply_weights(torch.from_numpy(a["means3D"]).cuda(), None,
                                        torch.from_numpy(a["opacities"]).cuda(), weights=wt,
                                        scales=torch.from_numpy(a["scales"]).cuda(),
                                        rotations=torch.from_numpy(a["rotations"]).cuda(), cnt=ct,
                                        image_weights=torch.from_numpy(iw).cuda())
    np.testing.assert_array_equal(ct.cpu().numpy(), c_ref)
    assert_close(wt.cpu().numpy(), w_ref, "weights", 1e-5)


def test_render_dropin_autograd(cuda_device, oracle):
    """render() through autograd: screen-space and parameter grads = oracle grads chained through the getters."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    sc = synthetic_scene(5000, seed=77, radius=1.5, scale=0.04, device=dev).requires_grad_(True)
    cam = orbit_camera(1, 4, 160, 120, device=dev)
    G = torch.randn(3, 120, 160, generator=torch.Generator().manual_seed(9)).to(dev)
    pkg = render(cam, sc, PipelineParams(), torch.zeros(3, device=dev))
    assert set(pkg) == {"render", "viewspace_points", "visibility_filter", "radii", "depth_3dgs"}
    assert pkg["render"].shape == (3, 120, 160) and pkg["depth_3dgs"].shape == (1, 120, 160)
    assert pkg["radii"].dtype == torch.int32 and pkg["visibility_filter"].dtype == torch.bool
    (pkg["render"] * G).sum().backward()

    from dge_amd.gaussian_renderer import _settings

    s = _settings(orbit_camera(1, 4, 160, 120, device="cpu"), torch.zeros(3), 1.0, 3)
    with torch.no_grad():
        kw = dict(means3D=sc.get_xyz.cpu().numpy(), opacities=sc.get_opacity.cpu().numpy(),
                  shs=sc.get_features.cpu().numpy(), scales=sc.get_scaling.cpu().numpy(),
                  rotations=sc.get_rotation.cpu().numpy())
    ref = run_oracle(oracle, s, G.cpu().numpy(), **kw)
    assert_close(pkg["render"].detach().cpu().numpy(), ref["color"], "render")
    assert_close(pkg["viewspace_points"].grad.cpu().numpy(), ref["dL_dmeans2D"], "viewspace grad")
    # chain the oracle's activated-parameter grads through the reference getters on the CPU
    cpu = synthetic_scene(5000, seed=77, radius=1.5, scale=0.04).requires_grad_(True)
    outs = [cpu.get_xyz, cpu.get_opacity, cpu.get_features, cpu.get_scaling, cpu.get_rotation]
    grads = [ref["dL_dmeans3D"], ref["dL_dopacity"], ref["dL_dsh"], ref["dL_dscales"], ref["dL_drotations"]]
    torch.autograd.backward(outs, [torch.from_numpy(g) for g in grads])
    for name, p_gpu, p_cpu in zip(["_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"],
                                  sc.parameters(), cpu.parameters()):
        assert_close(p_gpu.grad.cpu().numpy(), p_cpu.grad.numpy(), name)


def test_python_sh_and_cov_paths_render(cuda_device, oracle):
    """convert_SHs_python / compute_cov3D_python (broken in the reference): the torch-side colours /
    covariances go to the kernels as colors_precomp / cov3D_precomp, and the image is bit-identical
    to the oracle's on those same inputs."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, _settings, render
    from dge_amd.scene import synthetic_scene
    from dge_amd.sh_utils import eval_sh

    dev = torch.device("cuda")
    sc = synthetic_scene(3000, seed=8, radius=1.5, scale=0.04, device=dev)
    cam = orbit_camera(0, 1, 96, 96, device=dev)
    bg = torch.zeros(3, device=dev)
    s = _settings(orbit_camera(0, 1, 96, 96, device="cpu"), torch.zeros(3), 1.0, 3)
    with torch.no_grad():
        py_sh = render(cam, sc, PipelineParams(convert_SHs_python=True), bg)["render"].cpu().numpy()
        py_cov = render(cam, sc, PipelineParams(compute_cov3D_python=True), bg)["render"].cpu().numpy()
        feats = sc.get_features
        dirs = sc.get_xyz - cam.camera_center.repeat(feats.shape[0], 1)
        dirs = dirs / dirs.norm(dim=1, keepdim=True)
        colors = torch.clamp_min(eval_sh(sc.active_sh_degree, feats.transpose(1, 2).reshape(-1, 3, 16), dirs) + 0.5,
                                 0.0).cpu().numpy()
        cov = sc.get_covariance(1.0).cpu().numpy()
        base = dict(means3D=sc.get_xyz.cpu().numpy(), opacities=sc.get_opacity.cpu().numpy())
        ref_sh = oracle.forward(s, colors_precomp=colors, scales=sc.get_scaling.cpu().numpy(),
                                rotations=sc.get_rotation.cpu().numpy(), **base)[1]
        ref_cov = oracle.forward(s, shs=feats.cpu().numpy(), cov3D_precomp=cov, **base)[1]
    np.testing.assert_array_equal(py_sh, ref_sh)
    np.testing.assert_array_equal(py_cov, ref_cov)


# ---------------------------------------------------------------------------
# full-size (configs[1] / [3]) parity and size-independent properties
# ---------------------------------------------------------------------------
def test_c2_full_size_vs_oracle(cuda_device, oracle):
    """configs[1]: 1.0M Gaussians, 512x512, fp32 fwd+bwd vs the oracle on the same inputs: forward bit-identical
    (lists, n_contrib, T, image), rasterizer sums within 1e-4 x magnitude, chain bit-identical."""
    a = scene_arrays(1_000_000, seed=0, radius=2.0, scale=0.02)
    g = np.random.default_rng(1).standard_normal((3, 512, 512)).astype(np.float32) * 1e-3
    kw = _sh_kw(a)
    ref = run_oracle(oracle, camera_settings(512, 512), g, **kw)
    got = run_gpu(camera_settings(512, 512, device="cuda"), g, **kw)
    compare_forward(got, ref, label="c2")
    compare_grads(got, ref, O=oracle, label="c2")


def test_c2_render_raw_parameter_grads_per_element(cuda_device, oracle):
    """The gradients DGE consumes, at the timed size: render()'s fused raw-parameter path (c2: 1M Gaussians,
    512x512, view 0 of the bench's 3-view orbit; activations and their derivatives in-kernel, gradients
    written straight into _xyz.grad ... _rotation.grad) against the oracle's activated-parameter gradients
    chained through the reference getters (sigmoid / exp / normalize, gaussian_model.py:221-258) by torch
    autograd on the CPU.

    Per element, no max-floor: |got - ref| <= 1e-4 (|ref| + m), where m is the magnitude of the terms the
    element is made of — the oracle's per-Gaussian raster-sum magnitudes (mag9: sums of |sub-term| over the
    contributing pixels) carried through the per-Gaussian chain in absolute arithmetic (every coefficient
    |c|, every subtraction an addition: oracle.backward_chain_mag, backward.cu:144-396) and through |J| of
    the getter.  A reordered sum, and the chain's own float rounding, can move an element by a fraction of
    m, never of its own value, so this is the bar a cancelling element can be held to (a scale gradient
    along a Gaussian axis seen end-on is such an element: terms of ~1e-5 cancelling to ~1e-11).  Printed: the worst err / (1e-4 (|ref| + m)) and the worst relative error |got-ref|/|ref|
    over the elements above the floor |ref| >= m / 100 (a sum cancelled by less than 100x); asserted <= 1e-4.
    The oracle runs on the device's activations (gs_activate_params) so the forward — and with it every
    blend decision — is bit-identical (asserted), as in the timed-path test."""
    import ctypes

    from dge_amd import _native as N
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, _fused_ok, _settings, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    P, W, H, V = 1_000_000, 512, 512, 3
    sc = synthetic_scene(P, sh_degree=3, seed=0, device=dev).requires_grad_(True)
    assert _fused_ok(sc, PipelineParams())
    G = (torch.randn(3, H, W, generator=torch.Generator().manual_seed(1)) * 1e-3).to(dev)
    pkg = render(orbit_camera(0, V, W, H, device=dev), sc, PipelineParams(), torch.zeros(3, device=dev))
    pkg["render"].backward(G)
    torch.cuda.synchronize()
    got = {n: p.grad.cpu().numpy().astype(np.float64) for n, p in
           zip(["_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"], sc.parameters())}
    got["viewspace"] = pkg["viewspace_points"].grad.cpu().numpy()[:, :2].astype(np.float64)
    with torch.no_grad():
        op, scl, rot = (torch.empty(P, k, device=dev) for k in (1, 3, 4))
        N.check(N.lib().gs_activate_params(P, sc._opacity.data_ptr(), sc._scaling.data_ptr(), sc._rotation.data_ptr(),
                                           op.data_ptr(), scl.data_ptr(), rot.data_ptr(),
                                           ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                "gs_activate_params")
        torch.cuda.synchronize()
        op, scl, rot = op.cpu().numpy(), scl.cpu().numpy(), rot.cpu().numpy()
    s = _settings(orbit_camera(0, V, W, H, device="cpu"), torch.zeros(3), 1.0, 3)
    nr, color, _, radii, st = oracle.forward(s, means3D=sc._xyz.detach().cpu().numpy(), opacities=op,
                                             shs=torch.cat([sc._features_dc, sc._features_rest], 1).detach().cpu().numpy(),
                                             scales=scl, rotations=rot)
    np.testing.assert_array_equal(pkg["radii"].cpu().numpy(), radii)
    np.testing.assert_array_equal(pkg["render"].detach().cpu().numpy(), color)  # every blend decision the oracle's
    ref = oracle.backward(st, G.cpu().numpy())
    mag9 = ref["mag9"].astype(np.float64)
    # the chain in absolute arithmetic over the 9 sums' magnitudes (oracle go_backward_chain_mag)
    cm = oracle.backward_chain_mag(st, ref["mag9"])
    # the getters (CPU torch autograd) for the reference values, |J| of each getter for the magnitudes
    cpu = synthetic_scene(P, sh_degree=3, seed=0).requires_grad_(True)
    torch.autograd.backward([cpu.get_xyz, cpu.get_opacity, cpu.get_features, cpu.get_scaling, cpu.get_rotation],
                            [torch.from_numpy(ref[k]) for k in
                             ("dL_dmeans3D", "dL_dopacity", "dL_dsh", "dL_dscales", "dL_drotations")])
    refs = {n: p.grad.numpy().astype(np.float64) for n, p in
            zip(["_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"], cpu.parameters())}
    refs["viewspace"] = ref["dL_dmeans2D"][:, :2].astype(np.float64)
    q = cpu._rotation.detach().numpy().astype(np.float64)
    qn = np.linalg.norm(q, axis=1, keepdims=True)
    y = q / qn
    jrot = np.abs((np.eye(4)[None] - y[:, :, None] * y[:, None, :]) / qn[:, :, None])  # d normalize / dq
    o = op.astype(np.float64)
    mags = {"_xyz": cm["dL_dmeans3D"], "_features_dc": cm["dL_dsh"][:, :1], "_features_rest": cm["dL_dsh"][:, 1:],
            "_opacity": mag9[:, 5:6] * o * (1 - o), "_scaling": cm["dL_dscales"] * scl.astype(np.float64),
            "_rotation": np.einsum("pij,pj->pi", jrot, cm["dL_drotations"]), "viewspace": mag9[:, 0:2]}
    worst = {}
    for n, r in refs.items():
        g, m = got[n], mags[n]
        assert g.shape == r.shape == m.shape, n
        err = np.abs(g - r)
        bound = RTOL * (np.abs(r) + m)
        ratio = np.where(bound > 0, err / np.maximum(bound, 1e-300), np.where(err > 0, np.inf, 0.0))
        above = (np.abs(r) >= m / 100) & (r != 0)
        rel = float((err[above] / np.abs(r[above])).max()) if above.any() else 0.0
        i = np.unravel_index(np.argmax(ratio), r.shape)
        worst[n] = (float(ratio.max()), rel, int(above.sum()), int(r.size), int((ratio > 1).sum()),
                    f"worst at {i}: got {g[i]:.6e} ref {r[i]:.6e} m {m[i]:.3e}")
    print("[parity c2 raw grads] per tensor (worst err/bound, worst rel err where |ref| >= m/100, "
          f"elements above the floor, elements, elements beyond the bound, worst element): {worst}")
    for n, w in worst.items():
        assert w[0] <= 1.0, f"{n}: worst err / (1e-4 (|ref| + m)) = {w[0]:.3g}, {w[4]} beyond; {w[5]}"
        assert w[1] <= RTOL, f"{n}: worst relative error {w[1]:.3g} above the floor"


def _fused_truth_check(O, sc, pkg, G, cam_cpu, label, index=None, half_sh=False):
    """render()'s fused raw-parameter gradients (already in sc's .grad, pkg its outputs) against the fp64
    truth (tests/helpers.py truth_bar).  The oracle runs on the device's own activations of the rendered rows
    (gs_activate_params: the device functions the fused kernels apply, so the forward — every blend decision —
    is bit-identical, asserted) with SH as stored (fp16 upcast when half_sh); the truth and the reference's fp32
    evaluations (five: the oracle's float sums and four atomic arrival orders) chain through the getters of
    the raw rows.  DGE_AMD_TRUTH_DUMP=<dir>: the compared rows are saved there (offline analysis)."""
    import ctypes
    import os

    from dge_amd import _native as N
    from dge_amd.gaussian_renderer import _settings
    from helpers import PARAM_NAMES, truth_bar, truth_case

    dev = sc._xyz.device
    params = dict(zip(PARAM_NAMES, sc.parameters()))
    rows = None if index is None else index.to(dev).long()
    raw = {k: (p.detach() if rows is None else p.detach()[rows]).contiguous() for k, p in params.items()}
    n = raw["_xyz"].shape[0]
    with torch.no_grad():
        op, scl, rot = (torch.empty(n, k, device=dev) for k in (1, 3, 4))
        N.check(N.lib().gs_activate_params(n, raw["_opacity"].data_ptr(), raw["_scaling"].data_ptr(),
                                           raw["_rotation"].data_ptr(), op.data_ptr(), scl.data_ptr(), rot.data_ptr(),
                                           ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)),
                "gs_activate_params")
        torch.cuda.synchronize()
    s = _settings(cam_cpu, torch.zeros(3), 1.0, sc.active_sh_degree)
    shs = torch.cat([raw["_features_dc"], raw["_features_rest"]], 1).float().cpu().numpy()
    _, color, _, radii, st = O.forward(s, means3D=raw["_xyz"].cpu().numpy(), opacities=op.cpu().numpy(), shs=shs,
                                       scales=scl.cpu().numpy(), rotations=rot.cpu().numpy())
    np.testing.assert_array_equal(pkg["radii"].cpu().numpy(), radii)
    np.testing.assert_array_equal(pkg["render"].detach().cpu().numpy(), color)  # every blend decision the oracle's
    truth, refs, names, live = truth_case(O, st, G.detach().cpu().numpy(), {k: v.cpu() for k, v in raw.items()},
                                          half_sh)
    got = {k: (p.grad if rows is None else p.grad[rows]).float().cpu().numpy().astype(np.float64)
           for k, p in params.items()}
    got["viewspace"] = pkg["viewspace_points"].grad.cpu().numpy()[:, :2].astype(np.float64)
    dead = np.ones(n, bool)
    dead[live] = False
    for k, v in got.items():  # a Gaussian with all-zero rasterizer sums has exactly zero gradients
        assert not np.any(v[dead]), f"{label} {k}: nonzero gradient at a Gaussian no pixel blended"
    got = {k: v[live] for k, v in got.items()}
    d = os.environ.get("DGE_AMD_TRUTH_DUMP")
    return truth_bar(got, truth, refs, label, dump=os.path.join(d, f"truth_{label}.npz") if d else None, names=names)


def test_c2_render_raw_grads_vs_fp64_truth(cuda_device, oracle):
    """The gradients DGE consumes, at the timed size (c2: 1M Gaussians, 512x512, view 0 of the bench's 3-view
    orbit; render()'s fused raw-parameter path: activations in-kernel, gradients written into _xyz.grad ...
    _rotation.grad), held per element to the fp64 truth: |got - truth| <= 4 E_ref + 1e-4 |truth|, E_ref the
    largest error of the reference's fp32 evaluations, at most 1% of a tensor's nonzero elements admitted by
    the second term alone (tests/helpers.py truth_bar; backward.cu:144-557, gaussian_model.py:221-258)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, _fused_ok, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    P, W, H, V = 1_000_000, 512, 512, 3
    sc = synthetic_scene(P, sh_degree=3, seed=0, device=dev).requires_grad_(True)
    assert _fused_ok(sc, PipelineParams())
    G = (torch.randn(3, H, W, generator=torch.Generator().manual_seed(1)) * 1e-3).to(dev)
    pkg = render(orbit_camera(0, V, W, H, device=dev), sc, PipelineParams(), torch.zeros(3, device=dev))
    pkg["render"].backward(G)
    torch.cuda.synchronize()
    _fused_truth_check(oracle, sc, pkg, G, orbit_camera(0, V, W, H, device="cpu"), "c2")


def test_c5_render_fp16_sh_local_edit_vs_fp64_truth(cuda_device, oracle):
    """configs[4] through render(): 1M-Gaussian scene, localize on a 200k mask, SH stored fp16 (upcast
    in-kernel, gradients written back as fp16), the fused index path — its subset-row gradients against the
    fp64 truth with the same bar as c2 (the reference's fp32 evaluations' SH gradients cast to fp16, as
    autograd casts them back to the half leaf)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    P, Psub, W, H = 1_000_000, 200_000, 512, 512
    sc = synthetic_scene(P, seed=0, device=dev)
    sc._features_dc = sc._features_dc.half()
    sc._features_rest = sc._features_rest.half()
    order = torch.argsort(sc._xyz[:, 0])
    mask = torch.zeros(P, dtype=torch.bool, device=dev)
    mask[order[:Psub]] = True
    sc.mask, sc.localize = mask, True
    sc.requires_grad_(True)
    G = (torch.randn(3, H, W, generator=torch.Generator().manual_seed(1)) * 1e-3).to(dev)
    pkg = render(orbit_camera(0, 1, W, H, device=dev), sc, PipelineParams(), torch.zeros(3, device=dev))
    (pkg["render"] * G).sum().backward()
    torch.cuda.synchronize()
    assert sc._features_dc.grad.dtype == torch.float16
    _fused_truth_check(oracle, sc, pkg, G, orbit_camera(0, 1, W, H, device="cpu"), "c5",
                       index=torch.nonzero(mask).flatten(), half_sh=True)


def test_render_dropin_autograd_vs_fp64_truth(cuda_device, oracle):
    """test_render_dropin_autograd's render() (5000 Gaussians, 160x120) held to the fp64 truth bar."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    sc = synthetic_scene(5000, seed=77, radius=1.5, scale=0.04, device=dev).requires_grad_(True)
    G = torch.randn(3, 120, 160, generator=torch.Generator().manual_seed(9)).to(dev)
    pkg = render(orbit_camera(1, 4, 160, 120, device=dev), sc, PipelineParams(), torch.zeros(3, device=dev))
    (pkg["render"] * G).sum().backward()
    torch.cuda.synchronize()
    _fused_truth_check(oracle, sc, pkg, G, orbit_camera(1, 4, 160, 120, device="cpu"), "dropin")


def test_c4_hd_forward_vs_oracle(cuda_device, oracle):
    """configs[3]: 2.5M Gaussians, 1920x1080 forward (8160 tiles -> two-pass tile sort), bit-identical."""
    from dge_amd.gaussian_renderer import _settings
    from dge_amd.cameras import orbit_camera

    a = scene_arrays(2_500_000, seed=2, radius=2.0, scale=0.02)
    kw = _sh_kw(a)
    ref = run_oracle(oracle, _settings(orbit_camera(0, 1, 1920, 1080, device="cpu"), torch.zeros(3), 1.0, 3), **kw)
    got = run_gpu(_settings(orbit_camera(0, 1, 1920, 1080, device="cuda"), torch.zeros(3, device="cuda"), 1.0, 3),
                  **kw)
    compare_forward(got, ref, label="c4")


def test_backward_is_deterministic_and_linear(cuda_device):
    a = scene_arrays(200_000, seed=5, radius=2.0, scale=0.02)
    kw = _sh_kw(a)
    s = camera_settings(384, 256, device="cuda")
    rng = np.random.default_rng(7)
    g1 = rng.standard_normal((3, 256, 384)).astype(np.float32)
    g2 = rng.standard_normal((3, 256, 384)).astype(np.float32)
    r1 = run_gpu(s, g1, intermediates=False, **kw)
    r1b = run_gpu(s, g1, intermediates=False, **kw)
    for n in GRAD_NAMES + ["color", "depth"]:
        np.testing.assert_array_equal(r1[n], r1b[n], err_msg=f"{n} not bitwise reproducible")
    r2 = run_gpu(s, g2, intermediates=False, **kw)
    r12 = run_gpu(s, 2.0 * g1 - 0.5 * g2, intermediates=False, **kw)
    for n in GRAD_NAMES:
        assert_close(r12[n], 2.0 * r1[n] - 0.5 * r2[n], n + " linearity", 1e-4)


@pytest.mark.parametrize("override", [False, True])
def test_fused_raw_parameter_path_matches_getter_path(cuda_device, monkeypatch, override):
    """render() on a standard GaussianModel reads the raw tensors in-kernel (activations fused);
    image, screen-space and raw-parameter gradients equal the getter path's."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, _fused_ok, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    cam = orbit_camera(2, 5, 200, 136, device=dev)
    G = torch.randn(3, 136, 200, generator=torch.Generator().manual_seed(11)).to(dev)
    outs = []
    for fused in (True, False):
        monkeypatch.setenv("DGE_AMD_FUSED", "1" if fused else "0")
        sc = synthetic_scene(20_000, seed=21, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
        assert _fused_ok(sc, PipelineParams()) == fused
        oc = None
        if override:
            oc = torch.rand(20_000, 3, generator=torch.Generator().manual_seed(2)).to(dev)
        pkg = render(cam, sc, PipelineParams(), torch.tensor([0.1, 0.0, 0.2], device=dev), override_color=oc)
        assert torch.equal(pkg["visibility_filter"], pkg["radii"] > 0)  # (fused: written by the preprocess)
        assert pkg["visibility_filter"].dtype == torch.bool
        (pkg["render"] * G).sum().backward()
        grads = [None if p.grad is None else p.grad.cpu().numpy() for p in sc.parameters()]
        outs.append((pkg["render"].detach().cpu().numpy(), pkg["radii"].cpu().numpy(),
                     pkg["viewspace_points"].grad.cpu().numpy(), grads))
    (img_f, r_f, vs_f, g_f), (img_r, r_r, vs_r, g_r) = outs
    np.testing.assert_array_equal(r_f, r_r)
    assert_close(img_f, img_r, "image", 1e-5)
    assert_close(vs_f, vs_r, "viewspace grad", 1e-4)
    for name, a, b in zip(["_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"], g_f, g_r):
        if b is None:
            assert a is None or not np.any(a), name
            continue
        assert_close(a, b, name, 1e-4)


@pytest.mark.gpu
def test_fused_gradient_accumulation(cuda_device):
    """The raw-parameter path writes/adds gradients straight into .grad where autograd would; the
    result is bitwise the autograd accumulation (same fp32 adds) over two views, a pre-existing .grad
    and a multi-view batch, and torch.autograd.grad still receives returned gradients."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.diff_gaussian_rasterization import set_fused_grad_accumulation
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    cams = [orbit_camera(k, 4, 160, 120, device=dev) for k in range(2)]
    Gs = [torch.randn(3, 120, 160, generator=torch.Generator().manual_seed(30 + k)).to(dev) for k in range(2)]
    bg = torch.zeros(3, device=dev)

    def run(fused, pre_grad, batched):
        prev = set_fused_grad_accumulation(fused)
        try:
            sc = synthetic_scene(15_000, seed=5, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
            if pre_grad:
                for p in sc.parameters():
                    p.grad = torch.full_like(p, 0.25)
            outs = [render(c, sc, PipelineParams(), bg)["render"] for c in cams]
            if batched:  # one backward through both views (autograd sums them)
                sum((o * g).sum() for o, g in zip(outs, Gs)).backward()
            else:
                for o, g in zip(outs, Gs):
                    (o * g).sum().backward()
            return [p.grad.clone() for p in sc.parameters()]
        finally:
            set_fused_grad_accumulation(prev)

    for pre_grad in (False, True):
        for batched in (False, True):
            a, b = run(True, pre_grad, batched), run(False, pre_grad, batched)
            for x, y in zip(a, b):
                if batched and pre_grad:
                    # autograd sums the views first, pre + (g1 + g2); the fused path adds each view into
                    # .grad, (pre + g1) + g2: one rounding apart
                    torch.testing.assert_close(x, y, rtol=1e-6, atol=1e-6)
                else:  # the same fp32 additions in the same (or a commutative) order
                    assert torch.equal(x, y)

    # torch.autograd.grad captures instead of accumulating: gradients come back, .grad stays untouched
    sc = synthetic_scene(15_000, seed=5, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
    out = render(cams[0], sc, PipelineParams(), bg)["render"]
    params = list(sc.parameters())
    grads = torch.autograd.grad((out * Gs[0]).sum(), params)
    assert all(p.grad is None for p in params)
    sc2 = synthetic_scene(15_000, seed=5, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
    prev = set_fused_grad_accumulation(False)
    try:
        (render(cams[0], sc2, PipelineParams(), bg)["render"] * Gs[0]).sum().backward()
    finally:
        set_fused_grad_accumulation(prev)
    for g, p in zip(grads, sc2.parameters()):
        assert torch.equal(g, p.grad)


@pytest.mark.parametrize("views,pre_grad,side", [(3, False, 2), (3, True, 2), (10, False, 2), (3, False, 0)])
def test_dge_loop_backward_merges_the_views_passes(cuda_device, views, pre_grad, side):
    """DGE's loop (DGE.py:179-222, 672): the views rendered one by one, their images stacked into one masked
    l1 loss, ONE backward.  Each view's backward enqueues its gradient replay and the views' per-Gaussian passes
    run merged at the end of the backward (an autograd final callback; DGE_AMD_DEFER_PASSES=0: one pass per
    view inside each view's backward).  Every parameter's .grad and every view-space gradient is bitwise the
    same; 10 views: two native calls of at most 8; side: the replays rotate over the current stream and that
    many side streams (DGE_AMD_REPLAY_STREAMS)."""
    from dge_amd import diff_gaussian_rasterization as R
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    W, H = 160, 120
    cams = [orbit_camera(k, views, W, H, device=dev) for k in range(views)]
    gts = torch.rand(views, H, W, 3, generator=torch.Generator().manual_seed(3)).to(dev)
    bg = torch.zeros(3, device=dev)

    def run(defer):
        prev, R._DEFER_PASSES = R._DEFER_PASSES, defer
        prev_side, R._REPLAY_SIDE = R._REPLAY_SIDE, side
        try:
            sc = synthetic_scene(20_000, seed=8, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
            if pre_grad:
                for p in sc.parameters():
                    p.grad = torch.full_like(p, 0.125)
            pkgs = [render(c, sc, PipelineParams(), bg) for c in cams]
            images = torch.stack([p["render"].permute(1, 2, 0) for p in pkgs], 0)
            m = (images.detach().mean(-1, keepdim=True) > 0.05).float()
            torch.nn.functional.l1_loss(images * m, gts * m).backward()
            assert not R._PENDING_PASSES  # (flushed before backward() returned)
            return [p.grad.clone() for p in sc.parameters()], [p["viewspace_points"].grad.clone() for p in pkgs]
        finally:
            R._DEFER_PASSES, R._REPLAY_SIDE = prev, prev_side

    (ga, va), (gb, vb) = run(True), run(False)
    for x, y in zip(ga, gb):
        assert torch.equal(x, y)
    for x, y in zip(va, vb):
        assert torch.equal(x, y)
    assert all(bool(v.abs().sum() > 0) for v in va)


@pytest.mark.parametrize("localize", [False, True])
def test_compiled_binding_matches_ctypes_path(cuda_device, localize):
    """render()'s per-view calls through the compiled binding (dge_amd/csrc/gs_torch.cpp: the forward's halves and
    the recolor) against the ctypes path on the same inputs: image, depth, radii, visibility, the semantic recolor
    render (the edit mask as override_color, served from the training blend's aux sums) and every raw-parameter
    gradient bitwise; the binding is the one loaded (in-tree .so)."""
    from dge_amd import _C
    from dge_amd import gaussian_renderer as GR
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    GT = _C._GT
    assert GT is not None and os.path.dirname(GT.__file__) == os.path.join(ROOT, "dge_amd", "lib")
    dev = torch.device("cuda")
    cam = orbit_camera(1, 3, 200, 136, device=dev)
    G = torch.randn(3, 136, 200, generator=torch.Generator().manual_seed(12)).to(dev)
    outs = []
    try:
        for gt in (GT, None):
            _C._GT = gt
            sc = synthetic_scene(20_000, seed=22, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
            sc.mask = (torch.rand(20_000, generator=torch.Generator().manual_seed(3)) < 0.3).to(dev)
            sc.localize = localize
            hits = GR._RECOLOR_HITS
            pkg = render(cam, sc, PipelineParams(), torch.tensor([0.1, 0.0, 0.2], device=dev))
            n = int(sc.mask.sum()) if localize else 20_000
            sem = render(cam, sc, PipelineParams(), torch.tensor([0.1, 0.0, 0.2], device=dev),
                         override_color=torch.ones(n, 3, device=dev))["render"]
            assert GR._RECOLOR_HITS == hits + 1  # (the semantic render took the recolor path)
            (pkg["render"] * G).sum().backward()
            torch.cuda.synchronize()
            outs.append([pkg["render"], pkg["depth_3dgs"], pkg["radii"], pkg["visibility_filter"], sem,
                         pkg["viewspace_points"].grad] + [p.grad for p in sc.parameters()])
    finally:
        _C._GT = GT
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_deferred_passes_survive_a_failed_backward(cuda_device):
    """A backward that raises after a view's per-Gaussian pass was deferred never runs its final callback.
    The next backward must still run its own deferred passes (its .grad fully written, equal to a backward
    that never deferred) — the pending list is tied to the graph task that queued its callback, and a stale
    list is flushed (its passes run into the failed backward's buffers) before the next one starts."""
    from dge_amd import diff_gaussian_rasterization as R
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    W, H = 160, 120
    cams = [orbit_camera(k, 2, W, H, device=dev) for k in range(2)]
    G = torch.randn(3, H, W, generator=torch.Generator().manual_seed(4)).to(dev)
    bg = torch.zeros(3, device=dev)

    class Raiser(torch.autograd.Function):
        @staticmethod
        def forward(ctx, x):
            return x * 1.0

        @staticmethod
        def backward(ctx, g):
            raise RuntimeError("injected backward failure")

    def loss(sc, fail):
        leaf = torch.ones(4, device=dev, requires_grad=True)
        side = Raiser.apply(leaf) if fail else leaf * 1.0  # (created first: autograd runs it after the renders)
        imgs = [render(c, sc, PipelineParams(), bg)["render"] for c in cams]
        return sum((im * G).sum() for im in imgs) + side.sum() * 0.0

    sc = synthetic_scene(15_000, seed=6, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
    with pytest.raises(RuntimeError, match="injected"):
        loss(sc, True).backward()
    assert R._PENDING_PASSES  # the failed backward left its deferred passes behind
    for p in sc.parameters():
        p.grad = None
    loss(sc, False).backward()
    torch.cuda.synchronize()
    assert not R._PENDING_PASSES
    got = [p.grad.clone() for p in sc.parameters()]

    prev, R._DEFER_PASSES = R._DEFER_PASSES, False
    try:
        ref = synthetic_scene(15_000, seed=6, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
        loss(ref, False).backward()
    finally:
        R._DEFER_PASSES = prev
    for g, p in zip(got, ref.parameters()):
        assert torch.equal(g, p.grad)


def test_c5_local_edit_fp16_sh_vs_oracle(cuda_device, oracle):
    """configs[4]: 1.0M-Gaussian scene, localize=True on a fixed 200k mask (sorted by x, first 20%),
    SH stored as fp16 and upcast in-kernel, fp32 covariance inputs, 512x512 fwd+bwd.
    (a) the rasterizer on the subset (the getters' pc[mask] tensors, SH kept fp16) against the oracle
        on the same values (SH = the fp16 values upcast): forward bit-identical,
        rasterizer sums within 1e-4 x magnitude, chain bit-identical;
    (b) render() — the fused index path that never materialises the subset — against (a): radii
        identical, image/gradients to the activation kernels' rounding (in-kernel sigmoid/exp/normalize
        vs torch's), counts printed; fp16 parameter gradients at the subset rows only."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, _settings, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    P, Psub, W, H = 1_000_000, 200_000, 512, 512
    sc = synthetic_scene(P, seed=0, device=dev)
    sc._features_dc = sc._features_dc.half()
    sc._features_rest = sc._features_rest.half()
    order = torch.argsort(sc._xyz[:, 0])
    mask = torch.zeros(P, dtype=torch.bool, device=dev)
    mask[order[:Psub]] = True
    sc.mask, sc.localize = mask, True
    G = (torch.randn(3, H, W, generator=torch.Generator().manual_seed(1)) * 1e-3).to(dev)
    s = _settings(orbit_camera(0, 1, W, H, device="cpu"), torch.zeros(3), 1.0, 3)
    with torch.no_grad():
        sub = dict(means3D=sc.get_xyz, opacities=sc.get_opacity, shs=sc.get_features, scales=sc.get_scaling,
                   rotations=sc.get_rotation)
    assert sub["shs"].dtype == torch.float16 and sub["shs"].shape == (Psub, 16, 3)
    # (a) reference-shaped rasterizer on the subset, fp16 SH upcast in-kernel
    from dge_amd import _C
    from helpers import compare_forward, compare_grads

    sd = _settings(orbit_camera(0, 1, W, H, device=dev), torch.zeros(3, device=dev), 1.0, 3)
    e = torch.empty(0, device=dev)
    K, color, depth, radii, geom, binning, img = _C.rasterize_gaussians(
        sd.bg, sub["means3D"], e, sub["opacities"], sub["scales"], sub["rotations"], 1.0, e, sd.viewmatrix,
        sd.projmatrix, sd.tanfovx, sd.tanfovy, H, W, sub["shs"], 3, sd.campos, False, False)
    dconic = torch.empty((Psub, 3), device=dev)
    grads = _C.rasterize_gaussians_backward(sd.bg, sub["means3D"], radii, e, sub["scales"], sub["rotations"], 1.0, e,
                                            sd.viewmatrix, sd.projmatrix, sd.tanfovx, sd.tanfovy, G, sub["shs"], 3,
                                            sd.campos, geom, K, binning, img, False, dL_dconic=dconic)
    torch.cuda.synchronize()
    got = dict(num_rendered=K, color=color.cpu().numpy(), depth=depth.cpu().numpy(), radii=radii.cpu().numpy(),
               dL_dconic3=dconic.cpu().numpy())
    for n, t in zip(GRAD_NAMES, grads):
        got[n] = t.cpu().numpy()
    kw = {k: v.float().cpu().numpy() for k, v in sub.items()}
    ref = run_oracle(oracle, s, G.cpu().numpy(), **kw)
    compare_forward(got, ref, label="c5")
    compare_grads(got, ref, O=oracle, label="c5")

    # (b) render(): the fused index path on the full model
    sc.requires_grad_(True)
    pkg = render(orbit_camera(0, 1, W, H, device=dev), sc, PipelineParams(), torch.zeros(3, device=dev))
    assert pkg["radii"].shape == (Psub,)
    (pkg["render"] * G).sum().backward()
    np.testing.assert_array_equal(pkg["radii"].cpu().numpy(), got["radii"])
    img_f = pkg["render"].detach().cpu().numpy()
    print(f"[parity c5] render() vs rasterizer(a): {int((img_f != got['color']).sum())} image elements differ, "
          f"max |d| {float(np.abs(img_f - got['color']).max()):.3e}")
    assert_close(img_f, got["color"], "render")
    assert_close(pkg["viewspace_points"].grad.cpu().numpy(), got["dL_dmeans2D"], "viewspace grad")
    gd = sc._features_dc.grad
    assert gd.dtype == torch.float16 and gd.shape == (P, 1, 3)
    m = mask.cpu().numpy()
    full = np.zeros((P, 16, 3), np.float32)
    full[m] = got["dL_dsh"].reshape(Psub, 16, 3)
    gsh = torch.cat([gd, sc._features_rest.grad], dim=1).float().cpu().numpy()
    assert_close(gsh, full.astype(np.float16).astype(np.float32), "dL_dsh (fp16)", rtol=2e-3)
    assert np.all(gsh[~m] == 0)


@pytest.mark.gpu
@pytest.mark.parametrize("half", [False, True], ids=["fp32_sh", "fp16_sh"])
@pytest.mark.parametrize("preexisting_grads", [False, True], ids=["fresh_grads", "accumulate"])
def test_fused_localize_index_path_matches_getter_path(cuda_device, monkeypatch, half, preexisting_grads):
    """`localize` on a boolean mask (the local-edit render, c5): the fused path gathers the subset's rows
    in-kernel (gs_params.index) and scatters the gradients into the full tensors' rows; image, radii,
    screen-space and full-size raw-parameter gradients equal the getter path's (t[mask] gathers +
    autograd scatter), rows outside the mask untouched."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, _fused_ok, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    cam = orbit_camera(1, 5, 200, 136, device=dev)
    G = torch.randn(3, 136, 200, generator=torch.Generator().manual_seed(12)).to(dev)
    outs = []
    for fused in (True, False):
        monkeypatch.setenv("DGE_AMD_FUSED", "1" if fused else "0")
        sc = synthetic_scene(30_000, seed=23, radius=1.5, scale=0.03, device=dev)
        if half:
            sc._features_dc = sc._features_dc.half()
            sc._features_rest = sc._features_rest.half()
        sc.requires_grad_(True)
        mask = torch.zeros(30_000, dtype=torch.bool, device=dev)
        mask[torch.argsort(sc._xyz[:, 0])[:9_000]] = True
        sc.mask, sc.localize = mask, True
        if preexisting_grads:
            for p in sc.parameters():
                p.grad = torch.full_like(p, 0.5)
        assert _fused_ok(sc, PipelineParams()) == fused
        pkg = render(cam, sc, PipelineParams(), torch.tensor([0.1, 0.0, 0.2], device=dev))
        (pkg["render"] * G).sum().backward()
        grads = [p.grad.float().cpu().numpy() for p in sc.parameters()]
        outs.append((pkg["render"].detach().cpu().numpy(), pkg["radii"].cpu().numpy(),
                     pkg["viewspace_points"].grad.cpu().numpy(), grads, mask.cpu().numpy()))
    (img_f, r_f, vs_f, g_f, m), (img_r, r_r, vs_r, g_r, _) = outs
    assert r_f.shape == (9_000,)
    np.testing.assert_array_equal(r_f, r_r)
    assert_close(img_f, img_r, "image", 1e-5)
    assert_close(vs_f, vs_r, "viewspace grad", 1e-4)
    for name, a, b in zip(["_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation"], g_f, g_r):
        # (fp16 feature grads are rounded to fp16 by autograd on both paths)
        assert_close(a, b, name, 2e-3 if half and "features" in name else 1e-4)
        np.testing.assert_array_equal(a[~m], 0.5 if preexisting_grads else 0.0, err_msg=name)


def _axis_camera(W, H, fov_deg=60.0, device="cpu"):
    """Camera at the origin looking down +z (identity view): view-space points are exact."""
    from dge_amd.cameras import get_projection_matrix
    from helpers import settings_from

    fov = math.radians(fov_deg)
    proj = get_projection_matrix(0.01, 100.0, fov, fov).transpose(0, 1).numpy()
    return settings_from(W, H, math.tan(fov / 2), math.tan(fov / 2), (0.0, 0.0, 0.0), np.eye(4, dtype=np.float32),
                         proj, (0.0, 0.0, 0.0), 3, device=device)


def _far_depth_scene(P=4000, zlo=3.0, zhi=6.0):
    rng = np.random.default_rng(11)
    xyz = np.stack([rng.uniform(-1, 1, P), rng.uniform(-1, 1, P), rng.uniform(zlo, zhi, P)], 1).astype(np.float32)
    # Gaussians beyond the 30-bit depth key (>= 2^125 ~ 4.25e37), on the axis (centre tile), in reverse
    # index order of depth, plus a tie: the order must still be the reference's (depth bits, index)
    far = np.array([[0, 0, 9e37], [0, 0, 6e37], [0, 0, 6e37], [0, 0, 5e37], [0.01, 0, 7e37]], np.float32)
    xyz = np.concatenate([xyz, far])
    n = xyz.shape[0]
    rot = rng.standard_normal((n, 4)).astype(np.float32)
    rot /= np.linalg.norm(rot, axis=1, keepdims=True)
    return dict(means3D=xyz, opacities=rng.uniform(0.2, 0.9, (n, 1)).astype(np.float32),
                shs=(rng.standard_normal((n, 16, 3)) * 0.3).astype(np.float32),
                scales=rng.uniform(0.01, 0.05, (n, 3)).astype(np.float32), rotations=rot)


@pytest.mark.parametrize("P,zlo,zhi", [(4000, 3.0, 6.0), (24000, 3.0, 3.5)], ids=["spread", "dense_band"])
def test_depth_beyond_30bit_key_range_keeps_reference_order(cuda_device, oracle, P, zlo, zhi):
    """Depth keys spanning ~30 bits (Gaussians beyond 5e37 beside depths 3..6): the MSD depth buckets are 2^20
    keys wide, so the near Gaussians share a handful of buckets — 'spread': ~1000 per bucket (the in-LDS local
    sort), 'dense_band' (24k Gaussians at depths 3..3.5): ~12k per bucket (the in-kernel global-memory LSD of
    an oversized bucket).  The lists, ranges and every output equal the oracle's (the reference's order)."""
    kw = _far_depth_scene(P, zlo, zhi)
    g = np.random.default_rng(3).standard_normal((3, 96, 96)).astype(np.float32) * 1e-3
    ref = run_oracle(oracle, _axis_camera(96, 96), g, **kw)
    got = run_gpu(_axis_camera(96, 96, device="cuda"), g, **kw)
    assert (ref["radii"][-5:] > 0).sum() >= 4  # the far Gaussians are rendered
    assert got["num_rendered"] == ref["num_rendered"]
    np.testing.assert_array_equal(got["radii"], ref["radii"])
    np.testing.assert_array_equal(got["ranges"], ref["ranges"])
    np.testing.assert_array_equal(got["point_list"], ref["point_list"])
    compare_forward(got, ref, label="far-depth")
    # (the five Gaussians beyond 5e37 overflow float32 in the chain — 1 / t.z near the smallest normal, its
    # square flushed — on either side in ways that differ only in which non-finite or subnormal value comes
    # out; this test is about their depth order, so their gradients are left out of the comparison)
    near = np.ones(ref["radii"].shape[0], bool)
    near[-5:] = False
    compare_grads(got, ref, O=oracle, label="far-depth", rows=near)


def test_forced_32bit_depth_keys_match_30bit_path(cuda_device, monkeypatch):
    """The 32-bit LSD fallback (DGE_AMD_DEPTH_KEYS32=1: four 8-bit passes over the full keys) and the MSD depth
    sort give the same lists and images."""
    a = scene_arrays(100_000, seed=4, radius=2.0, scale=0.02)
    kw = _sh_kw(a)
    s = camera_settings(256, 256, device="cuda")
    base = run_gpu(s, **kw)
    monkeypatch.setenv("DGE_AMD_DEPTH_KEYS32", "1")
    forced = run_gpu(s, **kw)
    for k in ("radii", "ranges", "point_list", "n_contrib", "color", "final_T"):
        np.testing.assert_array_equal(forced[k], base[k], err_msg=k)


@pytest.mark.parametrize("P,W,H,scale", [(3_000, 1920, 1080, 0.02), (300_000, 1920, 1080, 0.02),
                                         (200_000, 2048, 1040, 0.02), (300_000, 1280, 720, 0.02),
                                         (200_000, 1024, 768, 0.02), (300_000, 512, 512, 0.02),
                                         (40_000, 160, 120, 0.02), (100_000, 720, 720, 0.02),
                                         (3_000, 512, 512, 0.15)])
def test_two_level_binning_matches_two_pass_sort(cuda_device, monkeypatch, P, W, H, scale):
    """Grids over 2048 tiles (c4: 120 x 68) bin in two levels — the emission writes the instances in
    tile-column order, one row pass follows, ranges come from per-tile counts; grids of at most 2048 tiles
    (c2: 32 x 32) bin by the direct emission — every instance written straight to its place in its tile's
    list; DGE_AMD_TILE_SORT=2pass runs the emission + the radix tile sort (+ k_ranges) instead.  Lists,
    ranges, the image and every gradient are bitwise the same (3k Gaussians: sort blocks spanning many tile
    columns, whose counts go through the global atomics; 2048 x 1040: the widest grid, 128 columns; 1280 x 720
    and 1024 x 768: 2049..4096 tiles, whose two-pass plan has 6-bit digits while the two-level tables hold
    128 — round 5 found those tables sized for 64, and fixed it; 512 x 512, 160 x 120 and 720 x 720: the
    direct emission's 10-, 8- and 11-bit tile digits; 3k large Gaussians at 512 x 512: blocks whose instances
    span several emission batches)."""
    a = scene_arrays(P, seed=6, radius=2.0, scale=scale)
    g = np.random.default_rng(8).standard_normal((3, H, W)).astype(np.float32) * 1e-3
    s = camera_settings(W, H, device="cuda")
    fused = run_gpu(s, g, **_sh_kw(a))
    monkeypatch.setenv("DGE_AMD_TILE_SORT", "2pass")
    ref = run_gpu(s, g, **_sh_kw(a))
    assert fused["num_rendered"] == ref["num_rendered"] > 0
    for k in ("ranges", "point_list", "n_contrib", "color", "final_T") + tuple(GRAD_NAMES):
        np.testing.assert_array_equal(fused[k], ref[k], err_msg=k)


@pytest.mark.parametrize("P,W,H,scale", [(300_000, 1920, 1080, 0.02), (2_000, 1920, 1080, 0.02),
                                         (200_000, 1280, 720, 0.02), (200_000, 1024, 768, 0.02),
                                         (150_000, 2048, 1536, 0.02), (4_000, 1920, 1080, 0.3),
                                         (60_000, 4000, 400, 0.05)])
def test_region_emission_matches_two_level_binning(cuda_device, monkeypatch, P, W, H, scale):
    """DGE_AMD_BINNING=region (opt-in; slower than the two-level binning at c4) bins grids of 2049..12288 tiles by
    the region emission — per-chunk tile counts, a scan over the chunks, then one workgroup per (depth chunk,
    band of tile rows) expands the chunk's instances in its rows and stores each tile's run straight into the
    lists.  Against the default (two-level binning: column emission + row pass) the (Gaussian, slot) pairs,
    ranges, image and every gradient are bitwise the same, and so is a forward-only render's image (Gaussian ids
    alone in the lists).  2k Gaussians at 1080p: a count table larger than the tile-sort key space it borrows
    (falls back to the two-level binning); 2048 x 1536: 12288 tiles, the largest grid; 4k Gaussians of scale
    0.3: rects spanning many regions and lists of more than one batch; 4000 x 400: 250 tiles wide, beyond the
    two-level binning's 128 columns (the default there is the emission + two-pass tile sort)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    a = scene_arrays(P, seed=6, radius=2.0, scale=scale)
    g = np.random.default_rng(8).standard_normal((3, H, W)).astype(np.float32) * 1e-3
    s = camera_settings(W, H, device="cuda")
    ref = run_gpu(s, g, **_sh_kw(a))
    monkeypatch.setenv("DGE_AMD_BINNING", "region")
    band = run_gpu(s, g, **_sh_kw(a))
    assert band["num_rendered"] == ref["num_rendered"] > 0
    for k in ("ranges", "point_pairs", "n_contrib", "color", "final_T") + tuple(GRAD_NAMES):
        np.testing.assert_array_equal(band[k], ref[k], err_msg=k)
    dev = torch.device("cuda")
    sc = synthetic_scene(P, sh_degree=3, seed=6, scale=scale, device=dev)
    cam = orbit_camera(1, 3, W, H, device=dev)
    bg = torch.tensor([0.1, 0.2, 0.3], device=dev)
    with torch.no_grad():
        one = render(cam, sc, PipelineParams(), bg)
        monkeypatch.delenv("DGE_AMD_BINNING")
        two = render(cam, sc, PipelineParams(), bg)
    torch.cuda.synchronize()
    for k in ("render", "radii", "depth_3dgs"):
        assert torch.equal(one[k], two[k]), k


@pytest.mark.parametrize("W,H", [(4128, 48), (4128, 320)], ids=["single_pass", "two_pass"])
def test_wide_grid_unpacked_rects_vs_oracle(cuda_device, oracle, W, H):
    """Grids more than 255 tiles wide carry tiles_touched instead of a packed rect through the depth sort
    (the emission gathers the rect): 258 x 3 tiles bin by the emission + a single-pass radix tile sort,
    258 x 20 by the emission + two tile-sort passes + k_ranges (too wide for the two-level binning).
    Every forward output equals the oracle's."""
    a = scene_arrays(20_000, seed=12, radius=2.0, scale=0.03)
    kw = _sh_kw(a)
    g = np.random.default_rng(2).standard_normal((3, H, W)).astype(np.float32) * 1e-3
    ref = run_oracle(oracle, camera_settings(W, H), g, **kw)
    got = run_gpu(camera_settings(W, H, device="cuda"), g, **kw)
    assert got["num_rendered"] == ref["num_rendered"] > 0
    compare_forward(got, ref, label=f"wide {W}x{H}")
    compare_grads(got, ref, O=oracle, label=f"wide {W}x{H}")




@pytest.mark.parametrize("localize", [False, True])
def test_semantic_render_reuses_the_training_forward(cuda_device, localize):
    """DGE's semantic render (DGE.py:198-204: the same camera and Gaussians right after the training render,
    the edit mask as override_color, grad mode on) reuses the training forward's preprocess, depth order and
    tile lists (gs_render_recolor: only the blend again): image, depth, radii and visibility bit-identical to
    the full semantic render; a backward through it still works (a full re-render first) and equals the full
    path's; a parameter changed in place (optimizer step) or another camera is never served from the cache.
    localize: the local-edit path (pc[mask] rows, override_color full-P as DGE passes it)."""
    from dge_amd import gaussian_renderer as GR
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    P, W, H = 60_000, 240, 176
    pipe, bg = PipelineParams(), torch.tensor([0.1, 0.0, 0.2], device=dev)
    cams = [orbit_camera(k, 4, W, H, device=dev) for k in range(2)]
    G = torch.randn(3, H, W, generator=torch.Generator().manual_seed(4)).to(dev)

    def scene():
        sc = synthetic_scene(P, seed=31, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
        m = torch.zeros(P, dtype=torch.bool, device=dev)
        m[torch.argsort(sc._xyz[:, 1])[: P // 3]] = True
        sc.mask = m
        sc.localize = localize
        return sc

    def run(reuse):
        GR._RECOLOR = reuse
        sc = scene()
        colors = sc.mask[..., None].float().repeat(1, 3)
        out, hits = [], []
        for cam in cams:
            tr = render(cam, sc, pipe, bg)  # the training render (its buffers stay alive: the graph holds them)
            h0 = GR._RECOLOR_HITS
            sem = render(cam, sc, pipe, bg, override_color=colors)
            hits.append(GR._RECOLOR_HITS - h0)
            out.append({k: sem[k].detach().clone() for k in ("render", "depth_3dgs", "radii", "visibility_filter")})
            out[-1]["train"] = tr["render"].detach().clone()
        # the semantic render of camera 0 after camera 1's forward: not the cached geometry, a full render
        h0 = GR._RECOLOR_HITS
        sem0 = render(cams[0], sc, pipe, bg, override_color=colors)
        hits.append(GR._RECOLOR_HITS - h0)
        # a backward through a (reused) semantic render: the lazy node re-renders in full, then backpropagates
        tr = render(cams[1], sc, pipe, bg)
        sem = render(cams[1], sc, pipe, bg, override_color=colors)
        (sem["render"] * G).sum().backward()
        grads = [p.grad.clone() for p in (sc._xyz, sc._opacity, sc._scaling, sc._rotation)]
        # an in-place parameter update (what an optimizer step is) invalidates the cached forward
        tr = render(cams[0], sc, pipe, bg)
        with torch.no_grad():
            sc._xyz.add_(0.001)
        h0 = GR._RECOLOR_HITS
        sem_after = render(cams[0], sc, pipe, bg, override_color=colors)["render"].detach().clone()
        hits.append(GR._RECOLOR_HITS - h0)
        del tr
        return out, sem0["render"].detach().clone(), grads, sem_after, hits

    prev = GR._RECOLOR
    try:
        got = run(True)
        ref = run(False)
    finally:
        GR._RECOLOR = prev
    assert got[4] == [1, 1, 0, 0], f"recolor hits {got[4]}"
    assert ref[4] == [0, 0, 0, 0]
    for v, (a, b) in enumerate(zip(got[0], ref[0])):
        for k in a:
            assert torch.equal(a[k], b[k]), f"camera {v}: {k}"
        assert not torch.equal(a["render"], a["train"])  # (the mask colours differ from the SH colours)
    assert torch.equal(got[1], ref[1])
    for a, b in zip(got[2], ref[2]):
        assert torch.equal(a, b)
    assert bool(got[2][0].abs().sum() > 0)
    assert torch.equal(got[3], ref[3])


@pytest.mark.parametrize("bg,W,H", [((0.0, 0.0, 0.0), 240, 176), ((0.1, 0.0, 0.2), 240, 176),
                                    ((0.1, 0.0, 0.2), 1024, 768)], ids=["black", "colour", "colour_two_level"])
def test_semantic_render_served_from_the_training_blend(cuda_device, bg, W, H):
    """gs_params.aux_mask: the training render of a model carrying an edit mask also composites the mask as a
    grey along its own alpha / transmittance chain; DGE's semantic render right after it (override_color = the
    mask repeated over the channels, DGE.py:198-204) is composed from those sums after a device-side check of
    the colours — bit-identical to the recolor blend and to a full render.  Other colours (half the mask's
    grey) fail the check and are blended; the training render itself is unchanged by the extra channel.  The
    mask rides as the sign of the Splat depth: every blend, depth and recolor must read |depth| (1024x768: the
    two-level binning's grid)."""
    from dge_amd import gaussian_renderer as GR
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    P = 60_000
    pipe, bgt = PipelineParams(), torch.tensor(bg, device=dev)
    cams = [orbit_camera(k, 4, W, H, device=dev) for k in range(2)]

    def run(aux, recolor):
        GR._AUX, GR._RECOLOR = aux, recolor
        sc = synthetic_scene(P, seed=31, radius=1.5, scale=0.03, device=dev).requires_grad_(True)
        sc.mask = torch.zeros(P, dtype=torch.bool, device=dev)
        sc.mask[torch.argsort(sc._xyz[:, 1])[: P // 3]] = True
        outs = []
        for cam in cams:
            tr = render(cam, sc, pipe, bgt)
            h0 = GR._AUX_HITS
            colors = sc.mask[..., None].float().repeat(1, 3)
            sem = render(cam, sc, pipe, bgt, override_color=colors)
            half = render(cam, sc, pipe, bgt, override_color=colors * 0.5)
            outs.append([t.detach().clone() for t in (tr["render"], tr["depth_3dgs"], sem["render"],
                                                      sem["depth_3dgs"], half["render"])] + [GR._AUX_HITS - h0])
        return outs

    prev = GR._AUX, GR._RECOLOR
    try:
        fused, recolor, full = run(True, True), run(False, True), run(False, False)
    finally:
        GR._AUX, GR._RECOLOR = prev
    names = ("training image", "training depth", "semantic image", "semantic depth", "half-grey image")
    for v in range(len(cams)):
        for i, name in enumerate(names):
            assert torch.equal(fused[v][i], recolor[v][i]), f"camera {v}: {name} (aux vs recolor)"
            assert torch.equal(fused[v][i], full[v][i]), f"camera {v}: {name} (aux vs full render)"
        assert not torch.equal(fused[v][2], fused[v][4])
    assert [o[5] for o in fused] == [2, 2] and [o[5] for o in recolor] == [0, 0]


def test_recolor_never_reuses_a_forward_only_render(cuda_device):
    """A training-shaped render of frozen parameters with grad mode on (the view-space placeholder keeps the
    graph, hence the buffers, alive) runs the forward-only kernels; on a grid over 2048 tiles (1024x768:
    two-level binning) its lists hold Gaussian ids only.  A later override_color render of the same camera
    must not be served from it (gs_render_recolor reads (Gaussian, slot) pairs): no recolor hit, and the
    image, depth and radii are bit-identical to the full render's."""
    from dge_amd import gaussian_renderer as GR
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.scene import synthetic_scene

    dev = torch.device("cuda")
    P, W, H = 200_000, 1024, 768
    cam = orbit_camera(0, 1, W, H, device=dev)
    pipe, bg = PipelineParams(), torch.tensor([0.1, 0.0, 0.2], device=dev)
    sc = synthetic_scene(P, seed=13, radius=1.5, scale=0.03, device=dev)  # frozen: requires_grad False
    colors = (torch.arange(P, device=dev) % 3 == 0)[:, None].float().repeat(1, 3)
    prev = GR._RECOLOR
    try:
        outs = []
        for reuse in (True, False):
            GR._RECOLOR = reuse
            GR._LAST_FORWARD.clear()
            tr = render(cam, sc, pipe, bg)  # grad mode on, nothing trainable: forward_only
            assert tr["viewspace_points"].requires_grad
            h0 = GR._RECOLOR_HITS
            sem = render(cam, sc, pipe, bg, override_color=colors)
            assert GR._RECOLOR_HITS == h0, "a forward-only render was reused"
            outs.append({k: sem[k].detach().clone() for k in ("render", "depth_3dgs", "radii")})
            del tr
        for k in outs[0]:
            assert torch.equal(outs[0][k], outs[1][k]), k
        assert bool(outs[0]["render"].abs().sum() > 0)
    finally:
        GR._RECOLOR = prev
