"""CPU tests: the oracle pinned against the reference's own functions,
an independent autograd derivation, known-answer scenes and the golden
fixtures.  (No GPU.)"""
from __future__ import annotations

import glob
import math
import os

import numpy as np
import pytest
import torch

from helpers import assert_close, camera_settings, golden_inputs, run_oracle, scene_arrays, settings_from, \
    settings_from_golden

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


# ---------------------------------------------------------------------------
# pinned against the reference's own eval_sh (tests/golden/sh_eval_ref.npz)
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("deg", [0, 1, 2, 3])
def test_sh_matches_reference_eval_sh(oracle, deg):
    z = np.load(os.path.join(GOLDEN, "sh_eval_ref.npz"))
    sh_cm, dirs = z["sh"], z["dirs"]  # reference layout [N, 3, 16]
    ref = z[f"rgb_deg{deg}"]
    shs = np.ascontiguousarray(np.transpose(sh_cm, (0, 2, 1)))  # kernel layout [N, 16, 3]
    campos = np.zeros(3, np.float32)
    pos = dirs * np.float32(2.5)  # direction from campos = dirs
    rgb, clamped = oracle.sh_to_rgb(deg, shs, pos, campos)
    expect = np.maximum(ref + 0.5, 0.0)
    np.testing.assert_allclose(rgb, expect, rtol=2e-6, atol=2e-6)
    np.testing.assert_array_equal(clamped, (ref + 0.5) < 0)


def test_dge_sh_utils_matches_reference(oracle):
    from dge_amd.sh_utils import eval_sh

    z = np.load(os.path.join(GOLDEN, "sh_eval_ref.npz"))
    for deg in range(4):
        got = eval_sh(deg, torch.from_numpy(z["sh"]), torch.from_numpy(z["dirs"])).numpy()
        np.testing.assert_allclose(got, z[f"rgb_deg{deg}"], rtol=1e-6, atol=1e-6)


# ---------------------------------------------------------------------------
# pinned against autograd of an independent dense formulation (tests/torch_ref.py)
# ---------------------------------------------------------------------------
def _pin_scene(P, seed, mode, W=64, H=64, bg=(0.1, 0.2, 0.3), deg=3, mod=1.0):
    a = scene_arrays(P, seed=seed, radius=1.0, scale=0.1, sh_degree=deg)
    # keep alpha below the 0.99 clamp (the reference's opacity gradient ignores it, backward.cu:554)
    a["opacities"] = (0.05 + 0.9 * (a["opacities"] - 0.0)).astype(np.float32) * 0.95
    s = camera_settings(W, H, bg=bg, sh_degree=deg, scale_modifier=mod)
    return a, s


@pytest.mark.parametrize("mode", ["sh", "colors_cov3d"])
def test_oracle_backward_matches_autograd(oracle, mode):
    import torch_ref as TR

    P, W, H = 300, 64, 64
    a, s = _pin_scene(P, 3 if mode == "sh" else 4, mode, W, H)
    rng = np.random.default_rng(2)
    G = rng.standard_normal((3, H, W)).astype(np.float32)
    if mode == "sh":
        kw = dict(shs=a["shs"], scales=a["scales"], rotations=a["rotations"])
    else:
        colors = rng.random((P, 3)).astype(np.float32)
        kw = dict(colors_precomp=colors, cov3D_precomp=a["cov3D"])
    ref = run_oracle(oracle, s, G, means3D=a["means3D"], opacities=a["opacities"], **kw)

    leaf = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in kw.items()}
    m3 = torch.tensor(a["means3D"], dtype=torch.float64, requires_grad=True)
    op = torch.tensor(a["opacities"], dtype=torch.float64, requires_grad=True)
    m2 = torch.zeros(P, 3, dtype=torch.float64, requires_grad=True)
    c, d, radii, nc = TR.dense_render(m3, op, s, shs=leaf.get("shs"), colors=leaf.get("colors_precomp"),
                                      scales=leaf.get("scales"), rotations=leaf.get("rotations"),
                                      cov3D=leaf.get("cov3D_precomp"), means2D=m2)
    np.testing.assert_array_equal(radii, ref["radii"])
    np.testing.assert_array_equal(nc.reshape(-1), ref["n_contrib"])
    assert_close(ref["color"], c.detach().numpy(), "color", 1e-5)
    assert_close(ref["depth"], d.detach().numpy(), "depth", 1e-5)
    (c * torch.as_tensor(G, dtype=torch.float64)).sum().backward()
    assert_close(ref["dL_dmeans3D"], m3.grad.numpy(), "dL_dmeans3D", 1e-4)
    assert_close(ref["dL_dopacity"].reshape(-1), op.grad.numpy().reshape(-1), "dL_dopacity", 1e-4)
    assert_close(ref["dL_dmeans2D"], m2.grad.numpy(), "dL_dmeans2D", 1e-4)
    if mode == "sh":
        assert_close(ref["dL_dsh"], leaf["shs"].grad.numpy(), "dL_dsh", 1e-4)
        assert_close(ref["dL_dscales"], leaf["scales"].grad.numpy(), "dL_dscales", 1e-4)
        assert_close(ref["dL_drotations"], leaf["rotations"].grad.numpy(), "dL_drotations", 1e-4)
    else:
        assert_close(ref["dL_dcolors"], leaf["colors_precomp"].grad.numpy(), "dL_dcolors", 1e-4)
        assert_close(ref["dL_dcov3D"], leaf["cov3D_precomp"].grad.numpy(), "dL_dcov3D", 1e-4)


# ---------------------------------------------------------------------------
# known-answer scenes
# ---------------------------------------------------------------------------
def _front_settings(W=64, H=64, bg=(0.0, 0.0, 0.0), deg=0):
    """Camera at the origin looking down +z (R = I, T = 0)."""
    from dge_amd.cameras import Camera
    from dge_amd.gaussian_renderer import _settings

    cam = Camera(np.eye(3), np.zeros(3), math.radians(60), math.radians(60), H, W, device="cpu")
    return _settings(cam, torch.tensor(bg, dtype=torch.float32), 1.0, deg)


def _iso(z, s, o, color, n=1, dz=0.0):
    P = n
    m = np.zeros((P, 3), np.float32)
    m[:, 2] = z + dz * np.arange(P)
    return dict(means3D=m, opacities=np.full((P, 1), o, np.float32),
                colors_precomp=np.tile(np.asarray(color, np.float32), (P, 1)),
                scales=np.full((P, 3), s, np.float32),
                rotations=np.tile(np.array([1, 0, 0, 0], np.float32), (P, 1)))


def _analytic_single(W, H, z, s, o, color, settings):
    fx = W / (2 * settings.tanfovx)
    sig2 = (fx * s / z) ** 2 + 0.3
    cx = ((0.0 + 1.0) * W - 1.0) * 0.5
    yy, xx = np.mgrid[0:H, 0:W].astype(np.float64)
    d2 = (cx - xx) ** 2 + (cx - yy) ** 2
    alpha = np.minimum(0.99, o * np.exp(-0.5 * d2 / sig2))
    alpha = np.where(alpha < 1 / 255, 0.0, alpha)
    lam = sig2 + math.sqrt(0.1)
    r = math.ceil(3 * math.sqrt(lam))
    x0, x1 = max(0, int((cx - r) / 16)), min(W // 16, int((cx + r + 15) / 16))
    mask = np.zeros((H, W), bool)
    mask[x0 * 16:x1 * 16, x0 * 16:x1 * 16] = True
    alpha = np.where(mask, alpha, 0.0)
    return np.stack([alpha * c for c in color]), alpha


def test_kat_single_isotropic_gaussian(oracle):
    W = H = 64
    s = _front_settings(W, H)
    sc = _iso(2.0, 0.05, 0.8, (1.0, 0.5, 0.25))
    out = run_oracle(oracle, s, **sc)
    expect, alpha = _analytic_single(W, H, 2.0, 0.05, 0.8, (1.0, 0.5, 0.25), s)
    np.testing.assert_allclose(out["color"], expect, rtol=1e-5, atol=1e-6)
    assert out["num_rendered"] == 4 and out["radii"][0] == 5


@pytest.mark.parametrize("side", [-1, 1])
def test_kat_alpha_threshold_edge(oracle, side):
    W = H = 64
    s = _front_settings(W, H)
    fx = W / (2 * s.tanfovx)
    sig2 = (fx * 0.05 / 2.0) ** 2 + 0.3
    g_center = math.exp(-0.5 * 0.5 / sig2)  # the four centre pixels sit at d = (0.5, 0.5)
    o = (1.0 / 255.0) / g_center * (1 + side * 1e-3)
    out = run_oracle(oracle, s, **_iso(2.0, 0.05, o, (1.0, 1.0, 1.0)))
    centre = out["color"][0, 31, 31]
    if side < 0:
        assert centre == 0.0 and out["n_contrib"].max() == 0
    else:
        assert centre > 0.0 and abs(centre - o * g_center) < 1e-6


def test_kat_early_termination(oracle):
    W = H = 64
    s = _front_settings(W, H)
    n = 12
    sc = _iso(2.0, 0.05, 0.9, (1.0, 0.0, 0.0), n=n, dz=0.01)
    sc["colors_precomp"] = np.stack([np.array([k / n, 1 - k / n, 0.5], np.float32) for k in range(n)])
    out = run_oracle(oracle, s, **sc)
    fx = W / (2 * s.tanfovx)
    T, C, last = 1.0, np.zeros(3), 0
    for k in range(n):
        z = 2.0 + 0.01 * k
        sig2 = (fx * 0.05 / z) ** 2 + 0.3
        a = min(0.99, 0.9 * math.exp(-0.5 * 0.5 / sig2))
        if T * (1 - a) < 1e-4:
            break
        C += sc["colors_precomp"][k] * a * T
        T *= 1 - a
        last = k + 1
    assert out["n_contrib"].reshape(H, W)[31, 31] == last and last < n
    np.testing.assert_allclose(out["color"][:, 31, 31], C, rtol=1e-5, atol=1e-6)
    assert abs(out["final_T"].reshape(H, W)[31, 31] - T) < 1e-7


def test_kat_depth_ties_keep_index_order(oracle):
    W = H = 64
    s = _front_settings(W, H)
    sc = _iso(2.0, 0.05, 0.7, (1.0, 0.0, 0.0), n=2)
    sc["colors_precomp"] = np.array([[1, 0, 0], [0, 1, 0]], np.float32)
    out = run_oracle(oracle, s, **sc)
    fx = W / (2 * s.tanfovx)
    a = 0.7 * math.exp(-0.5 * 0.5 / ((fx * 0.05 / 2.0) ** 2 + 0.3))
    np.testing.assert_allclose(out["color"][:, 31, 31], [a, a * (1 - a), 0.0], rtol=1e-5, atol=1e-7)


def test_kat_near_plane(oracle):
    s = _front_settings(64, 64)
    for z, vis in [(0.2, False), (0.2001, True)]:
        out = run_oracle(oracle, s, **_iso(z, 0.001, 0.5, (1, 1, 1)))
        assert (out["radii"][0] > 0) == vis, z
    assert not oracle.mark_visible(np.array([[0, 0, 0.2]], np.float32), s.viewmatrix, s.projmatrix)[0]


def test_empty_and_culled_scenes(oracle):
    s = _front_settings(48, 40, bg=(0.3, 0.2, 0.1))
    empty = dict(means3D=np.zeros((0, 3), np.float32), opacities=np.zeros((0, 1), np.float32),
                 colors_precomp=np.zeros((0, 3), np.float32), scales=np.zeros((0, 3), np.float32),
                 rotations=np.zeros((0, 4), np.float32))
    out = run_oracle(oracle, s, **empty)  # P == 0: zero image, not bg (rasterize_points.cu:57-72)
    assert out["num_rendered"] == 0 and not out["color"].any()
    behind = _iso(-3.0, 0.05, 0.9, (1, 1, 1), n=5)
    out = run_oracle(oracle, s, np.ones((3, 40, 48), np.float32), **behind)
    assert out["num_rendered"] == 0
    np.testing.assert_allclose(out["color"], np.broadcast_to(np.array([0.3, 0.2, 0.1])[:, None, None], (3, 40, 48)),
                               rtol=1e-7)
    assert not out["dL_dmeans3D"].any() and not out["dL_dopacity"].any()


def test_ragged_image_matches_dense_reference(oracle):
    import torch_ref as TR

    a = scene_arrays(200, seed=9, radius=1.0, scale=0.1, sh_degree=2)
    s = camera_settings(100, 37, sh_degree=2, bg=(0.0, 0.1, 0.0))
    shs = a["shs"][:, :9]
    out = run_oracle(oracle, s, means3D=a["means3D"], opacities=a["opacities"], shs=shs, scales=a["scales"],
                     rotations=a["rotations"])
    c, d, radii, nc = TR.dense_render(torch.from_numpy(a["means3D"]), torch.from_numpy(a["opacities"]), s,
                                      shs=torch.from_numpy(shs), scales=torch.from_numpy(a["scales"]),
                                      rotations=torch.from_numpy(a["rotations"]))
    np.testing.assert_array_equal(radii, out["radii"])
    assert_close(out["color"], c.numpy(), "color", 1e-5)


# ---------------------------------------------------------------------------
# golden fixtures: the oracle still reproduces what was committed
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("path", sorted(glob.glob(os.path.join(GOLDEN, "scene_*.npz"))), ids=os.path.basename)
def test_oracle_reproduces_golden(oracle, path):
    rec = np.load(path)
    s = settings_from_golden(rec)
    out = run_oracle(oracle, s, rec["dL_dpix"], **golden_inputs(rec))
    assert out["num_rendered"] == int(rec["num_rendered"])
    np.testing.assert_array_equal(out["radii"], rec["radii"])
    np.testing.assert_array_equal(out["point_list"], rec["point_list"])
    for k in ("color", "depth", "final_T", "dL_dmeans3D", "dL_dsh", "dL_dscales", "dL_drotations", "dL_dopacity",
              "dL_dcov3D", "dL_dmeans2D", "dL_dcolors"):
        assert_close(out[k], rec[k], k, 1e-6)


def test_apply_weights_counts(oracle):
    W = H = 64
    s = _front_settings(W, H)
    sc = _iso(2.0, 0.05, 0.8, (1, 1, 1))
    iw = np.ones((1, H, W), np.float32)
    w, cnt = oracle.apply_weights(s, sc["means3D"], sc["opacities"], np.zeros((1, 1), np.float32),
                                  np.zeros((1,), np.int32), iw, scales=sc["scales"], rotations=sc["rotations"])
    _, alpha = _analytic_single(W, H, 2.0, 0.05, 0.8, (1, 1, 1), s)
    assert cnt[0] == int((alpha > 0).sum()) and abs(w[0, 0] - (alpha > 0).sum()) < 1e-3


def test_chain_magnitudes_bound_the_chain(oracle):
    """oracle.backward_chain_mag (the chain in absolute arithmetic, the scale of the per-element gradient bar
    of test_c2_render_raw_parameter_grads_per_element) bounds the float chain for any sums within the
    magnitudes: for random g with |g| <= m9, |chain(g)| <= chain_mag(m9) (to the chain's own rounding);
    it is zero for the Gaussians that are not rendered."""
    a = scene_arrays(3000, seed=12, radius=4.0, scale=0.05)
    s = camera_settings(160, 120)
    nr, _, _, radii, st = oracle.forward(s, means3D=a["means3D"], opacities=a["opacities"], shs=a["shs"],
                                         scales=a["scales"], rotations=a["rotations"])
    g = np.random.default_rng(3).standard_normal((3, 120, 160)).astype(np.float32)
    ref = oracle.backward(st, g)
    m9 = ref["mag9"]
    mag = oracle.backward_chain_mag(st, m9)
    rng = np.random.default_rng(4)
    for _ in range(4):
        g9 = (m9 * rng.uniform(-1, 1, m9.shape)).astype(np.float32)
        ch = oracle.backward_chain(st, g9)
        for n in ("dL_dmeans3D", "dL_dcov3D", "dL_dsh", "dL_dscales", "dL_drotations"):
            assert np.all(np.abs(ch[n]) <= mag[n] * (1 + 1e-5) + 1e-30), n
    dead = radii == 0
    assert dead.any() and (~dead).any()
    for n in ("dL_dmeans3D", "dL_dscales", "dL_drotations"):
        assert not mag[n][dead].any()
        assert (mag[n][~dead & (m9.max(1) > 0)] > 0).any()


def test_blend_exp_accuracy(oracle):
    """The blend's exp (gs_expf: fused shifter, degree-7 Horner, exact 2^n scale) against fp64 exp: <= 0.86 ulp
    over every 97th float of [-6, 0) (the live range of alpha = o G >= 1/255; every float measured 0.854 in
    round 5), <= 1 ulp on [-10, 1]; NaN -> NaN; far below the live range a value < 1/255 (skipped)."""
    lo = np.array(-6.0, np.float32).view(np.uint32)
    x = np.arange(0x80000001, int(lo), 97, dtype=np.uint32).view(np.float32)  # -tiny .. -6
    x = np.concatenate([x, np.random.default_rng(0).uniform(-10, 1, 1_000_000).astype(np.float32)])
    y = oracle.expf(x)
    ref = np.exp(x.astype(np.float64))
    ulps = np.abs(y.astype(np.float64) - ref) / np.spacing(ref.astype(np.float32)).astype(np.float64)
    assert ulps[: -1_000_000].max() <= 0.86 and ulps.max() <= 1.0, ulps.max()
    odd = oracle.expf(np.array([np.nan, -np.inf, -1e30, -200.0, -90.0, -83.5], np.float32))
    assert np.isnan(odd[0]) and np.all(odd[1:] < 1.0 / 255.0)


# ---------------------------------------------------------------------------
# the fp64 truth of the per-element gradient bar (oracle/gs_truth.c, tests/helpers.py truth_bar)
# ---------------------------------------------------------------------------
def test_truth_matches_dense_float64_autograd(oracle):
    """The truth (backward.cu's formulas in double at the float forward's state) against autograd of the
    independent dense float64 formulation (tests/torch_ref.py, which also recomputes the forward in double):
    equal to the forward state's float rounding, <= 1e-5 x (|autograd| + the terms' magnitude) per element
    (measured ~1.5e-6); the double sums agree with the oracle's double sums of its float terms to the terms'
    own float rounding (<= 1e-5 x magnitude)."""
    import torch_ref as TR

    P, W, H = 300, 64, 64
    a, s = _pin_scene(P, 3, "sh", W, H)
    G = np.random.default_rng(2).standard_normal((3, H, W)).astype(np.float32)
    kw = dict(shs=a["shs"], scales=a["scales"], rotations=a["rotations"])
    ref = run_oracle(oracle, s, G, means3D=a["means3D"], opacities=a["opacities"], **kw)
    st = ref["state"]
    tb = oracle.backward_truth(st, G)
    from helpers import raster_sums

    mag9 = ref["mag9"].astype(np.float64)
    assert np.all(np.abs(tb["sums_d"] - raster_sums(ref)) <= 1e-5 * mag9 + 1e-30)
    ch = oracle.backward_chain_f64(st, tb["sums_d"])
    leaf = {k: torch.tensor(v, dtype=torch.float64, requires_grad=True) for k, v in kw.items()}
    m3 = torch.tensor(a["means3D"], dtype=torch.float64, requires_grad=True)
    op = torch.tensor(a["opacities"], dtype=torch.float64, requires_grad=True)
    m2 = torch.zeros(P, 3, dtype=torch.float64, requires_grad=True)
    c, _, _, _ = TR.dense_render(m3, op, s, means2D=m2, **leaf)
    (c * torch.as_tensor(G, dtype=torch.float64)).sum().backward()
    mag = oracle.backward_chain_mag(st, ref["mag9"])
    for name, t, ag, m in [("dL_dmeans3D", ch["dL_dmeans3D"], m3.grad, mag["dL_dmeans3D"]),
                           ("dL_dsh", ch["dL_dsh"], leaf["shs"].grad, mag["dL_dsh"]),
                           ("dL_dscales", ch["dL_dscales"], leaf["scales"].grad, mag["dL_dscales"]),
                           ("dL_drotations", ch["dL_drotations"], leaf["rotations"].grad, mag["dL_drotations"]),
                           ("dL_dopacity", tb["sums_d"][:, 5], op.grad.reshape(-1), mag9[:, 5]),
                           ("dL_dmeans2D", tb["sums_d"][:, :2], m2.grad[:, :2], mag9[:, :2])]:
        ag = ag.numpy()
        worst = float((np.abs(t - ag) / (np.abs(ag) + m + 1e-300)).max())
        assert worst <= 1e-5, f"{name}: truth vs dense float64 autograd {worst:.3g}"


def test_truth_bar_admits_the_references_arithmetic_and_catches_an_error(oracle):
    """Every fp32 evaluation of the reference's backward (3 contraction models x (the double sum rounded + 4
    atomic arrival orders)) lies within 1e-4 x magnitude of the truth's rasterizer sums; the bar admits one of
    them as `got`, and rejects it once 5% of its elements carry a relative error of 5e-4."""
    from dge_amd.gaussian_renderer import _settings
    from dge_amd.cameras import orbit_camera
    from dge_amd.scene import synthetic_scene
    from helpers import PARAM_NAMES, truth_bar, truth_case

    W, H = 128, 128
    sc = synthetic_scene(20_000, seed=3, radius=1.5, scale=0.03)
    raw = dict(zip(PARAM_NAMES, [p.detach() for p in sc.parameters()]))
    with torch.no_grad():
        op, scl, rot = sc.get_opacity, sc.get_scaling, sc.get_rotation
    s = _settings(orbit_camera(0, 1, W, H, device="cpu"), torch.zeros(3), 1.0, 3)
    shs = torch.cat([raw["_features_dc"], raw["_features_rest"]], 1).numpy()
    _, _, _, _, st = oracle.forward(s, means3D=raw["_xyz"].numpy(), opacities=op.numpy(), shs=shs,
                                    scales=scl.numpy(), rotations=rot.numpy())
    G = np.random.default_rng(5).standard_normal((3, H, W)).astype(np.float32)
    base = oracle.backward(st, G)
    tb = oracle.backward_truth(st, G)
    mag9 = base["mag9"].astype(np.float64)
    for model in oracle.MODELS:
        t = oracle.backward_truth(st, G, model=model, double=False)
        for o in range(oracle.TRUTH_ORDERS):
            assert np.all(np.abs(t["sums_f"][o] - tb["sums_d"]) <= 1e-4 * mag9 + 1e-30), (model, o)
    truth, refs, names, rows = truth_case(oracle, st, G, raw)
    assert len(refs) == 3 * (1 + oracle.TRUTH_ORDERS) and len(rows) > 1000
    k = names.index("fma_clang:order3")
    got = refs[k]
    others = [r for j, r in enumerate(refs) if j != k]
    onames = [n for j, n in enumerate(names) if j != k]
    truth_bar(got, truth, others, "self", names=onames)
    rng = np.random.default_rng(0)
    bad = {n: v * np.where(rng.random(v.shape) < 0.05, 1 + 5e-4, 1.0) for n, v in got.items()}
    with pytest.raises(AssertionError):
        truth_bar(bad, truth, others, "perturbed", names=onames)
