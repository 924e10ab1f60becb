"""GaussianModel host logic on CPU: PLY I/O, learning-rate schedule, densification and
optimizer-state surgery, grad-mask hooks (reference: gaussiansplatting/scene/gaussian_model.py,
utils/general_utils.py).  The reference module itself cannot be imported here (CUDA-only
simple_knn, plyfile), so these tests pin the restatement with known answers computed
independently below; the optimizer for the CPU runs is torch.optim.Adam (the reference's own)."""
import math

import numpy as np
import pytest
import torch

from dge_amd.gaussian_model import GaussianModel, OptimizationParams, get_expon_lr_func, inverse_sigmoid
from dge_amd.ply import attribute_names, read_ply, write_ply
from dge_amd.scene import synthetic_scene


def _model(P=300, deg=3, seed=0):
    sc = synthetic_scene(P, sh_degree=deg, seed=seed)
    m = GaussianModel.from_scene(sc, device="cpu")
    m.spatial_lr_scale = 1.0
    return m


def test_ply_roundtrip_and_layout(tmp_path):
    m = _model(50, deg=3)
    path = str(tmp_path / "pc" / "point_cloud.ply")
    m.save_ply(path)
    raw = open(path, "rb").read()
    head = raw[:raw.index(b"end_header\n") + len(b"end_header\n")].decode()
    assert "format binary_little_endian 1.0" in head and "element vertex 50" in head
    names = [ln.split()[-1] for ln in head.splitlines() if ln.startswith("property")]
    # construct_list_of_attributes order (gaussian_model.py:396-408), 62 float properties at degree 3
    assert names == attribute_names(3, 45) and len(names) == 62
    assert len(raw) - len(head) == 50 * 62 * 4
    m2 = GaussianModel(0, device="cpu").load_ply(path)
    assert m2.max_sh_degree == 3 and m2.active_sh_degree == 3
    for f in GaussianModel._FIELDS:
        assert torch.equal(getattr(m, f).detach(), getattr(m2, f).detach()), f
    # f_dc_k / f_rest_k are channel-major: f_rest_1 is channel 0 of SH coefficient 2
    v = read_ply(path)["vertex"]
    assert np.array_equal(v["f_rest_1"], m._features_rest.detach()[:, 1, 0].numpy())
    assert np.array_equal(v["f_rest_15"], m._features_rest.detach()[:, 0, 1].numpy())


def test_ply_ascii_and_reordered_properties(tmp_path):
    """load_ply sorts f_rest_*/scale_*/rot_* by numeric suffix whatever the file order."""
    names = ["x", "y", "z", "opacity", "f_dc_0", "f_dc_1", "f_dc_2", "rot_1", "rot_0", "rot_3", "rot_2",
             "scale_2", "scale_0", "scale_1"] + [f"f_rest_{i}" for i in (2, 0, 1, 5, 3, 4, 8, 6, 7)]
    rng = np.random.default_rng(0)
    vals = rng.standard_normal((4, len(names))).astype(np.float32)
    lines = ["ply", "format ascii 1.0", "comment made by a test", "element vertex 4"]
    lines += [f"property float {n}" for n in names] + ["end_header"]
    lines += [" ".join(repr(float(x)) for x in row) for row in vals]
    path = tmp_path / "a.ply"
    path.write_text("\n".join(lines) + "\n")
    m = GaussianModel(0, device="cpu").load_ply(str(path))
    col = {n: vals[:, i] for i, n in enumerate(names)}
    assert m.max_sh_degree == 1
    assert np.array_equal(m._rotation.detach().numpy(), np.stack([col[f"rot_{i}"] for i in range(4)], 1))
    assert np.array_equal(m._scaling.detach().numpy(), np.stack([col[f"scale_{i}"] for i in range(3)], 1))
    # rest [P, 3 channels, 3 coeffs] -> [P, coeff, channel]
    rest = np.stack([col[f"f_rest_{i}"] for i in range(9)], 1).reshape(4, 3, 3).transpose(0, 2, 1)
    assert np.array_equal(m._features_rest.detach().numpy(), rest)


def test_write_ply_rejects_unknown_dtype(tmp_path):
    from dge_amd.ply import PlyError

    v = np.zeros(2, dtype=[("x", "c8")])
    with pytest.raises(PlyError):
        write_ply(str(tmp_path / "bad.ply"), v)


def test_expon_lr_schedule_known_answers():
    f = get_expon_lr_func(1e-3, 1e-5, lr_delay_mult=0.01, max_steps=100)
    assert f(-1) == 0.0
    assert math.isclose(f(0), 1e-3, rel_tol=1e-12)
    assert math.isclose(f(100), 1e-5, rel_tol=1e-12)
    assert math.isclose(f(50), math.sqrt(1e-3 * 1e-5), rel_tol=1e-12)
    g = get_expon_lr_func(1e-3, 1e-5, lr_delay_steps=10, lr_delay_mult=0.5, max_steps=100)
    assert math.isclose(g(0), 0.5e-3, rel_tol=1e-12)
    assert math.isclose(g(5), (0.5 + 0.5 * math.sin(0.25 * math.pi)) * 1e-3 ** 0.95 * 1e-5 ** 0.05, rel_tol=1e-12)


def test_expon_lr_schedule_matches_reference_outputs():
    """get_expon_lr_func / inverse_sigmoid against the reference's own functions
    (gaussiansplatting/utils/general_utils.py:18-19, 29-62) evaluated by tools/make_golden.py lr:
    DGE's position schedule, a delayed one, a disabled one and a short one, at steps before, at and past
    every breakpoint -- equal to the last bit (the same numpy double operations)."""
    import os

    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "lr_schedule_ref.npz"))
    for i, (lr_init, lr_final, delay, mult, max_steps) in enumerate(d["cases"]):
        f = get_expon_lr_func(lr_init=float(lr_init), lr_final=float(lr_final), lr_delay_steps=int(delay),
                              lr_delay_mult=float(mult), max_steps=int(max_steps))
        got = np.array([float(f(int(s))) for s in d["steps"]])
        np.testing.assert_array_equal(got, d[f"lr_{i}"], err_msg=f"case {i}")
    x = torch.from_numpy(d["inv_sigmoid_x"])
    np.testing.assert_array_equal(inverse_sigmoid(x).numpy(), d["inv_sigmoid"])


def test_model_learning_rate_follows_reference_schedule():
    """GaussianModel.update_learning_rate sets the xyz group's lr to the reference schedule's value
    (gaussian_model.py:382-389) at each step."""
    import os

    d = np.load(os.path.join(os.path.dirname(__file__), "golden", "lr_schedule_ref.npz"))
    m = GaussianModel(3, device="cpu")
    m.set_parameters(*[torch.zeros(4, *s) for s in ((3,), (1, 3), (15, 3), (1,), (3,), (4,))])
    opt = OptimizationParams(max_steps=30_000)
    m.spatial_lr_scale = 2.5
    m.training_setup(opt, optimizer_cls=torch.optim.Adam)
    lr_init, lr_final, delay, mult, max_steps = d["cases"][0]
    assert math.isclose(opt.position_lr_init * 2.5, lr_init) and math.isclose(opt.position_lr_final * 2.5, lr_final)
    for s, ref in zip(d["steps"], d["lr_0"]):
        if s < 0:
            continue
        m.update_learning_rate(int(s))
        xyz_group = next(g for g in m.optimizer.param_groups if g["name"] == "xyz")
        assert xyz_group["lr"] == ref


def _setup(m):
    m.training_setup(OptimizationParams(max_steps=1000), optimizer_cls=torch.optim.Adam)
    # one optimizer step so every group has state
    for p in m.parameters():
        p.grad = torch.full_like(p, 1e-3)
    m.optimizer.step()
    m.optimizer.zero_grad(set_to_none=True)


def _check_consistent(m):
    P = m._xyz.shape[0]
    for group in m.optimizer.param_groups:
        p = group["params"][0]
        assert p is getattr(m, GaussianModel._GROUPS[group["name"]])
        assert p.shape[0] == P and p.is_leaf and p.requires_grad
        st = m.optimizer.state[p]
        assert st["exp_avg"].shape == p.shape and st["exp_avg_sq"].shape == p.shape
    assert m.mask.shape == (P,) and m._generation.shape == (P,)
    assert m.xyz_gradient_accum.shape == (P, 1) and m.denom.shape == (P, 1) and m.max_radii2D.shape == (P,)


def test_training_setup_groups_and_lr_schedule():
    m = _model(40)
    _setup(m)
    names = [g["name"] for g in m.optimizer.param_groups]
    assert names == ["xyz", "f_dc", "f_rest", "opacity", "scaling", "rotation"]
    lrs = {g["name"]: g["lr"] for g in m.optimizer.param_groups}
    assert math.isclose(lrs["f_rest"], lrs["f_dc"] / 20.0) and lrs["opacity"] == 0.05
    m.update_learning_rate(1000)
    assert math.isclose([g["lr"] for g in m.optimizer.param_groups if g["name"] == "xyz"][0], 0.000016)
    _check_consistent(m)


def test_densify_clone_split_prune_known_counts():
    torch.manual_seed(0)
    P = 300
    m = _model(P)
    _setup(m)
    extent = 2.0
    # gradient statistic: every 3rd Gaussian above the threshold
    grads = torch.zeros(P, 1)
    grads[::3] = 1.0
    m.xyz_gradient_accum = grads.clone()
    m.denom = torch.ones(P, 1)
    scale_max = m.get_scaling.detach().max(dim=1).values
    big = scale_max > m.percent_dense * extent
    sel = grads.squeeze(1) >= 0.5
    n_clone = int((sel & ~big).sum())
    n_split = int((sel & big).sum())
    opac_low = m.get_opacity.detach().squeeze(1) < 0.005
    m.densify_and_clone(grads, 0.5, extent)
    assert m._xyz.shape[0] == P + n_clone
    _check_consistent(m)
    # clones are exact copies appended in index order, new generation
    idx = torch.nonzero(sel & ~big).squeeze(1)
    assert torch.equal(m._xyz.detach()[P:], m._xyz.detach()[idx])
    assert torch.all(m._generation[P:] == 1)
    parents = m.get_scaling.detach()[:P][sel & big]
    m.densify_and_split(grads, 0.5, extent)
    assert m._xyz.shape[0] == P + n_clone - n_split + 2 * n_split
    _check_consistent(m)
    # split children: scale / (0.8 * 2) in activated space, parents removed
    kids = m.get_scaling.detach()[-2 * n_split:]
    assert torch.allclose(kids, torch.cat([parents, parents]) / 1.6, rtol=1e-5)
    n_before = m._xyz.shape[0]
    low = m.get_opacity.detach().squeeze(1) < 0.005
    m.prune_points(low)
    assert m._xyz.shape[0] == n_before - int(low.sum())
    _check_consistent(m)
    assert int(opac_low.sum()) >= 0


def test_densify_and_prune_respects_mask_and_resets_hooks():
    P = 200
    m = _model(P, seed=3)
    _setup(m)
    mask = torch.zeros(P, dtype=torch.bool)
    mask[:100] = True
    m.remove_grad_mask()
    m.apply_grad_mask(mask)
    m.xyz_gradient_accum = torch.ones(P, 1)
    m.denom = torch.ones(P, 1)
    m.densify_and_prune(0.5, 1.0, 0.005, 2.0, 0)
    _check_consistent(m)
    # every Gaussian outside the mask survives unchanged (densify/prune only act inside it)
    assert int((~m.mask).sum()) == 100
    assert len(m.hooks) == 5
    # generation bookkeeping: schedule grew by one, anchor refreshed
    assert m.generation_num == 2 and torch.equal(m.anchor["_xyz"], m._xyz.detach())


def test_grad_mask_hooks_mask_all_but_rotation():
    m = _model(10)
    mask = torch.tensor([True, False] * 5)
    m.remove_grad_mask()
    m.apply_grad_mask(mask)
    loss = sum((p * torch.arange(1, p.numel() + 1, dtype=torch.float32).view_as(p)).sum() for p in m.parameters())
    loss.backward()
    for f in GaussianModel._FIELDS:
        g = getattr(m, f).grad
        if f == "_rotation":
            assert torch.all(g[~mask] != 0)
        else:
            assert torch.all(g[~mask] == 0) and torch.all(g[mask] != 0), f


def test_reset_opacity_and_inverse_sigmoid():
    m = _model(20)
    _setup(m)
    m.reset_opacity()
    assert torch.all(m.get_opacity <= 0.01 + 1e-6)
    x = torch.tensor([0.25, 0.5, 0.75])
    assert torch.allclose(torch.sigmoid(inverse_sigmoid(x)), x)
    _check_consistent(m)
    st = m.optimizer.state[m._opacity]
    assert torch.all(st["exp_avg"] == 0) and torch.all(st["exp_avg_sq"] == 0)


def test_default_optimizer_needs_gpu():
    m = _model(5)
    with pytest.raises(RuntimeError, match="GPU"):
        m.training_setup(OptimizationParams())


def test_fused_adam_rejects_cpu_and_unsupported_options():
    from dge_amd.optim import FusedAdam

    p = torch.nn.Parameter(torch.zeros(4))
    with pytest.raises(ValueError):
        FusedAdam([p], weight_decay=0.1)
    opt = FusedAdam([p], lr=0.1)
    p.grad = torch.ones(4)
    with pytest.raises(RuntimeError, match="GPU"):
        opt.step()
