"""GPU tests of the optimizer step and the grad mask:
FusedAdam (one gfx950 kernel) bit for bit against torch.optim.Adam on the GPU
(the foreach path DGE runs), within 1e-5 of torch.optim.Adam on the CPU — the
oracle SURVEY.md names (ATen's CPU kernels round differently) — and the
GaussianModel's grad-mask hooks applied in-kernel against the same hooks run by
autograd."""
from __future__ import annotations

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def test_fused_adam_matches_torch_adam_gpu_foreach(cuda_device):
    """FusedAdam against the optimizer DGE actually runs: torch.optim.Adam on GPU tensors (the foreach
    implementation; lerp / mul+addcmul / sqrt, div, add / addcdiv).  Reports the bitwise agreement."""
    from dge_amd.optim import FusedAdam

    g = torch.Generator().manual_seed(1)
    shapes = [(1000, 3), (1000, 1, 3), (1000, 15, 3), (1000, 1), (1000, 3), (1001, 4)]
    lrs = [1.6e-4, 0.0125, 0.0125 / 20, 0.05, 0.005, 0.001]
    init = [torch.randn(s, generator=g) for s in shapes]
    ref = [torch.nn.Parameter(t.clone().to(cuda_device)) for t in init]
    dev = [torch.nn.Parameter(t.clone().to(cuda_device)) for t in init]
    mk = lambda ps: [{"params": [p], "lr": lr, "name": f"g{i}"} for i, (p, lr) in enumerate(zip(ps, lrs))]  # noqa
    opt_ref = torch.optim.Adam(mk(ref), lr=0.0, betas=(0.9, 0.99), eps=1e-15)
    opt_dev = FusedAdam(mk(dev), lr=0.0, betas=(0.9, 0.99), eps=1e-15)
    for it in range(5):
        for k, (a, b) in enumerate(zip(ref, dev)):
            gr = (torch.randn(a.shape, generator=g) * (10.0 ** (k % 3 - 2))).to(cuda_device)
            a.grad = gr.clone()
            b.grad = gr.clone()
        opt_ref.step()
        opt_dev.step()
    torch.cuda.synchronize()
    diff = total = 0
    for a, b in zip(ref, dev):
        diff += int((a.detach() != b.detach()).sum())
        total += a.numel()
        for key in ("exp_avg", "exp_avg_sq"):
            diff += int((opt_dev.state[b][key] != opt_ref.state[a][key]).sum())
            total += a.numel()
    print(f"[parity adam] {diff} of {total} parameter/moment elements differ bitwise from torch.optim.Adam (GPU, foreach)")
    assert diff == 0


def test_fused_adam_with_row_major_bucket_grads(cuda_device):
    """The GaussianModel's six parameters with their .grad in a row-major GradBucket (every .grad a column
    block of one [P, 64] matrix: rows at a pitch): FusedAdam (the gathered-gradient segments) against
    torch.optim.Adam (foreach) stepping the same parameters with contiguous copies of the gradients,
    bitwise, over five steps."""
    from dge_amd.multiview import GradBucket
    from dge_amd.optim import FusedAdam

    g = torch.Generator().manual_seed(3)
    shapes = [(1001, 3), (1001, 1, 3), (1001, 15, 3), (1001, 1), (1001, 3), (1001, 4)]
    lrs = [1.6e-4, 0.0125, 0.0125 / 20, 0.05, 0.005, 0.001]
    init = [torch.randn(s, generator=g) for s in shapes]
    ref = [torch.nn.Parameter(t.clone().to(cuda_device)) for t in init]
    dev = [torch.nn.Parameter(t.clone().to(cuda_device)) for t in init]
    bucket = GradBucket(dev)
    assert bucket.rows is not None and not dev[2].grad.is_contiguous()
    mk = lambda ps: [{"params": [p], "lr": lr, "name": f"g{i}"} for i, (p, lr) in enumerate(zip(ps, lrs))]  # noqa
    opt_ref = torch.optim.Adam(mk(ref), lr=0.0, betas=(0.9, 0.99), eps=1e-15)
    opt_dev = FusedAdam(mk(dev), lr=0.0, betas=(0.9, 0.99), eps=1e-15)
    for it in range(5):
        bucket.zero()
        for k, (a, b) in enumerate(zip(ref, dev)):
            gr = (torch.randn(a.shape, generator=g) * (10.0 ** (k % 3 - 2))).to(cuda_device)
            a.grad = gr.clone()
            b.grad.copy_(gr)  # (into the bucket's strided view)
        opt_ref.step()
        opt_dev.step()
    torch.cuda.synchronize()
    for a, b in zip(ref, dev):
        assert torch.equal(a.detach(), b.detach())
        for key in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(opt_dev.state[b][key], opt_ref.state[a][key])


def test_fused_adam_matches_torch_adam_cpu(cuda_device):
    from dge_amd.optim import FusedAdam

    g = torch.Generator().manual_seed(0)
    shapes = [(1000, 3), (1000, 1, 3), (1000, 15, 3), (1000, 1), (1000, 3), (1001, 4), (7,), (3, 5)]
    lrs = [1.6e-4, 0.0125, 0.0125 / 20, 0.05, 0.005, 0.001, 0.1, 0.02]
    ref = [torch.nn.Parameter(torch.randn(s, generator=g)) for s in shapes]
    dev = [torch.nn.Parameter(p.detach().clone().to(cuda_device)) for p in ref]
    mk = lambda ps: [{"params": [p], "lr": lr, "name": f"g{i}"} for i, (p, lr) in enumerate(zip(ps, lrs))]  # noqa
    opt_ref = torch.optim.Adam(mk(ref), lr=0.0, betas=(0.9, 0.99), eps=1e-15)
    opt_dev = FusedAdam(mk(dev), lr=0.0, betas=(0.9, 0.99), eps=1e-15)
    for it in range(5):
        for k, (a, b) in enumerate(zip(ref, dev)):
            if it == 2 and k == 1:  # a parameter without a gradient this step keeps its own step count
                a.grad = b.grad = None
                continue
            gr = torch.randn(a.shape, generator=g) * (10.0 ** (k % 3 - 2))
            a.grad = gr.clone()
            b.grad = gr.to(cuda_device)
        opt_ref.step()
        opt_dev.step()
    torch.cuda.synchronize()
    for a, b in zip(ref, dev):
        sa, sb = opt_ref.state[a], opt_dev.state[b]
        assert float(sa["step"]) == float(sb["step"])
        torch.testing.assert_close(b.detach().cpu(), a.detach(), rtol=1e-5, atol=1e-7)
        # the moments: 1e-5 of the tensor's scale (the lerp's g - m cancels for a few elements, and
        # ATen's CPU lerp may or may not fuse its multiply-add depending on the vector ISA)
        for key in ("exp_avg", "exp_avg_sq"):
            ref_t = sa[key]
            torch.testing.assert_close(sb[key].cpu(), ref_t, rtol=1e-5, atol=1e-5 * float(ref_t.abs().max()))


def test_fused_adam_state_dict_roundtrip(cuda_device):
    from dge_amd.optim import FusedAdam

    p = torch.nn.Parameter(torch.ones(64, device=cuda_device))
    opt = FusedAdam([{"params": [p], "lr": 0.1, "name": "x"}], lr=0.0, eps=1e-15)
    p.grad = torch.ones_like(p)
    opt.step()
    sd = copy.deepcopy(opt.state_dict())  # state_dict() aliases the live state tensors
    q = torch.nn.Parameter(p.detach().clone())
    opt2 = FusedAdam([{"params": [q], "lr": 0.1, "name": "x"}], lr=0.0, eps=1e-15)
    opt2.load_state_dict(sd)
    p.grad = q.grad = torch.full_like(p, 0.5)
    opt.step()
    opt2.step()
    assert torch.equal(p, q)


def _masked_model(dev, P=12_000, seed=4):
    from dge_amd.gaussian_model import GaussianModel
    from dge_amd.scene import synthetic_scene

    m = GaussianModel.from_scene(synthetic_scene(P, seed=seed, radius=1.5, scale=0.03), device=dev)
    mask = torch.rand(P, generator=torch.Generator().manual_seed(seed)) < 0.5
    m.remove_grad_mask()
    m.apply_grad_mask(mask.to(dev))
    return m


def test_grad_mask_in_kernel_matches_autograd_hooks(cuda_device):
    """apply_grad_mask hooks (gaussian_model.py:837-856) keep the fused path; the in-kernel mask gives
    the gradients autograd's hooks give (rotation unmasked, as in the reference)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.diff_gaussian_rasterization import set_fused_grad_accumulation
    from dge_amd.gaussian_renderer import PipelineParams, render

    cams = [orbit_camera(k, 3, 128, 96, device=cuda_device) for k in range(2)]
    G = [torch.randn(3, 96, 128, generator=torch.Generator().manual_seed(9 + k)).to(cuda_device) for k in range(2)]
    bg = torch.zeros(3, device=cuda_device)
    res = {}
    for fused in (True, False):
        prev = set_fused_grad_accumulation(fused)
        try:
            m = _masked_model(cuda_device)
            for c, g in zip(cams, G):
                (render(c, m, PipelineParams(), bg)["render"] * g).sum().backward()
            res[fused] = (m.mask.clone(), [p.grad.clone() for p in m.parameters()])
        finally:
            set_fused_grad_accumulation(prev)
    mask, ga = res[True]
    _, gb = res[False]
    for name, x, y in zip(("xyz", "dc", "rest", "opacity", "scaling", "rotation"), ga, gb):
        torch.testing.assert_close(x, y, rtol=1e-6, atol=1e-9, msg=name)
        if name != "rotation":
            assert torch.all(x[~mask] == 0), name
    assert torch.any(ga[5][~mask] != 0)  # rotation is not masked


def test_edit_step_render_adam_densify(cuda_device):
    """One DGE-style step on the GPU end to end: two views through render(), fused backward into the
    masked model, densification statistics, FusedAdam step, densify_and_prune, and a render after."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_model import OptimizationParams
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.optim import FusedAdam

    m = _masked_model(cuda_device, P=20_000)
    m.spatial_lr_scale = 1.0
    m.training_setup(OptimizationParams(max_steps=100))
    assert isinstance(m.optimizer, FusedAdam)
    bg = torch.zeros(3, device=cuda_device)
    before = [p.detach().clone() for p in m.parameters()]
    radii_max = torch.zeros(m.num_points(), device=cuda_device)
    for k in range(2):
        pkg = render(orbit_camera(k, 2, 128, 128, device=cuda_device), m, PipelineParams(), bg)
        pkg["render"].mean().backward()
        vis = pkg["visibility_filter"]
        radii_max = torch.max(radii_max, pkg["radii"].float())
        m.add_densification_stats(pkg["viewspace_points"].grad, vis)
    m.max_radii2D = radii_max
    m.optimizer.step()
    m.optimizer.zero_grad(set_to_none=True)
    after = [p.detach() for p in m.parameters()]
    assert any(not torch.equal(a, b) for a, b in zip(before, after))
    # masked-out Gaussians do not move (their gradients are zero; Adam with zero state keeps them)
    assert torch.equal(before[0][~m.mask], after[0][~m.mask])
    n0 = m.num_points()
    m.densify_and_prune(1e-7, 1.0, 0.005, 2.0, 0, generator=torch.Generator(device=cuda_device).manual_seed(0))
    assert m.num_points() != n0
    pkg = render(orbit_camera(0, 2, 128, 128, device=cuda_device), m, PipelineParams(), bg)
    assert torch.isfinite(pkg["render"]).all()


@pytest.mark.parametrize("grads_exist", [False, True])
def test_render_views_on_streams_matches_sequential(cuda_device, grads_exist):
    """render_views over a 2-stream pool + ONE backward (each view's backward on its stream, the fused
    .grad writes ordered across them) gives the gradients of the sequential per-view loop, and the
    default stream sees them (read there right after backward returns)."""
    from dge_amd.cameras import orbit_camera
    from dge_amd.gaussian_renderer import PipelineParams, render
    from dge_amd.multiview import render_backward_views, render_views
    from dge_amd.scene import synthetic_scene

    cams = [orbit_camera(k, 4, 160, 128, device=cuda_device) for k in range(4)]
    G = [torch.randn(3, 128, 160, generator=torch.Generator().manual_seed(30 + k)).to(cuda_device) * 1e-2
         for k in range(4)]
    bg = torch.zeros(3, device=cuda_device)
    res = {}
    for mode in ("sequential", "streams", "interleaved", "bucket"):
        sc = synthetic_scene(20_000, seed=4, device=cuda_device).requires_grad_(True)
        if grads_exist:
            for p in sc.parameters():
                p.grad = torch.full_like(p, 0.25)
        if mode == "bucket":
            # the bench's step: forwards on 3 streams, then a dirty flat bucket zeroed on the default stream
            # (only the in-kernel gradient writes wait for it), one backward; grads_exist: 0.25 added after
            from dge_amd.multiview import GradBucket

            bucket = GradBucket(sc.parameters())
            bucket.flat.fill_(7.0)
            outs = render_views(cams, sc, PipelineParams(), bg, streams=3)
            bucket.zero(overlap=True)
            torch.autograd.backward([o["render"] for o in outs], G)
            imgs = [o["render"].detach() for o in outs]
            if grads_exist:
                for p in sc.parameters():
                    p.grad += 0.25
        elif mode == "sequential":
            imgs = []
            for c, g in zip(cams, G):
                out = render(c, sc, PipelineParams(), bg)
                out["render"].backward(g)
                imgs.append(out["render"].detach())
        elif mode == "streams":
            outs = render_views(cams, sc, PipelineParams(), bg, streams=2)
            torch.autograd.backward([o["render"] for o in outs], G)
            imgs = [o["render"].detach() for o in outs]
        else:
            outs = render_backward_views(cams, sc, PipelineParams(), bg, G, streams=2)
            imgs = [o["render"] for o in outs]
        res[mode] = ([p.grad.clone() for p in sc.parameters()], [i.clone() for i in imgs])
    torch.cuda.synchronize()
    for mode in ("streams", "interleaved", "bucket"):
        for a, b in zip(res["sequential"][1], res[mode][1]):
            torch.testing.assert_close(a, b, rtol=0, atol=0, msg=f"image ({mode})")
        for i, (a, b) in enumerate(zip(res["sequential"][0], res[mode][0])):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-7, msg=lambda m: f"parameter {i} ({mode}): {m}")
