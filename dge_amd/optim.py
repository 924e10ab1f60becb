"""Fused Adam for the Gaussian parameters.

The reference optimises a GaussianModel with ``torch.optim.Adam(l, lr=0.0,
eps=1e-15)`` over six single-tensor groups (gaussiansplatting/scene/
gaussian_model.py:336-380) and edits the optimizer state in place when it
densifies or prunes (``replace_tensor_to_optimizer``, ``_prune_optimizer``,
``cat_tensors_to_optimizer``, :553-641).  ``FusedAdam`` keeps that contract —
same constructor, ``param_groups`` (with their ``name``/``lr`` keys), and
per-parameter state ``step`` / ``exp_avg`` / ``exp_avg_sq`` — but its step is
ONE gfx950 kernel over every group (``gs_adam_step``, dge_amd/csrc/gs_optim.hip)
instead of torch's per-tensor chain of elementwise kernels.

Arithmetic: torch's foreach Adam (torch/optim/adam.py, the path torch.optim.Adam
takes for GPU tensors) in the float32 operation order its kernels compile to,
with the bias corrections and 1 - beta computed in double on the host as torch
does with Python floats: bit-identical to it (tests/test_gpu_model.py).
Only the configuration the reference uses is supported (weight_decay = 0, no
amsgrad/maximize); anything else raises, as does a CPU tensor: there is no
fallback path.
"""
from __future__ import annotations

import ctypes

import torch

from . import _C
from . import _native as N


class FusedAdam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False, *,
                 maximize=False):
        if weight_decay != 0.0 or amsgrad or maximize:
            raise ValueError("FusedAdam supports weight_decay=0, amsgrad=False, maximize=False "
                             "(the GaussianModel's torch.optim.Adam configuration)")
        if not 0.0 <= eps or not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f"invalid Adam hyper-parameters: betas={betas}, eps={eps}")
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=0.0, amsgrad=False, maximize=False)
        super().__init__(params, defaults)

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        launches = {}  # (device, beta1, beta2, eps) -> [gs_adam_segment]
        keep = []
        for group in self.param_groups:
            beta1, beta2 = group["betas"]
            lr, eps = float(group["lr"]), float(group["eps"])
            for p in group["params"]:
                if p.grad is None:
                    continue
                g = p.grad
                if g.is_sparse:
                    raise RuntimeError("FusedAdam does not support sparse gradients")
                state = self.state[p]
                if len(state) == 0:
                    state["step"] = torch.tensor(0.0, dtype=torch.float32)
                    state["exp_avg"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    state["exp_avg_sq"] = torch.zeros_like(p, memory_format=torch.preserve_format)
                m, v = state["exp_avg"], state["exp_avg_sq"]
                # (the gradient may also be a column block of a row-major gradient bucket: rows at a pitch)
                strided = not g.is_contiguous() and _C.row_pitch_ok(g) and p.dim() >= 1
                for name, t in (("param", p), ("grad", g), ("exp_avg", m), ("exp_avg_sq", v)):
                    if not t.is_cuda:
                        raise RuntimeError(f"FusedAdam: {name} must live on the GPU (no CPU path)")
                    if t.dtype != torch.float32 or t.shape != p.shape or not (t.is_contiguous() or
                                                                              (t is g and strided)):
                        raise RuntimeError(f"FusedAdam: {name} must be a contiguous float32 tensor of the "
                                           f"parameter's shape (the gradient: or rows at a pitch)")
                state["step"] += 1
                t = float(state["step"].item())
                bias_correction1 = 1 - beta1 ** t
                bias_correction2 = 1 - beta2 ** t
                seg = N.AdamSegment()
                seg.param, seg.grad = p.data_ptr(), g.data_ptr()
                seg.exp_avg, seg.exp_avg_sq = m.data_ptr(), v.data_ptr()
                seg.n = p.numel()
                if strided:
                    seg.grad_width, seg.grad_pitch = int(p[0].numel()), int(g.stride(0))
                seg.step_size = lr / bias_correction1
                seg.bias_correction2_sqrt = bias_correction2 ** 0.5
                launches.setdefault((p.device, float(beta1), float(beta2), eps), []).append(seg)
                keep.append((p, g, m, v))
        for (dev, b1, b2, eps), segs in launches.items():
            arr = (N.AdamSegment * len(segs))(*segs)
            stream = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
            N.check(N.lib().gs_adam_step(arr, len(segs), b1, b2, eps, stream), "gs_adam_step")
        del keep
        return loss
