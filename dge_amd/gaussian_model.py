"""GaussianModel: the trainable Gaussian scene around the rasterizer.

Restates gaussiansplatting/scene/gaussian_model.py of the reference — the
part DGE's edit loop drives between two renders:
  * optimizer setup and the xyz learning-rate schedule (:336-394), with the
    Adam step as ONE gfx950 kernel (dge_amd.optim.FusedAdam) instead of
    torch.optim.Adam's per-tensor kernel chain;
  * densification: clone / split / prune and the optimizer-state surgery that
    goes with them (:553-815), generation bookkeeping and the anchor loss
    (:92-184);
  * the grad-mask hooks (:834-863) — tagged so the rasterizer's backward
    applies the mask in-kernel and keeps its fused gradient accumulation;
  * PLY I/O (:396-551) through dge_amd.ply (plyfile is not available here).
Out of scope (not on the rasterizer path): create_from_pcd (simple-knn),
get_near_gaussians_by_mask / concat_gaussians (KNN helpers).
"""
from __future__ import annotations

import os

import numpy as np
import torch
from torch import nn

from .ply import gaussians_to_vertex, read_ply, vertex_to_gaussians, write_ply
from .scene import GaussianScene, build_rotation

MAX_ANCHOR_WEIGHT = 10  # gaussian_model.py:37


def inverse_sigmoid(x):
    """general_utils.py:18-19."""
    return torch.log(x / (1 - x))


def get_expon_lr_func(lr_init, lr_final, lr_delay_steps=0, lr_delay_mult=1.0, max_steps=1000000):
    """general_utils.py:29-65: log-linear decay from lr_init to lr_final with an optional delay."""

    def helper(step):
        if step < 0 or (lr_init == 0.0 and lr_final == 0.0):
            return 0.0
        if lr_delay_steps > 0:
            delay_rate = lr_delay_mult + (1 - lr_delay_mult) * np.sin(0.5 * np.pi * np.clip(step / lr_delay_steps, 0, 1))
        else:
            delay_rate = 1.0
        t = np.clip(step / max_steps, 0, 1)
        log_lerp = np.exp(np.log(lr_init) * (1 - t) + np.log(lr_final) * t)
        return delay_rate * log_lerp

    return helper


class OptimizationParams:
    """arguments/__init__.py:71-89 (the values, without the argparse plumbing)."""

    def __init__(self, max_steps=30_000, lr_scaler=1, lr_final_scaler=1, color_lr_scaler=1, opacity_lr_scaler=1,
                 scaling_lr_scaler=1, rotation_lr_scaler=1):
        self.iterations = max_steps
        self.position_lr_init = 0.00016 * lr_scaler
        self.position_lr_final = 0.000016 * lr_final_scaler
        self.position_lr_delay_mult = 0.01
        self.position_lr_max_steps = max_steps
        self.feature_lr = 0.0125 * color_lr_scaler
        self.opacity_lr = 0.05 * opacity_lr_scaler
        self.scaling_lr = 0.005 * scaling_lr_scaler
        self.rotation_lr = 0.001 * rotation_lr_scaler
        self.percent_dense = 0.01
        self.lambda_dssim = 0.2
        self.densification_interval = 100
        self.opacity_reset_interval = 3000
        self.densify_from_iter = 500
        self.densify_until_iter = 15_000
        self.densify_grad_threshold = 0.0002


def _default_optimizer(params, device):
    if device.type == "cuda":
        from .optim import FusedAdam

        return FusedAdam(params, lr=0.0, eps=1e-15)
    raise RuntimeError("GaussianModel.training_setup: the product optimizer (FusedAdam) runs on the GPU only; "
                       "pass optimizer_cls= explicitly for CPU use")


class GaussianModel(GaussianScene):
    _FIELDS = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")
    _GROUPS = {"xyz": "_xyz", "f_dc": "_features_dc", "f_rest": "_features_rest", "opacity": "_opacity",
               "scaling": "_scaling", "rotation": "_rotation"}
    # gaussian_model.py:851: the grad-mask hooks cover every field but _rotation
    _MASKED_FIELDS = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling")

    def __init__(self, sh_degree: int, anchor_weight_init_g0: float = 1.0, anchor_weight_init: float = 0.1,
                 anchor_weight_multiplier: float = 2.0, device="cuda"):
        e = torch.empty(0, device=device)
        super().__init__(e, e, e, e, e, e, sh_degree=sh_degree)
        self.device = torch.device(device)
        self.active_sh_degree = 0
        self.anchor_weight_init = anchor_weight_init
        self.anchor_weight_multiplier = anchor_weight_multiplier
        self.anchor_weight_init_g0 = anchor_weight_init_g0
        self._anchor_loss_schedule = torch.tensor([anchor_weight_init_g0], device=self.device)
        self._generation = torch.empty(0, dtype=torch.int64, device=self.device)
        self.max_radii2D = torch.empty(0, device=self.device)
        self.xyz_gradient_accum = torch.empty(0, device=self.device)
        self.denom = torch.empty(0, device=self.device)
        self.optimizer = None
        self.percent_dense = 0
        self.spatial_lr_scale = 0
        self.anchor = {}
        self.hooks = []
        self.scaling_activation, self.scaling_inverse_activation = torch.exp, torch.log
        self.opacity_activation, self.inverse_opacity_activation = torch.sigmoid, inverse_sigmoid
        self.rotation_activation = torch.nn.functional.normalize

    # -- construction -------------------------------------------------------
    def set_parameters(self, xyz, features_dc, features_rest, opacity, scaling, rotation, active_sh_degree=None):
        """Raw tensors -> leaf nn.Parameters (what load_ply / create_from_pcd end with, :505-551)."""
        dev = self.device
        for name, t in zip(self._FIELDS, (xyz, features_dc, features_rest, opacity, scaling, rotation)):
            setattr(self, name, nn.Parameter(torch.as_tensor(t, dtype=torch.float32, device=dev).contiguous()
                                             .requires_grad_(True)))
        P = self._xyz.shape[0]
        self.active_sh_degree = self.max_sh_degree if active_sh_degree is None else active_sh_degree
        self.max_radii2D = torch.zeros(P, device=dev)
        self._generation = torch.zeros(P, dtype=torch.int64, device=dev)
        self.set_mask(torch.ones(P, dtype=torch.bool, device=dev))
        self.apply_grad_mask(self.mask)
        self.update_anchor()
        return self

    @classmethod
    def from_scene(cls, scene: GaussianScene, device=None):
        m = cls(scene.max_sh_degree, device=device or scene._xyz.device)
        return m.set_parameters(scene._xyz.detach(), scene._features_dc.detach(), scene._features_rest.detach(),
                                scene._opacity.detach(), scene._scaling.detach(), scene._rotation.detach(),
                                scene.active_sh_degree)

    def parameters(self):
        return [getattr(self, n) for n in self._FIELDS]

    # -- optimizer (:336-394) -----------------------------------------------
    def training_setup(self, training_args, optimizer_cls=None):
        self.percent_dense = training_args.percent_dense
        P = self._xyz.shape[0]
        self.xyz_gradient_accum = torch.zeros((P, 1), device=self.device)
        self.denom = torch.zeros((P, 1), device=self.device)
        lr = {"xyz": training_args.position_lr_init * self.spatial_lr_scale, "f_dc": training_args.feature_lr,
              "f_rest": training_args.feature_lr / 20.0, "opacity": training_args.opacity_lr,
              "scaling": training_args.scaling_lr, "rotation": training_args.rotation_lr}
        groups = [{"params": [getattr(self, f)], "lr": lr[n], "name": n} for n, f in self._GROUPS.items()]
        self.params_list = groups
        if optimizer_cls is None:
            self.optimizer = _default_optimizer(groups, self.device)
        else:
            self.optimizer = optimizer_cls(groups, lr=0.0, eps=1e-15)
        self.xyz_scheduler_args = get_expon_lr_func(
            lr_init=training_args.position_lr_init * self.spatial_lr_scale,
            lr_final=training_args.position_lr_final * self.spatial_lr_scale,
            lr_delay_mult=training_args.position_lr_delay_mult, max_steps=training_args.position_lr_max_steps)

    def update_learning_rate(self, iteration):
        for group in self.optimizer.param_groups:
            if group["name"] == "xyz":
                group["lr"] = self.xyz_scheduler_args(iteration)

    def capture(self):
        return (self.active_sh_degree, self._xyz, self._features_dc, self._features_rest, self._scaling,
                self._rotation, self._opacity, self.max_radii2D, self.xyz_gradient_accum, self.denom,
                self.optimizer.state_dict(), self.spatial_lr_scale)

    def restore(self, model_args, training_args):
        (self.active_sh_degree, self._xyz, self._features_dc, self._features_rest, self._scaling, self._rotation,
         self._opacity, self.max_radii2D, xyz_gradient_accum, denom, opt_dict, self.spatial_lr_scale) = model_args
        self.xyz_gradient_accum = xyz_gradient_accum
        self.denom = denom
        self.optimizer.load_state_dict(opt_dict)

    def oneupSHdegree(self):
        if self.active_sh_degree < self.max_sh_degree:
            self.active_sh_degree += 1

    # -- optimizer-state surgery (:553-641) -----------------------------------
    def replace_tensor_to_optimizer(self, tensor, name):
        out = {}
        for group in self.optimizer.param_groups:
            if group["name"] == name:
                stored = self.optimizer.state.get(group["params"][0], None)
                stored["exp_avg"] = torch.zeros_like(tensor)
                stored["exp_avg_sq"] = torch.zeros_like(tensor)
                del self.optimizer.state[group["params"][0]]
                group["params"][0] = nn.Parameter(tensor.requires_grad_(True))
                self.optimizer.state[group["params"][0]] = stored
                out[group["name"]] = group["params"][0]
        return out

    def _prune_optimizer(self, mask):
        out = {}
        for group in self.optimizer.param_groups:
            stored = self.optimizer.state.get(group["params"][0], None)
            if stored is not None:
                stored["exp_avg"] = stored["exp_avg"][mask]
                stored["exp_avg_sq"] = stored["exp_avg_sq"][mask]
                del self.optimizer.state[group["params"][0]]
                group["params"][0] = nn.Parameter(group["params"][0][mask].requires_grad_(True))
                self.optimizer.state[group["params"][0]] = stored
            else:
                group["params"][0] = nn.Parameter(group["params"][0][mask].requires_grad_(True))
            out[group["name"]] = group["params"][0]
        return out

    def _take(self, tensors):
        for n, f in self._GROUPS.items():
            setattr(self, f, tensors[n])

    def prune_points(self, mask):
        valid = ~mask
        self._take(self._prune_optimizer(valid))
        self.xyz_gradient_accum = self.xyz_gradient_accum[valid]
        self.denom = self.denom[valid]
        self.max_radii2D = self.max_radii2D[valid]
        self.mask = self.mask[valid]
        self._generation = self._generation[valid]

    def cat_tensors_to_optimizer(self, tensors_dict):
        out = {}
        for group in self.optimizer.param_groups:
            assert len(group["params"]) == 1
            ext = tensors_dict[group["name"]]
            stored = self.optimizer.state.get(group["params"][0], None)
            if stored is not None:
                stored["exp_avg"] = torch.cat((stored["exp_avg"], torch.zeros_like(ext)), dim=0)
                stored["exp_avg_sq"] = torch.cat((stored["exp_avg_sq"], torch.zeros_like(ext)), dim=0)
                del self.optimizer.state[group["params"][0]]
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
                self.optimizer.state[group["params"][0]] = stored
            else:
                group["params"][0] = nn.Parameter(torch.cat((group["params"][0], ext), dim=0).requires_grad_(True))
            out[group["name"]] = group["params"][0]
        return out

    def densification_postfix(self, new_xyz, new_features_dc, new_features_rest, new_opacities, new_scaling,
                              new_rotation):
        d = {"xyz": new_xyz, "f_dc": new_features_dc, "f_rest": new_features_rest, "opacity": new_opacities,
             "scaling": new_scaling, "rotation": new_rotation}
        self._take(self.cat_tensors_to_optimizer(d))
        P = self._xyz.shape[0]
        self.xyz_gradient_accum = torch.zeros((P, 1), device=self.device)
        self.denom = torch.zeros((P, 1), device=self.device)
        self.max_radii2D = torch.zeros(P, device=self.device)

    # -- densification (:643-815) ---------------------------------------------
    def densify_and_split(self, grads, grad_threshold, scene_extent, N=2, generator=None):
        n_init = self._xyz.shape[0]
        padded = torch.zeros(n_init, device=self.device)
        padded[: grads.shape[0]] = grads.squeeze()
        sel = torch.where(padded >= grad_threshold, True, False)
        sel = torch.logical_and(sel, torch.max(self.get_scaling, dim=1).values > self.percent_dense * scene_extent)
        stds = self.get_scaling[sel].repeat(N, 1)
        means = torch.zeros((stds.size(0), 3), device=self.device)
        samples = torch.normal(mean=means, std=stds, generator=generator)
        rots = build_rotation(self._rotation[sel]).repeat(N, 1, 1)
        new_xyz = torch.bmm(rots, samples.unsqueeze(-1)).squeeze(-1) + self.get_xyz[sel].repeat(N, 1)
        new_scaling = self.scaling_inverse_activation(self.get_scaling[sel].repeat(N, 1) / (0.8 * N))
        new_rotation = self._rotation[sel].repeat(N, 1)
        new_features_dc = self._features_dc[sel].repeat(N, 1, 1)
        new_features_rest = self._features_rest[sel].repeat(N, 1, 1)
        new_opacity = self._opacity[sel].repeat(N, 1)
        self.densification_postfix(new_xyz, new_features_dc, new_features_rest, new_opacity, new_scaling,
                                   new_rotation)
        self.mask = torch.cat([self.mask, torch.cat([self.mask[sel]] * N, dim=0)], dim=0)
        new_gen = torch.full((int(sel.sum()),), self.generation_num, dtype=torch.int64, device=self.device)
        self._generation = torch.cat([self._generation, torch.cat([new_gen] * N, dim=0)])
        prune_filter = torch.cat((sel, torch.zeros(N * int(sel.sum()), device=self.device, dtype=torch.bool)))
        self.prune_points(prune_filter)

    def densify_and_clone(self, grads, grad_threshold, scene_extent):
        sel = torch.where(torch.norm(grads, dim=-1) >= grad_threshold, True, False)
        sel = torch.logical_and(sel, torch.max(self.get_scaling, dim=1).values <= self.percent_dense * scene_extent)
        self.densification_postfix(self._xyz[sel], self._features_dc[sel], self._features_rest[sel],
                                   self._opacity[sel], self._scaling[sel], self._rotation[sel])
        assert len(torch.nonzero(self.mask[sel] == 0)) == 0, "nontarget area should not be densified"
        self.mask = torch.cat([self.mask, self.mask[sel]], dim=0)
        new_gen = torch.full((int(sel.sum()),), self.generation_num, dtype=torch.int64, device=self.device)
        self._generation = torch.cat([self._generation, new_gen])

    def densify_and_prune(self, max_grad, max_densify_percent, min_opacity, extent, max_screen_size,
                          generator=None):
        grads = self.xyz_gradient_accum / self.denom
        grads[grads.isnan()] = 0.0
        grads[~self.mask] = 0.0
        if max_densify_percent < 1:
            valid_percent = len(grads.nonzero()) * max_densify_percent / grads.shape[0]
            threshold = torch.quantile(grads, 1 - valid_percent)
            grads[grads < threshold] = 0.0
        self.densify_and_clone(grads, max_grad, extent)
        self.densify_and_split(grads, max_grad, extent, generator=generator)
        prune_mask = (self.get_opacity < min_opacity).squeeze()
        if max_screen_size:
            big_vs = self.max_radii2D > max_screen_size
            big_ws = self.get_scaling.max(dim=1).values > 0.1 * extent
            prune_mask = torch.logical_or(torch.logical_or(prune_mask, big_vs), big_ws)
        prune_mask = torch.logical_and(prune_mask, self.mask)
        self.prune_points(prune_mask)
        self.remove_grad_mask()
        self.apply_grad_mask(self.mask)
        self.update_anchor()
        self.update_anchor_loss_schedule()

    def add_densification_stats(self, viewspace_point_tensor, update_filter):
        self.xyz_gradient_accum[update_filter] += torch.norm(viewspace_point_tensor[update_filter, :2], dim=-1,
                                                             keepdim=True)
        self.denom[update_filter] += 1

    def reset_opacity(self):
        new = inverse_sigmoid(torch.min(self.get_opacity, torch.ones_like(self.get_opacity) * 0.01))
        self._opacity = self.replace_tensor_to_optimizer(new, "opacity")["opacity"]

    def prune_with_mask(self, new_mask=None):
        self.prune_points(self.mask)
        if new_mask is not None:
            self.mask = new_mask
        else:
            self.mask[:] = 1
        self.remove_grad_mask()
        self.apply_grad_mask(self.mask)
        self.update_anchor()

    # -- grad mask (:834-863) -------------------------------------------------
    def set_mask(self, mask):
        self.mask = mask

    def apply_grad_mask(self, mask):
        assert self.mask.shape[0] == self._xyz.shape[0]
        self.set_mask(mask)

        def hook(grad):
            if grad is None:  # the fused backward already wrote the (masked) gradient into .grad
                return None
            return grad * (self.mask[:, None] if grad.ndim == 2 else self.mask[:, None, None])

        # the rasterizer's fused backward recognises this hook and applies the current
        # self.mask in-kernel (dge_amd/diff_gaussian_rasterization: _mask_owner)
        hook._dge_grad_mask_owner = self
        self.hooks = []
        for field in self._MASKED_FIELDS:
            t = getattr(self, field)
            assert t.is_leaf and t.requires_grad
            self.hooks.append(t.register_hook(hook))

    def remove_grad_mask(self):
        for h in self.hooks:
            h.remove()
        self.hooks = []

    # -- generations and anchor loss (:92-184) ---------------------------------
    @property
    def generation_num(self):
        return len(self._anchor_loss_schedule)

    def update_anchor_term(self, anchor_weight_init_g0, anchor_weight_init, anchor_weight_multiplier):
        self.anchor_weight_init = anchor_weight_init
        self.anchor_weight_multiplier = anchor_weight_multiplier
        self._anchor_loss_schedule = torch.tensor([anchor_weight_init_g0], device=self.device)
        self.anchor_weight_init_g0 = anchor_weight_init_g0

    def anchor_postfix(self):
        self._generation[...] = 0
        self._anchor_loss_schedule = torch.tensor([self.anchor_weight_init_g0], device=self.device)

    def update_anchor(self):
        self.anchor = {f: getattr(self, f).detach().clone() for f in
                       ("_xyz", "_features_dc", "_features_rest", "_scaling", "_rotation", "_opacity")}

    def update_anchor_loss_schedule(self):
        for i, w in enumerate(self._anchor_loss_schedule):
            self._anchor_loss_schedule[i] = min(self.anchor_weight_multiplier * w, MAX_ANCHOR_WEIGHT)
        if self.generation_num > 1:
            assert self._anchor_loss_schedule[-1] == 0
            self._anchor_loss_schedule[-1] = self.anchor_weight_init
        self._anchor_loss_schedule = torch.cat([self._anchor_loss_schedule, torch.tensor([0], device=self.device)])

    def anchor_loss(self):
        out = {"loss_anchor_color": 0, "loss_anchor_geo": 0, "loss_anchor_opacity": 0, "loss_anchor_scale": 0}
        w = torch.gather(self._anchor_loss_schedule, dim=0, index=self._generation[self.mask])
        for key, value in self.anchor.items():
            delta = torch.nn.functional.mse_loss(getattr(self, key)[self.mask], value[self.mask], reduction="none")
            delta = delta * (w[:, None, None] if "feature" in key else w[:, None])
            delta = torch.mean(delta)
            if key in ("_xyz", "_rotation"):
                out["loss_anchor_geo"] += delta
            elif key in ("_features_dc", "_features_rest"):
                out["loss_anchor_color"] += delta
            elif key == "_opacity":
                out["loss_anchor_opacity"] += delta
            else:
                out["loss_anchor_scale"] += delta
        return out

    # -- PLY (:396-551) ---------------------------------------------------------
    def construct_list_of_attributes(self):
        from .ply import attribute_names

        return attribute_names(self._features_dc.shape[1] * self._features_dc.shape[2],
                               self._features_rest.shape[1] * self._features_rest.shape[2],
                               self._scaling.shape[1], self._rotation.shape[1])

    def save_ply(self, path):
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        v = gaussians_to_vertex(*(getattr(self, f).detach().cpu().numpy() for f in
                                  ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")))
        write_ply(path, v)

    def load_ply(self, path):
        xyz, f_dc, f_rest, opacity, scaling, rotation, max_deg = vertex_to_gaussians(read_ply(path)["vertex"])
        self.max_sh_degree = max_deg
        self.set_parameters(xyz, f_dc, f_rest, opacity, scaling, rotation, active_sh_degree=max_deg)
        return self

    def apply_weights(self, camera, weights, weights_cnt, image_weights):
        """:817-832 — back-project image weights through the gfx950 apply_weights kernel."""
        from .gaussian_renderer import camera2rasterizer

        rasterizer = camera2rasterizer(camera, torch.tensor([0.0, 0.0, 0.0], dtype=torch.float32, device=self.device))
        rasterizer.apply_weights(self.get_xyz, None, self.get_opacity, None, weights, self.get_scaling,
                                 self.get_rotation, None, weights_cnt, image_weights)
