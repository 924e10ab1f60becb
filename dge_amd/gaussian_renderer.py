"""render() entry points with the reference's signatures and return dicts.

Restates gaussiansplatting/gaussian_renderer/__init__.py:
  camera2rasterizer  (:21-42)
  render             (:45-150)   -> {"render","viewspace_points","visibility_filter","radii","depth_3dgs"}
  point_cloud_render (:156-250)
on top of ``dge_amd.diff_gaussian_rasterization``.  Two reference paths are
broken in the reference and work here: the
``compute_cov3D_python`` path (scales.float() on None, :137) and the
``convert_SHs_python`` path (shs.float() on None, :124).
"""
from __future__ import annotations

import math
import os
import weakref

import torch
import torch.nn.functional as F

from .diff_gaussian_rasterization import (GaussianRasterizationSettings, GaussianRasterizer, RecolorPrepared,
                                         rasterize_gaussian_model)
from .sh_utils import eval_sh


class PipelineParams:
    """arguments/__init__.py:63-68 defaults."""

    def __init__(self, convert_SHs_python=False, compute_cov3D_python=False, debug=False):
        self.convert_SHs_python = convert_SHs_python
        self.compute_cov3D_python = compute_cov3D_python
        self.debug = debug


def _settings(cam, bg_color, scaling_modifier, sh_degree, debug=False):
    return GaussianRasterizationSettings(
        image_height=int(cam.image_height), image_width=int(cam.image_width),
        tanfovx=math.tan(cam.FoVx * 0.5), tanfovy=math.tan(cam.FoVy * 0.5), bg=bg_color,
        scale_modifier=scaling_modifier, viewmatrix=cam.world_view_transform, projmatrix=cam.full_proj_transform,
        sh_degree=sh_degree, campos=cam.camera_center, prefiltered=False, debug=debug)


def camera2rasterizer(viewpoint_camera, bg_color: torch.Tensor, sh_degree: int = 0):
    return GaussianRasterizer(raster_settings=_settings(viewpoint_camera, bg_color, 1.0, sh_degree))


def _fused_ok(pc, pipe) -> bool:
    """The raw-parameter path applies when the model is a standard GaussianModel
    (activations exp / sigmoid / F.normalize; fp32 parameters, features fp32 or
    fp16; a `localize` subset given by a boolean mask over the rows) and the
    pipeline asks for the in-kernel SH and covariance (the defaults)."""
    if os.environ.get("DGE_AMD_FUSED", "1") == "0":
        return False
    if pipe.compute_cov3D_python or pipe.convert_SHs_python:
        return False
    need = ("_xyz", "_features_dc", "_features_rest", "_opacity", "_scaling", "_rotation")
    if not all(isinstance(getattr(pc, n, None), torch.Tensor) for n in need):
        return False
    for attr, fn in (("scaling_activation", torch.exp), ("opacity_activation", torch.sigmoid),
                     ("rotation_activation", F.normalize)):
        if getattr(pc, attr, fn) is not fn:
            return False
    if getattr(pc, "localize", False):
        m = getattr(pc, "mask", None)
        if not (isinstance(m, torch.Tensor) and m.dtype == torch.bool and m.shape == (pc._xyz.shape[0],)
                and m.device == pc._xyz.device):
            return False
    feats = (pc._features_dc.dtype, pc._features_rest.dtype)
    if feats not in ((torch.float32, torch.float32), (torch.float16, torch.float16)):
        return False
    return all(getattr(pc, n).is_cuda for n in need) and all(
        getattr(pc, n).dtype == torch.float32 for n in ("_xyz", "_opacity", "_scaling", "_rotation"))


_MASK_INDEX = {}  # id(mask) -> (weakref(mask), version, int32 rows)


def _mask_rows(mask):
    """Ascending int32 rows of a boolean mask (the order of pc[mask]); one host sync per mask change."""
    key = id(mask)
    ent = _MASK_INDEX.get(key)
    if ent is not None and ent[0]() is mask and ent[1] == mask._version:
        return ent[2]
    rows = torch.nonzero(mask.detach()).squeeze(1).to(torch.int32)
    _MASK_INDEX[key] = (weakref.ref(mask, lambda _r, k=key: _MASK_INDEX.pop(k, None)), mask._version, rows)
    return rows


def render(viewpoint_camera, pc, pipe, bg_color: torch.Tensor, scaling_modifier=1.0, override_color=None):
    if _fused_ok(pc, pipe):
        return _render_fused(viewpoint_camera, pc, pipe, bg_color, scaling_modifier, override_color)
    xyz = pc.get_xyz
    screenspace_points = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True, device=xyz.device) + 0
    try:
        screenspace_points.retain_grad()
    except Exception:
        pass
    rasterizer = GaussianRasterizer(
        raster_settings=_settings(viewpoint_camera, bg_color, scaling_modifier, pc.active_sh_degree,
                                  getattr(pipe, "debug", False)))
    means3D, means2D, opacity = xyz, screenspace_points, pc.get_opacity

    scales = rotations = cov3D_precomp = None
    if pipe.compute_cov3D_python:
        cov3D_precomp = pc.get_covariance(scaling_modifier)
    else:
        scales, rotations = pc.get_scaling, pc.get_rotation

    shs = colors_precomp = None
    if override_color is None:
        if pipe.convert_SHs_python:
            feats = pc.get_features
            shs_view = feats.transpose(1, 2).reshape(-1, 3, (pc.max_sh_degree + 1) ** 2)
            dir_pp = xyz - viewpoint_camera.camera_center.repeat(feats.shape[0], 1)
            dir_pp = dir_pp / dir_pp.norm(dim=1, keepdim=True)
            colors_precomp = torch.clamp_min(eval_sh(pc.active_sh_degree, shs_view, dir_pp) + 0.5, 0.0)
        else:
            # fp16 SH storage (the local-edit path) goes to the kernels as is and is upcast there;
            # the reference's .float() would materialise an fp32 copy first
            feats = pc.get_features
            shs = feats if feats.dtype == torch.float16 else feats.float()
    else:
        colors_precomp = override_color

    rendered_image, radii, depth = rasterizer(
        means3D=means3D.float(), means2D=means2D.float(), shs=shs, colors_precomp=colors_precomp,
        opacities=opacity.float(), scales=None if scales is None else scales.float(),
        rotations=None if rotations is None else rotations.float(), cov3D_precomp=cov3D_precomp)
    return {
        "render": rendered_image,
        "viewspace_points": screenspace_points,
        "visibility_filter": radii > 0,
        "radii": radii,
        "depth_3dgs": depth,
    }


_VIEWSPACE_ZEROS = {}  # device -> (zero buffer, its version when last known zero)


def _viewspace_zeros(n, dtype, device):
    """A fresh leaf of n x 3 zeros (the means2D placeholder whose .grad receives dL/dmeans2D) without a fill
    kernel per view: every call returns a new leaf over one cached zero buffer, re-zeroed only if
    someone wrote into it (its version counter moved)."""
    ent = _VIEWSPACE_ZEROS.get(device)
    if ent is None or ent[0].shape[0] < n or ent[0].dtype != dtype:
        buf = torch.zeros((max(n, 1), 3), dtype=dtype, device=device)
        ent = _VIEWSPACE_ZEROS[device] = (buf, buf._version)
    buf, ver = ent
    if buf._version != ver:
        buf.zero_()
        _VIEWSPACE_ZEROS[device] = (buf, buf._version)
    return buf[:n].detach().requires_grad_(True)


def _render_fused(viewpoint_camera, pc, pipe, bg_color, scaling_modifier=1.0, override_color=None):
    """render() for a standard GaussianModel without the getters' torch kernels:
    the rasterizer consumes _xyz, _features_dc, _features_rest, _opacity,
    _scaling, _rotation directly and returns their gradients."""
    return _fused_end(_fused_begin(viewpoint_camera, pc, pipe, bg_color, scaling_modifier, override_color), pc)


_LAZY_OVERRIDE = os.environ.get("DGE_AMD_LAZY_OVERRIDE", "1") != "0"
_RECOLOR = os.environ.get("DGE_AMD_RECOLOR", "1") != "0"
# A training forward of a model carrying a boolean `mask` over its Gaussians (DGE's edit mask) also
# composites that mask as a grey colour along its own alpha / transmittance chain (gs_params.aux_mask): the
# semantic render DGE issues right after it (override_color = mask repeated over the channels) is then
# served from those sums — checked on the device, bit for bit — instead of a second blend.
_AUX = os.environ.get("DGE_AMD_AUX", "1") != "0"
_AUX_HITS = 0  # recolor renders offered a forward's aux sums (tests, bench)

# The last fused forward with backward bookkeeping per device: DGE renders each view for training, then
# the same camera and Gaussians again with the edit mask as override_color (DGE.py:181, 198-204) —
# identical preprocess, depth order and tile lists, only the colours differ.  A gradient-free recolor
# render whose geometry inputs are the ones of that forward (the same tensors at the same versions, the
# same camera matrices, image size, fields of view, scale modifier, localize rows) reuses its buffers:
# only the blend runs again (gs_render_recolor), bit-identical to the full forward.  Weak references: an
# entry never keeps a forward's buffers alive (its autograd graph does, until its backward).
_LAST_FORWARD = {}  # device index -> _ForwardEntry
_RECOLOR_HITS = 0  # recolor renders served from a cached forward (tests, bench)


def _tensor_key(t):
    return None if t is None else (id(t), t._version)


class _ForwardEntry:
    """num_rendered: the binning layout's instance count."""

    def __init__(self, key, refs, num_rendered, P, stream, radii, visible, aux=None):
        self.key, self.refs, self.num_rendered, self.P = key, refs, num_rendered, P
        self.stream, self.radii, self.visible = stream, radii, visible
        # aux: (weakref to the mask the forward composited, its version then)
        self.aux = None if aux is None else (weakref.ref(aux), aux._version)

    def aux_mask(self):
        """The mask this forward composited (gs_params.aux_mask), if it is alive and unchanged since."""
        if self.aux is None:
            return None
        m = self.aux[0]()
        return m if m is not None and m._version == self.aux[1] else None

    def buffers(self):
        bufs = [r() for r in self.refs]
        return None if any(b is None for b in bufs) else bufs


def _geometry_key(pc, rs, index):
    return (_tensor_key(pc._xyz), _tensor_key(pc._opacity), _tensor_key(pc._scaling), _tensor_key(pc._rotation),
            _tensor_key(index), _tensor_key(rs.viewmatrix), _tensor_key(rs.projmatrix), int(rs.image_height),
            int(rs.image_width), float(rs.tanfovx), float(rs.tanfovy), float(rs.scale_modifier), bool(rs.prefiltered))


def _recolor_source(pc, rs, index):
    """The cached forward a recolor render of these inputs may reuse, or None."""
    if not _RECOLOR:
        return None
    ent = _LAST_FORWARD.get(pc._xyz.device.index)
    if ent is None or ent.key != _geometry_key(pc, rs, index):
        return None
    # (ids and versions match; the weak references confirm the very tensors are alive, not recycled ids)
    if any(r() is None for r in ent.tensor_refs) or ent.buffers() is None:
        return None
    return ent


def _may_backward(*tensors) -> bool:
    """Whether autograd can run a backward of a forward of these inputs (grad mode on and one of them
    requires grad): else the kernels skip the backward's scratch (gs_params.forward_only).  The view-space
    placeholder render() adds is a fresh leaf that requires grad, so it does not count."""
    return torch.is_grad_enabled() and any(t is not None and t.requires_grad for t in tensors)


def _fused_begin(viewpoint_camera, pc, pipe, bg_color, scaling_modifier=1.0, override_color=None):
    """The first half of _render_fused: settings, the visibility output and the native forward's first half
    (preprocess, depth sort, instance scan) enqueued on the current stream without a host wait."""
    from . import _C

    xyz = pc._xyz
    index = _mask_rows(pc.mask) if getattr(pc, "localize", False) else None
    n = index.numel() if index is not None else xyz.shape[0]
    rs = _settings(viewpoint_camera, bg_color, scaling_modifier, pc.active_sh_degree, getattr(pipe, "debug", False))
    if override_color is None:
        f_dc, f_rest, colors = pc._features_dc, pc._features_rest, None
    else:
        f_dc, f_rest, colors = None, None, override_color.float()
    visible = torch.empty(n, dtype=torch.bool, device=xyz.device)  # radii > 0, written by the preprocess
    may_bwd = _may_backward(xyz, f_dc, f_rest, colors, pc._opacity, pc._scaling, pc._rotation)
    aux = None
    if _AUX and _RECOLOR and override_color is None and index is None and may_bwd:
        m = getattr(pc, "mask", None)
        if (isinstance(m, torch.Tensor) and m.dtype == torch.bool and m.shape == (xyz.shape[0],)
                and m.device == xyz.device and m.is_contiguous()):
            aux = m
    # DGE's semantic render (DGE.py:198-204: override_color = the edit mask, grad mode on, its image only
    # thresholded) never receives a gradient: render it with the forward-only kernels and, should a
    # backward come after all, recompute the forward with the backward's bookkeeping then (lazy)
    lazy = may_bwd and colors is not None and not colors.requires_grad and _LAZY_OVERRIDE
    # forward_only: the kernels skip the backward's bookkeeping, and a two-level binning then keeps the
    # Gaussian ids alone (gs_raster.h gs_render_recolor): such a forward is never a recolor source
    forward_only = lazy or not may_bwd
    st = {"rs": rs, "index": index, "n": n, "f_dc": f_dc, "f_rest": f_rest, "colors": colors, "visible": visible,
          "prepared": None, "lazy": lazy, "forward_only": forward_only, "aux": aux}
    if rs.debug:  # debug mode: the one-call forward, which keeps the reference's failure snapshot
        return st
    if colors is not None and not colors.requires_grad and forward_only:
        src = _recolor_source(pc, rs, index)
        if src is not None:  # the same geometry as the last forward: only its blend again, other colours
            global _RECOLOR_HITS
            _RECOLOR_HITS += 1
            geom, binning, img = src.buffers()
            cur = torch.cuda.current_stream(xyz.device)
            if src.stream != cur:
                cur.wait_stream(src.stream)
                # (the source's graph may be freed on its stream while this blend still reads its buffers)
                for t in (geom, binning, img):
                    t.record_stream(cur)
            src_aux = src.aux_mask()
            if src_aux is not None:
                global _AUX_HITS
                _AUX_HITS += 1
            color, depth = _C.render_recolor(rs.bg, colors, rs.viewmatrix, rs.projmatrix, rs.campos, rs.tanfovx,
                                             rs.tanfovy, rs.image_height, rs.image_width, rs.sh_degree,
                                             rs.scale_modifier, rs.prefiltered, n, src.num_rendered, geom, binning,
                                             img, src_aux_mask=src_aux)
            st["visible"] = src.visible.clone()
            st["prepared"] = RecolorPrepared(src.num_rendered, color, depth, src.radii.clone())
            st["lazy"] = may_bwd  # (a backward, should one come, renders these inputs in full first)
            return st
    empty = torch.empty(0, dtype=torch.float32, device=xyz.device)
    st["prepared"] = _C.rasterize_gaussians_fused_begin(
        rs.bg, xyz, empty if f_dc is None else f_dc, empty if f_rest is None else f_rest,
        empty if colors is None else colors, pc._opacity, pc._scaling, pc._rotation, rs.scale_modifier,
        rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, rs.sh_degree,
        rs.campos, rs.prefiltered, rs.debug, index=index, visible=visible, forward_only=forward_only, aux_mask=aux)
    return st


def _fused_end(st, pc):
    """The second half: the autograd node over the native forward's second half; render()'s dict."""
    xyz = pc._xyz
    screenspace_points = _viewspace_zeros(st["n"], xyz.dtype, xyz.device)
    prep = st["prepared"]
    rendered_image, radii, depth = rasterize_gaussian_model(
        xyz, screenspace_points, st["f_dc"], st["f_rest"], st["colors"], pc._opacity, pc._scaling, pc._rotation,
        st["rs"], st["index"], st["visible"], prepared=prep, recompute=st["lazy"] and prep is not None)
    fin = getattr(prep, "finished", None)
    if fin is not None and _RECOLOR and not st.get("forward_only", True):
        # a forward with backward bookkeeping: later recolor renders may reuse it
        nr, geom, binning, img = fin
        prep.finished = None
        ent = _ForwardEntry(_geometry_key(pc, st["rs"], st["index"]), [weakref.ref(geom), weakref.ref(binning),
                            weakref.ref(img)], nr, st["n"], torch.cuda.current_stream(xyz.device), radii, st["visible"],
                            aux=st.get("aux"))
        ent.tensor_refs = [weakref.ref(t) for t in (pc._xyz, pc._opacity, pc._scaling, pc._rotation,
                                                    st["rs"].viewmatrix, st["rs"].projmatrix) if t is not None]
        if st["index"] is not None:
            ent.tensor_refs.append(weakref.ref(st["index"]))
        _LAST_FORWARD[xyz.device.index] = ent
    return {
        "render": rendered_image,
        "viewspace_points": screenspace_points,
        "visibility_filter": st["visible"],
        "radii": radii,
        "depth_3dgs": depth,
    }


def point_cloud_render(viewpoint_camera, xyz, pipe, bg_color: torch.Tensor, scaling_modifier=1.0,
                       override_color=None):
    screenspace_points = torch.zeros_like(xyz, dtype=xyz.dtype, requires_grad=True, device=xyz.device) + 0
    try:
        screenspace_points.retain_grad()
    except Exception:
        pass
    rasterizer = GaussianRasterizer(raster_settings=_settings(viewpoint_camera, bg_color, scaling_modifier, 0))
    opacity = torch.ones_like(xyz[..., 0:1])
    scales = torch.ones_like(xyz) * 0.005
    rotations = torch.zeros([xyz.shape[0], 4], dtype=xyz.dtype, device=xyz.device)
    rotations[..., 0] = 1.0
    colors_precomp = torch.ones_like(xyz[..., 0:1]).repeat(1, 3)
    rendered_image, radii, depth = rasterizer(
        means3D=xyz.float(), means2D=screenspace_points.float(), shs=None, colors_precomp=colors_precomp,
        opacities=opacity.float(), scales=scales.float(), rotations=rotations.float(), cov3D_precomp=None)
    return {
        "render": rendered_image,
        "viewspace_points": screenspace_points,
        "visibility_filter": radii > 0,
        "radii": radii,
        "depth_3dgs": depth,
    }
