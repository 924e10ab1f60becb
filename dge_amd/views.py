"""A batch of views of one scene in one native call (gs_views_* of include/gs_raster.h).

DGE renders a batch of edited views of one scene per step and back-propagates their summed
loss (threestudio/systems/DGE.py:170-239 renders, :617-699 the step).  ``render()`` serves that
loop one view at a time, as the reference does (gaussian_renderer/__init__.py:45-150, one
``_C.rasterize_gaussians`` per view with its host sync, rasterizer_impl.cu:236-239).  This module
renders the whole batch through ONE autograd node over ONE native forward and ONE native
backward:

  * ``gs_views_forward`` enqueues every view's first half (preprocess, depth sort, instance scan)
    on the view's HIP stream before any second half, and — ``speculate`` — sizes each view's
    binning buffer from the instance counts the library has seen for this (P, W, H) instead of
    waiting for the count: the emission, tile sort and blend read it on the device, so the host
    never waits inside a step.  ``RenderedViews.check()`` reads the counts afterwards (the step's
    one host wait, on the forwards' preprocess only) and reports a view that overflowed its
    capacity: the caller renders the batch again (the capacity has grown by then);
  * ``gs_views_backward`` replays every view on its stream and chains the views' per-Gaussian
    passes in view order, accumulating straight into the parameters' ``.grad`` (the fused
    gradient accumulation of ``diff_gaussian_rasterization._RasterizeGaussiansFused``): the
    summed gradient is the one the reference's per-view loop accumulates, bit for bit in the
    per-view sums and in a fixed view order.

Outputs per view are render()'s dict ("render", "viewspace_points", "visibility_filter", "radii",
"depth_3dgs") plus "_live_rows" (the Gaussians some pixel of the view blends: the rows the
backward makes nonzero, multiview.GradBucket.allreduce_begin).
"""
from __future__ import annotations

import ctypes
import weakref

import torch

from . import _C
from . import _native as N
from . import diff_gaussian_rasterization as _R


class _Buffers:
    """gs_alloc_fn target of one gs_views_forward: which 0 = the batch's buffer, 16 + v = view v's
    exact binning buffer (torch caching allocator, current stream)."""

    __slots__ = ("device", "buffers", "fn")

    def __init__(self, device):
        self.device = device
        self.buffers = {}
        _C._TLS.alloc = self
        self.fn = _C._ALLOC_CB


class ViewBatch:
    """The native handle of one gs_views_forward call and what its backward and check need."""

    def __init__(self, handle, bufs, n, P, W, H, dev, keep):
        self.handle, self.bufs, self.n, self.P, self.W, self.H, self.dev = handle, bufs, n, P, W, H, dev
        self.keep = keep
        self.status = None
        self.num_rendered = None
        self._fin = weakref.finalize(self, N.lib().gs_views_release, handle)

    def check(self) -> bool:
        """True when every view's binning fitted (the outputs are valid); False when a speculated view
        overflowed its capacity (render the batch again).  Waits for the views' preprocess only."""
        if self.status is None:
            counts = (ctypes.c_int * self.n)()
            rc = N.lib().gs_views_check(self.handle, counts)
            self.num_rendered = list(counts)
            if rc not in (N.GS_OK, N.GS_ERR_RETRY):
                N.check(rc, "render_views")
            self.status = rc
        return self.status == N.GS_OK

    def buffer(self, v: int, which: int):
        """(torch byte tensor, offset) of view v's buffer (0 geometry, 1 binning, 2 image)."""
        ptr = N.lib().gs_views_buffer(self.handle, v, which)
        for t in self.bufs.buffers.values():
            base = t.data_ptr()
            if ptr is not None and base <= ptr < base + t.numel():
                return t, ptr - base
        raise RuntimeError("view buffer not found")

    def touched(self, v: int):
        """uint8 [P] view of view v's `touched` bytes (the Gaussians some pixel blended)."""
        t, off = self.buffer(v, 0)
        o = N.lib().gs_buffer_offset(b"geometry", b"touched", self.P, self.W, self.H, 0)
        return t[off + o:off + o + self.P]


def _fill_settings(rs, dev):
    s, keep = _C._settings(rs.bg, rs.viewmatrix, rs.projmatrix, rs.campos, rs.tanfovx, rs.tanfovy, rs.image_height,
                           rs.image_width, rs.sh_degree, rs.scale_modifier, rs.prefiltered, rs.debug)
    return s, keep


class _RasterizeViews(torch.autograd.Function):
    """Forward of a batch of views of one GaussianModel (raw tensors, activations in-kernel) and the
    backward of their images, each through one native call."""

    @staticmethod
    def forward(ctx, meta, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, *means2D):
        settings, streams, speculate, index, visible = meta["settings"], meta["streams"], meta["speculate"], \
            meta["index"], meta["visible"]
        n = len(settings)
        dev = xyz.device
        P = index.numel() if index is not None else xyz.size(0)
        H, W = int(settings[0].image_height), int(settings[0].image_width)
        for rs in settings:
            if int(rs.image_height) != H or int(rs.image_width) != W:
                raise ValueError("render_views: every view of a batch must have the same image size")
        out = torch.empty((n, 4, H, W), dtype=torch.float32, device=dev)  # colour (3) + depth (1) per view
        radii = torch.empty((n, P), dtype=torch.int32, device=dev)
        ss, gs, keep = [], [], [xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, index]
        for v, rs in enumerate(settings):
            s, k = _fill_settings(rs, dev)
            keep += k
            g = _C._params(P, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, index,
                           visible[v] if visible is not None else None, meta["forward_only"])
            ss.append(s)
            gs.append(g)
        s_arr = (ctypes.c_void_p * n)(*[ctypes.addressof(x) for x in ss])
        g_arr = (ctypes.c_void_p * n)(*[ctypes.addressof(x) for x in gs])
        base = out.data_ptr()
        plane = 4 * H * W * 4
        c_arr = (ctypes.c_void_p * n)(*[base + v * plane for v in range(n)])
        d_arr = (ctypes.c_void_p * n)(*[base + v * plane + 3 * H * W * 4 for v in range(n)])
        r_arr = (ctypes.c_void_p * n)(*[radii.data_ptr() + 4 * P * v for v in range(n)])
        st_arr = (ctypes.c_void_p * n)(*[st.cuda_stream for st in streams])
        bufs = _Buffers(dev)
        h = ctypes.c_void_p(None)
        join = torch.cuda.current_stream(dev).cuda_stream
        rc = N.lib().gs_views_forward(n, s_arr, g_arr, c_arr, d_arr, r_arr,
                                      N.VIEWS_SPECULATE if speculate else N.VIEWS_EXACT, bufs.fn, None, st_arr,
                                      join, ctypes.byref(h))
        N.check(rc, "render_views")
        # (the backward reads the radii through the handle: kept alive with the batch, not only by the
        # caller's outputs — DGE's loop drops a view's radii dict once it has taken their max)
        keep.append(radii)
        batch = ViewBatch(h.value, bufs, n, P, W, H, dev, keep)
        if P == 0:
            radii.zero_()
        meta["batch"] = batch
        ctx.batch, ctx.meta, ctx.n, ctx.P = batch, meta, n, P
        ctx.has_sh = f_dc is not None and f_dc.numel() != 0
        ctx.save_for_backward(xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation)
        colors_out = [out[v, :3] for v in range(n)]
        depths = [out[v, 3:] for v in range(n)]
        radii_out = [radii[v] for v in range(n)]
        ctx.mark_non_differentiable(*radii_out)
        ctx.set_materialize_grads(False)
        return (*colors_out, *radii_out, *depths)

    @staticmethod
    def backward(ctx, *grads):
        n, P, batch = ctx.n, ctx.P, ctx.batch
        gimg = grads[:n]
        none = (None,) * (8 + n)
        if all(g is None for g in gimg):
            return none
        xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation = ctx.saved_tensors
        index = ctx.meta["index"]
        dev = xyz.device
        H, W = batch.H, batch.W
        opts = dict(dtype=torch.float32, device=dev)
        zero_img = None
        gpix = []
        for g in gimg:  # a view whose image took no part in the loss contributes nothing
            if g is None:
                if zero_img is None:
                    zero_img = torch.zeros((3, H, W), **opts)
                g = zero_img
            gpix.append(_C._f32(g, "dL_dout_color"))
        # where each parameter gradient goes: into p.grad (fused accumulation: "add" into an existing
        # .grad, "new" writes a fresh one that becomes p.grad), else a fresh tensor handed to autograd
        nf = ctx.next_functions  # tensor inputs: xyz 0, f_dc 1, f_rest 2, colors 3, opacity 4, scaling 5, rotation 6
        fuse = _R._FUSED_GRAD_ACCUM and not torch.is_grad_enabled()
        params = {"xyz": (xyz, nf[0][0], N.ACC_MEANS3D), "opacity": (raw_opacity, nf[4][0], N.ACC_OPACITY),
                  "scaling": (raw_scaling, nf[5][0], N.ACC_SCALES), "rotation": (raw_rotation, nf[6][0], N.ACC_ROTATIONS)}
        if ctx.has_sh:
            params["f_dc"] = (f_dc, nf[1][0], N.ACC_SH)
            params["f_rest"] = (f_rest, nf[2][0], N.ACC_SH)
        modes = {k: (_R._accumulation_mode(p, node) if fuse else (None, None)) for k, (p, node, _) in params.items()}
        if ctx.has_sh and not (modes["f_dc"][0] == modes["f_rest"][0] and modes["f_dc"][1] is modes["f_rest"][1]):
            modes["f_dc"] = modes["f_rest"] = (None, None)  # both SH tensors go the same way (one SH output)
        owners = {id(o): o for m, o in modes.values() if m is not None and o is not None}
        grad_mask, mask_bits = None, 0
        if owners:
            mask = next(iter(owners.values())).mask if len(owners) == 1 else None
            if mask is None or mask.dtype != torch.bool or mask.shape != (xyz.shape[0],) or mask.device != dev:
                # not expressible in-kernel: hand those gradients back to autograd (which runs the hooks)
                modes = {k: ((None, None) if o is not None else (m, o)) for k, (m, o) in modes.items()}
            else:
                grad_mask = mask.contiguous().view(torch.uint8)
                mask_bits = 0
                for k, (m, o) in modes.items():
                    if m is not None and o is not None:
                        mask_bits |= params[k][2]
        zi = index is not None
        targets, direct, returned, acc0 = {}, [], {}, 0
        for k, (p, _, bit) in params.items():
            m = modes[k][0]
            if m == "add":
                targets[k] = p.grad
                acc0 |= bit
                continue
            t = (torch.zeros_like if zi else torch.empty_like)(p, dtype=torch.float32,
                                                              memory_format=torch.contiguous_format)
            targets[k] = t
            if m == "new":
                direct.append((p, t))
            else:
                returned[k] = t
        if not ctx.has_sh:
            targets["colors"] = torch.empty_like(colors) if colors is not None and colors.numel() else None
        zeroed = _R.zeroed_bits(dev, [targets[k] for k, (p, _, bit) in params.items() if acc0 & bit], acc0)
        dirty = _R.dirty_rows(dev, [targets[k] for k in params])
        acc_all = N.ACC_MEANS3D | N.ACC_OPACITY | N.ACC_SCALES | N.ACC_ROTATIONS | (N.ACC_SH if ctx.has_sh else 0)
        if not ctx.has_sh and targets.get("colors") is not None:
            acc_all |= N.ACC_COLORS
        d_m2 = torch.empty((n, P, 3), **opts)
        gg = []
        for v in range(n):
            o = N.GsGrads()
            o.dL_dmeans2D = d_m2[v].data_ptr()
            o.dL_dcolors = None if ctx.has_sh else _C._ptr(targets.get("colors"))
            o.dL_dopacity = targets["opacity"].data_ptr()
            o.dL_dmeans3D = targets["xyz"].data_ptr()
            o.dL_dcov3D = None
            if ctx.has_sh:
                o.dL_dsh_dc = targets["f_dc"].data_ptr()
                o.dL_dsh_rest = _C._ptr(targets["f_rest"])
            o.dL_dscales = targets["scaling"].data_ptr()
            o.dL_drotations = targets["rotation"].data_ptr()
            # row pitches: a .grad that is a column block of a row-major gradient bucket is written in place
            rest = targets["f_rest"] if ctx.has_sh and f_rest is not None and f_rest.numel() else None
            _C.set_grad_pitches(o, targets["xyz"], targets["opacity"], targets["scaling"], targets["rotation"],
                                targets["f_dc"] if ctx.has_sh else None, rest)
            # the first view writes (or adds into an existing .grad), the others add; into a .grad buffer
            # zeroed this step, a Gaussian's first gradient is stored, not added (gs_grads.zeroed)
            o.accumulate = acc0 if v == 0 else acc_all
            o.dirty_rows = _C._ptr(dirty)  # (the bucket's written rows: its next zero() clears only those)
            if v == 0:
                o.zeroed = zeroed
            if grad_mask is not None:
                o.grad_mask = grad_mask.data_ptr()
                o.mask_bits = mask_bits
            gg.append(o)
        stream = torch.cuda.current_stream(dev)
        ev = _R.grad_writes_event(dev, stream)
        after = ev.cuda_event if ev is not None else None
        dp = (ctypes.c_void_p * n)(*[g.data_ptr() for g in gpix])
        go = (ctypes.c_void_p * n)(*[ctypes.addressof(o) for o in gg])
        st_arr = (ctypes.c_void_p * n)(*[st.cuda_stream for st in ctx.meta["streams"]])
        rc = N.lib().gs_views_backward(batch.handle, dp, go, st_arr, after, stream.cuda_stream)
        N.check(rc, "render_views backward")
        if _R._SIDE_STREAMS:  # later backward calls on other streams order their .grad writes after these
            _R._GRAD_WRITES[dev.index] = (stream, None)  # (the event recorded by the next writer that needs it)
        for p, t in direct:
            p.grad = t
        colors_grad = None if ctx.has_sh else targets.get("colors")
        return (None, returned.get("xyz"), returned.get("f_dc"), returned.get("f_rest"), colors_grad,
                returned.get("opacity"), returned.get("scaling"), returned.get("rotation"),
                *[d_m2[v] for v in range(n)])


class RenderedViews(list):
    """render_views()' list of per-view dicts; check() validates a speculated batch (see ViewBatch.check)."""

    batch = None

    def check(self) -> bool:
        return True if self.batch is None else self.batch.check()


def render_views_batched(cameras, pc, pipe, bg_color, streams, scaling_modifier=1.0, override_color=None,
                         speculate=False):
    """The views of `cameras` through one _RasterizeViews node (see the module docstring); the caller
    checks _fused_ok(pc, pipe) and the batch size (<= GS_MAX_VIEWS)."""
    from .gaussian_renderer import _mask_rows, _settings, _viewspace_zeros

    xyz = pc._xyz
    dev = xyz.device
    index = _mask_rows(pc.mask) if getattr(pc, "localize", False) else None
    n_pts = index.numel() if index is not None else xyz.shape[0]
    debug = getattr(pipe, "debug", False)
    settings = [_settings(cam, bg_color, scaling_modifier, pc.active_sh_degree, debug) for cam in cameras]
    n = len(cameras)
    visible = torch.empty((n, n_pts), dtype=torch.bool, device=dev)
    if override_color is None:
        f_dc, f_rest, colors = pc._features_dc, pc._features_rest, None
    else:
        f_dc, f_rest, colors = None, None, _C._f32(override_color.float(), "colors")
    empty = torch.empty(0, dtype=torch.float32, device=dev)
    means2D = [_viewspace_zeros(n_pts, xyz.dtype, dev) for _ in range(n)]
    from .gaussian_renderer import _may_backward

    meta = {"settings": settings, "streams": [streams[v % len(streams)] for v in range(n)], "speculate": speculate,
            "index": None if index is None else _C._index32(index), "visible": visible,
            "forward_only": not _may_backward(xyz, f_dc, f_rest, colors, pc._opacity, pc._scaling, pc._rotation)}
    res = _RasterizeViews.apply(meta, _C._f32(xyz, "xyz"),
                                empty if f_dc is None else _C._features(f_dc, "features_dc"),
                                empty if f_rest is None else _C._features(f_rest, "features_rest"),
                                empty if colors is None else colors, _C._f32(pc._opacity, "opacity"),
                                _C._f32(pc._scaling, "scaling"), _C._f32(pc._rotation, "rotation"), *means2D)
    batch = meta["batch"]
    outs = RenderedViews()
    outs.batch = batch
    for v in range(n):
        d = {"render": res[v], "viewspace_points": means2D[v], "visibility_filter": visible[v], "radii": res[n + v],
             "depth_3dgs": res[2 * n + v]}
        if index is None and not meta["forward_only"]:  # (a forward-only render writes no marks)
            d["_live_rows"] = batch.touched(v)
        outs.append(d)
    return outs
