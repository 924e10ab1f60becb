"""Drop-in ``diff_gaussian_rasterization`` package backed by the gfx950 kernels.

Same public names, argument order, return tuples and errors as the
reference wrapper (gaussiansplatting/submodules/diff-gaussian-rasterization/
diff_gaussian_rasterization/__init__.py:26-364), so
``gaussiansplatting/gaussian_renderer/__init__.py`` imports it unchanged once
this package is on the import path under that name.

Differences that are deliberate:
  * the native calls go through the C ABI (include/gs_raster.h) on the
    caller's current HIP stream, not the legacy default stream;
  * the backward needs no zero-filled gradient tensors (every element is
    written) and is bitwise reproducible (no float atomics).
"""
from __future__ import annotations

from typing import NamedTuple

import os

import torch
import torch.nn as nn

from .. import _C


def cpu_deep_copy_tuple(input_tuple):
    return tuple(item.cpu().clone() if isinstance(item, torch.Tensor) else item for item in input_tuple)


def rasterize_gaussians(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                        raster_settings):
    return _RasterizeGaussians.apply(means3D, means2D, sh, colors_precomp, opacities, scales, rotations,
                                     cov3Ds_precomp, raster_settings)


def _call_with_snapshot(fn, args, debug, dump_name, what):
    """Debug mode keeps a CPU copy of the arguments and dumps it on failure (reference __init__.py:88-107)."""
    if not debug:
        return fn(*args)
    cpu_args = cpu_deep_copy_tuple(args)
    try:
        return fn(*args)
    except Exception:
        torch.save(cpu_args, dump_name)
        print(f"\nAn error occured in {what}. Please forward {dump_name} for debugging.")
        raise


def _no_grad_materialization(ctx, radii):
    """radii are integer and depth is forward-only: without this autograd would zero-fill a P-element
    int32 and an HxW fp32 gradient for them before every backward (two kernels per view)."""
    ctx.mark_non_differentiable(radii)
    ctx.set_materialize_grads(False)


def _serialize_scratch(ctx, dev):
    """The backward reuses scratch inside the forward's buffers (gradient records and flags, the live
    list, counters: gs_raster.h, gs_rasterize_backward), so two backward calls of ONE forward
    (retain_graph=True, or torch.autograd.grad then .backward) must not overlap.  On one stream they
    cannot; when a later call runs on another stream than the previous one, it first waits for that
    stream."""
    cur = torch.cuda.current_stream(dev)
    prev = getattr(ctx, "_bwd_stream", None)
    if prev is not None and prev != cur:
        cur.wait_stream(prev)
    ctx._bwd_stream = cur


class _RasterizeGaussians(torch.autograd.Function):
    @staticmethod
    def forward(ctx, means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3Ds_precomp,
                raster_settings):
        rs = raster_settings
        args = (rs.bg, means3D, colors_precomp, opacities, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, sh,
                rs.sh_degree, rs.campos, rs.prefiltered, rs.debug)
        num_rendered, color, depth, radii, geomBuffer, binningBuffer, imgBuffer = _call_with_snapshot(
            _C.rasterize_gaussians, args, rs.debug, "snapshot_fw.dump", "forward")
        ctx.raster_settings = rs
        ctx.num_rendered = num_rendered
        ctx.save_for_backward(colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer,
                              binningBuffer, imgBuffer)
        _no_grad_materialization(ctx, radii)
        return color, radii, depth

    @staticmethod
    def backward(ctx, grad_out_color, grad_radii, grad_depth):
        # depth is forward-only, as in the reference (__init__.py:137, 155-177)
        if grad_out_color is None:  # the image took no part in the loss: every gradient is zero
            return (None,) * 9
        rs = ctx.raster_settings
        (colors_precomp, means3D, scales, rotations, cov3Ds_precomp, radii, sh, geomBuffer, binningBuffer,
         imgBuffer) = ctx.saved_tensors
        _serialize_scratch(ctx, means3D.device)
        args = (rs.bg, means3D, radii, colors_precomp, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_out_color, sh, rs.sh_degree, rs.campos,
                geomBuffer, ctx.num_rendered, binningBuffer, imgBuffer, rs.debug)
        (grad_means2D, grad_colors_precomp, grad_opacities, grad_means3D, grad_cov3Ds_precomp, grad_sh, grad_scales,
         grad_rotations) = _call_with_snapshot(_C.rasterize_gaussians_backward, args, rs.debug, "snapshot_bw.dump",
                                               "backward")
        return (grad_means3D, grad_means2D, grad_sh, grad_colors_precomp, grad_opacities, grad_scales, grad_rotations,
                grad_cov3Ds_precomp, None)


class RecolorPrepared:
    """`prepared` of _RasterizeGaussiansFused for a render that is already finished: the recolor of an earlier
    forward's buffers with other colours (dge_amd.gaussian_renderer, DGE's semantic render)."""

    def __init__(self, num_rendered, color, depth, radii):
        self.num_rendered, self.color, self.depth, self.radii = num_rendered, color, depth, radii


class _RasterizeGaussiansFused(torch.autograd.Function):
    """Rasterize straight from a GaussianModel's raw tensors (not part of the
    reference API; used by dge_amd.gaussian_renderer.render when the model has
    the standard activations).  Same outputs as getters + rasterize_gaussians;
    the backward returns gradients w.r.t. the raw tensors (what autograd through
    the getters would produce), without the getters' separate torch kernels."""

    @staticmethod
    def forward(ctx, xyz, means2D, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, raster_settings,
                index=None, visible=None, prepared=None, recompute=False):
        # prepared: the first half of this very forward, already enqueued by rasterize_gaussians_fused_begin
        # with these inputs (dge_amd.multiview.render_views begins every view before ending any).
        # recompute: `prepared` is a forward_only render (no backward bookkeeping in its buffers); a
        # backward, if one comes, first renders the same inputs again with it
        rs = raster_settings
        if isinstance(prepared, RecolorPrepared):  # (finished already: gs_render_recolor over another forward)
            num_rendered, color, depth, radii = prepared.num_rendered, prepared.color, prepared.depth, prepared.radii
            geomBuffer = binningBuffer = imgBuffer = torch.empty(0, dtype=torch.uint8, device=xyz.device)
        elif prepared is not None:
            num_rendered, color, depth, radii, geomBuffer, binningBuffer, imgBuffer = \
                _C.rasterize_gaussians_fused_end(prepared)
            if not recompute:  # (a forward with backward bookkeeping: a recolor may reuse its buffers)
                prepared.finished = (num_rendered, geomBuffer, binningBuffer, imgBuffer)
        else:
            args = (rs.bg, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, rs.scale_modifier,
                    rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width,
                    rs.sh_degree, rs.campos, rs.prefiltered, rs.debug)
            num_rendered, color, depth, radii, geomBuffer, binningBuffer, imgBuffer = _call_with_snapshot(
                lambda *a: _C.rasterize_gaussians_fused(*a, index=index, visible=visible), args, rs.debug,
                "snapshot_fw.dump", "forward")
        ctx.raster_settings = rs
        ctx.index = index
        ctx.num_rendered = num_rendered
        ctx.recompute = bool(recompute)
        ctx.means2D = means2D  # (a deferred backward hands its gradient over itself: _defer_pass)
        ctx.has_sh = f_dc is not None and f_dc.numel() != 0
        ctx.save_for_backward(xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, radii, geomBuffer,
                              binningBuffer, imgBuffer)
        _no_grad_materialization(ctx, radii)
        return color, radii, depth

    @staticmethod
    def backward(ctx, grad_out_color, grad_radii, grad_depth):
        if grad_out_color is None:
            return (None,) * 13
        rs = ctx.raster_settings
        (xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, radii, geomBuffer, binningBuffer,
         imgBuffer) = ctx.saved_tensors
        if ctx.recompute:  # (a lazy forward-only render: its buffers hold no backward bookkeeping)
            fa = (rs.bg, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, rs.scale_modifier,
                  rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width,
                  rs.sh_degree, rs.campos, rs.prefiltered, rs.debug)
            ctx.num_rendered, _, _, radii, geomBuffer, binningBuffer, imgBuffer = _C.rasterize_gaussians_fused(
                *fa, index=ctx.index)
            ctx.recompute = False
            ctx.lazy_buffers = (radii, geomBuffer, binningBuffer, imgBuffer)  # (a second backward reuses them)
        elif getattr(ctx, "lazy_buffers", None) is not None:
            radii, geomBuffer, binningBuffer, imgBuffer = ctx.lazy_buffers
        # Fused gradient accumulation: where autograd would add this gradient into a parameter's .grad
        # itself, the kernel writes (or adds) it there directly and autograd receives None — saving the
        # separate read-modify-write pass over every parameter.
        into, direct = {}, []
        masked, owners = set(), set()
        if _FUSED_GRAD_ACCUM and not torch.is_grad_enabled():
            # forward inputs: xyz 0, means2D 1, f_dc 2, f_rest 3, colors 4, opacity 5, scaling 6, rotation 7
            try:
                nf = ctx.next_functions
            except Exception:
                nf = None
            node = (lambda i: nf[i][0]) if nf is not None else (lambda i: None)
            for name, p, i in (("xyz", xyz, 0), ("opacity", raw_opacity, 5), ("scaling", raw_scaling, 6),
                               ("rotation", raw_rotation, 7)):
                mode, owner = _accumulation_mode(p, node(i))
                if mode is not None:
                    into[name] = _into_target(p, mode, direct, ctx.index is not None)
                    if owner is not None:
                        masked.add(name)
                        owners.add(owner)
            if ctx.has_sh:
                (m_dc, o_dc), (m_rest, o_rest) = _accumulation_mode(f_dc, node(2)), _accumulation_mode(f_rest, node(3))
                if m_dc is not None and m_dc == m_rest and o_dc is o_rest:
                    zi = ctx.index is not None
                    into["sh"] = ((_into_target(f_dc, m_dc, direct, zi)[0],
                                   _into_target(f_rest, m_rest, direct, zi)[0]), m_dc == "add")
                    if o_dc is not None:
                        masked.add("sh")
                        owners.add(o_dc)
        if masked:
            # the GaussianModel's grad-mask hooks, applied in-kernel with the owner's current mask
            mask = next(iter(owners)).mask if len(owners) == 1 else None
            if (mask is None or mask.dtype != torch.bool or mask.shape != (xyz.shape[0],)
                    or mask.device != xyz.device):
                # not expressible in-kernel: hand those gradients back to autograd (which runs the hooks)
                for name in masked:
                    if name == "sh":
                        tgt = (f_dc, f_rest)
                    else:
                        tgt = ({"xyz": xyz, "opacity": raw_opacity, "scaling": raw_scaling,
                                "rotation": raw_rotation}[name],)
                    direct[:] = [(p, t) for p, t in direct if all(p is not q for q in tgt)]
                    del into[name]
                masked = set()
            else:
                into["grad_mask"] = (mask.contiguous().view(torch.uint8), masked)
        args = (rs.bg, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, radii, rs.scale_modifier,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, grad_out_color, rs.sh_degree, rs.campos,
                geomBuffer, ctx.num_rendered, binningBuffer, imgBuffer, rs.debug)
        _serialize_scratch(ctx, xyz.device)
        _ZEROED.pop(xyz.device.index, None)  # (this backward writes .grad: the buffer is no longer all zeros)
        _DIRTY.pop(xyz.device.index, None)   # (... at rows it does not record)
        m2 = getattr(ctx, "means2D", None)
        m2_mode = _accumulation_mode(m2, node(1))[0] if into and _DEFER_PASSES else None
        if (m2_mode is not None and ctx.index is None and ctx.has_sh and not rs.debug
                and all(k in into for k in ("xyz", "opacity", "scaling", "rotation", "sh"))):
            # every gradient goes into a .grad: enqueue the gradient replay now and this view's per-Gaussian
            # pass at the end of the backward, merged with the other views' (_defer_pass)
            # (consecutive views' replays on different streams: the latency-bound replays overlap)
            side = _replay_stream(xyz.device)
            if side is not None:
                side.wait_stream(torch.cuda.current_stream(xyz.device))
            out, pend = _C.rasterize_gaussians_fused_backward(*args, into=into, index=None, defer=True, stream=side)
            for p, t in direct:  # (written by the deferred pass; the next view's backward adds into them)
                p.grad = t
            _defer_pass(xyz.device, pend, m2, m2_mode, out[0], [t for _, t in direct], side)
            return (None,) * 13
        ordered = bool(into) and _SIDE_STREAMS
        stream, after = _order_grad_writes_begin(xyz.device) if ordered else (None, None)
        d_m2, d_xyz, d_dc, d_rest, d_col, d_op, d_sc, d_rot = _call_with_snapshot(
            lambda *a: _C.rasterize_gaussians_fused_backward(*a, into=into, index=ctx.index, writes_after=after),
            args, rs.debug, "snapshot_bw.dump", "backward")
        if ordered:
            _order_grad_writes_end(xyz.device, stream, [t for _, t in direct])
        for p, t in direct:  # parameters whose .grad was None: the kernel wrote it, hand it over
            p.grad = t
        if ctx.has_sh:
            d_col = None
        else:
            d_dc = d_rest = None
        if "xyz" in into:
            d_xyz = None
        if "opacity" in into:
            d_op = None
        if "scaling" in into:
            d_sc = None
        if "rotation" in into:
            d_rot = None
        if "sh" in into:
            d_dc = d_rest = None
        return d_xyz, d_m2, d_dc, d_rest, d_col, d_op, d_sc, d_rot, None, None, None, None, None


_FUSED_GRAD_ACCUM = os.environ.get("DGE_AMD_FUSED_GRAD_ACCUM", "1") != "0"

# Deferred per-Gaussian passes.  DGE renders its views one by one and backpropagates their stacked loss once
# (threestudio/systems/DGE.py:179-222, 672): autograd then runs the views' backward nodes one after
# another.  When a view's gradients all go into .grad buffers (the fused accumulation above), its backward
# enqueues only the gradient replay; the per-Gaussian passes of all such views of the backward run at its
# end (an autograd final callback, before backward() returns) as ONE merged pass
# (gs_rasterize_backward_passes, the pass the batched views path runs) — the same sums in the same view
# order, bitwise.  The view-space gradients (dL/dmeans2D) are handed to their leaves there.
_DEFER_PASSES = os.environ.get("DGE_AMD_DEFER_PASSES", "1") != "0"
_PENDING_PASSES = {}  # device index -> [(PendingBackward, replay event, means2D leaf, mode, dL/dmeans2D, fresh)]
_REPLAY_STREAMS = {}  # device index -> the side streams deferred replays rotate over (with the current one)
# (2 side streams measured within the noise of one stream in DGE's loop, 1101-1171 vs 1107-1220 views/s:
# its replays follow one another on the caller's stream by default)
_REPLAY_SIDE = int(os.environ.get("DGE_AMD_REPLAY_STREAMS", "0"))


_PENDING_TASK = {}  # device index -> the autograd graph task whose final callback runs _PENDING_PASSES


def _flush_stale_passes(dev):
    """Run the deferred passes a previous backward left behind.  A backward that raised after a view was
    deferred (OOM, anomaly mode, an interrupt) never ran its final callback; its pending list is tied to that
    graph task, so the next backward sees another task id, runs the stale passes first (the .grad buffers
    they target are then fully written, never left as uninitialised memory) and queues its own callback."""
    if dev.index in _PENDING_PASSES and _PENDING_TASK.get(dev.index) != torch._C._current_graph_task_id():
        _run_deferred_passes(dev)


def _replay_stream(dev):
    """The stream the next deferred replay of this backward runs on: the current stream for the first, then
    _REPLAY_SIDE side streams in turn (None: the current stream).  The replay reads and writes only tensors
    its PendingBackward holds, and the deferred passes wait for it."""
    _flush_stale_passes(dev)
    k = len(_PENDING_PASSES.get(dev.index, ()))
    if _REPLAY_SIDE <= 0 or k % (_REPLAY_SIDE + 1) == 0:
        return None
    pool = _REPLAY_STREAMS.get(dev.index)
    if pool is None:
        pool = _REPLAY_STREAMS[dev.index] = [torch.cuda.Stream(device=dev) for _ in range(_REPLAY_SIDE)]
    return pool[k % (_REPLAY_SIDE + 1) - 1]


def _defer_pass(dev, pend, m2, m2_mode, d_m2, fresh, stream=None):
    _flush_stale_passes(dev)
    lst = _PENDING_PASSES.get(dev.index)
    if lst is None:
        lst = _PENDING_PASSES[dev.index] = []
        _PENDING_TASK[dev.index] = torch._C._current_graph_task_id()
        torch.autograd.Variable._execution_engine.queue_callback(lambda d=dev: _run_deferred_passes(d))
    ev = (stream if stream is not None else torch.cuda.current_stream(dev)).record_event()
    lst.append((pend, ev, m2, m2_mode, d_m2, fresh))


def _run_deferred_passes(dev):
    lst = _PENDING_PASSES.pop(dev.index, None)
    _PENDING_TASK.pop(dev.index, None)
    if not lst:
        return
    cur = torch.cuda.current_stream(dev)
    for _, ev, *_rest in lst:
        cur.wait_event(ev)
    pend = [e[0] for e in lst if e[0] is not None]
    stream, after = _order_grad_writes_begin(dev) if _SIDE_STREAMS else (None, None)
    if pend:
        pend[0].set_writes_after(after)
        _C.rasterize_backward_passes(pend)
    if _SIDE_STREAMS:
        _order_grad_writes_end(dev, stream, [t for e in lst for t in e[5]])
    for _, _, m2, mode, d_m2, _ in lst:  # (what means2D's AccumulateGrad would have done)
        if m2.grad is None:
            m2.grad = d_m2
        else:
            m2.grad.add_(d_m2)

# In-kernel .grad writes of backward calls that autograd runs on different streams (views rendered
# concurrently, dge_amd.multiview.render_views: each view's backward runs on its forward's stream)
# are chained with events, and the default stream waits for them, so an optimizer step or an
# all-reduce issued there sees the gradients.  Backward calls on the default stream need nothing.
_GRAD_WRITES = {}  # device index -> (stream, event) of the last side-stream .grad write
_SIDE_STREAMS = False  # set once dge_amd.multiview.stream_pool hands out streams
# device index -> (flat gradient buffer, its version counter right after GradBucket.zero()): the buffer
# holds zeros until a backward writes into it (the native backward calls take the entry; a torch
# in-place write shows as a version change).  A batched backward whose .grad targets all lie in it stores
# each Gaussian's first gradient instead of adding it (gs_grads.zeroed: the zeros are never read).
_ZEROED = {}
# device index -> [flat, dirty, version]: a row-major GradBucket's record of the rows written since its last
# clear (gs_grads.dirty_rows: the batched backward marks its live rows; the sparse all-reduce marks the rows
# it scatters).  Valid while the buffer's version is unchanged and no unmarked writer ran (the per-view fused
# backward drops it): the bucket's next zero() then clears those rows only (gs_rows_zero_dirty).
_DIRTY = {}


def dirty_rows(dev, tensors):
    """The dirty-row mask (a uint8 tensor) of the tracked bucket on `dev` if every tensor lies in it, else None."""
    rec = _DIRTY.get(dev.index)
    if rec is None or rec[0]._version != rec[2]:
        return None
    flat = rec[0]
    lo, hi = flat.data_ptr(), flat.data_ptr() + 4 * flat.numel()
    for t in tensors:
        if t is None or not (lo <= t.data_ptr() and t.data_ptr() + 4 * t.numel() <= hi):
            return None
    return rec[1]


def zeroed_bits(dev, tensors, bits: int) -> int:
    """`bits` if every tensor lies in the buffer GradBucket.zero() registered for `dev` and nothing has
    written into that buffer since (the entry is taken: the caller's backward is the next writer), else 0."""
    ent = _ZEROED.pop(dev.index, None)
    if ent is None or not bits or os.environ.get("DGE_AMD_ZEROED", "1") == "0":  # (=0: A/B against the add path)
        return 0
    flat, version = ent
    if flat._version != version:
        return 0
    lo, hi = flat.data_ptr(), flat.data_ptr() + 4 * flat.numel()
    for t in tensors:
        if t is None or t.dtype != torch.float32 or not (lo <= t.data_ptr() and t.data_ptr() + 4 * t.numel() <= hi):
            return 0
    return bits


def _order_grad_writes_begin(dev):
    """(current stream, the event its .grad writes must wait for or None).  The wait is placed by the
    backward itself right before its per-Gaussian pass (gs_grads.writes_after), so this view's gradient
    replay still overlaps the previous view's gradient writes on the other stream."""
    cur = torch.cuda.current_stream(dev)
    return cur, grad_writes_event(dev, cur)


def grad_writes_event(dev, cur):
    """The event `cur`'s .grad writes must wait for: the last gradient writer's, when it was another stream,
    else None.  A writer may leave its event unrecorded (None: views' batched backward, whose stream is then
    recorded here, on demand — after everything enqueued on it so far, a superset of its gradient writes), so
    a step whose next writer is on the same stream puts no event (a system-fenced marker) in its queue."""
    last = _GRAD_WRITES.get(dev.index)
    if last is None or last[0] == cur:
        return None
    if last[1] is None:
        last = _GRAD_WRITES[dev.index] = (last[0], last[0].record_event())
    return last[1]


def _order_grad_writes_end(dev, cur, fresh):
    dflt = torch.cuda.default_stream(dev)
    if cur == dflt:
        _GRAD_WRITES.pop(dev.index, None)
        return
    ev = cur.record_event()
    dflt.wait_event(ev)
    for t in fresh:  # new .grad tensors allocated on the side stream, used on the default one
        t.record_stream(dflt)
    _GRAD_WRITES[dev.index] = (cur, ev)


def set_fused_grad_accumulation(enabled: bool) -> bool:
    """Switch the fused gradient accumulation of the raw-parameter path on/off; returns the previous
    setting (environment default: DGE_AMD_FUSED_GRAD_ACCUM, on unless "0")."""
    global _FUSED_GRAD_ACCUM
    prev, _FUSED_GRAD_ACCUM = _FUSED_GRAD_ACCUM, bool(enabled)
    return prev


def _mask_owner(p):
    """(ok, owner): p's tensor hooks are none (owner None) or only GaussianModel grad-mask hooks of one
    model (dge_amd/gaussian_model.py apply_grad_mask, tagged _dge_grad_mask_owner); ok False otherwise."""
    hooks = getattr(p, "_backward_hooks", None)
    if not hooks:
        return True, None
    owners = {id(getattr(h, "_dge_grad_mask_owner", None)): getattr(h, "_dge_grad_mask_owner", None)
              for h in hooks.values()}
    if len(owners) == 1:
        owner = next(iter(owners.values()))
        if owner is not None:
            return True, owner
    return False, None


def _accumulation_mode(p, node=None):
    """("add" | "new" | None, mask owner): "add"/"new" when this backward's gradient for leaf `p` may go
    straight into p.grad.

    Only where autograd itself would run p's AccumulateGrad in this backward (so torch.autograd.grad
    callers, which capture instead, still get returned gradients), p has no post-accumulate hooks and
    no tensor hooks other than a GaussianModel's grad mask (applied in-kernel), and an existing .grad is
    a plain contiguous fp32 buffer of p's shape."""
    if (not isinstance(p, torch.Tensor) or not p.requires_grad or p.grad_fn is not None or p.numel() == 0
            or p.dtype != torch.float32):  # (the kernels write fp32 gradients)
        return None, None
    ok, owner = _mask_owner(p)
    if not ok or getattr(p, "_post_accumulate_grad_hooks", None):
        return None, None
    try:
        if node is None or getattr(node, "variable", None) is not p:
            # the leaf's AccumulateGrad node (callers inside a backward pass the one from
            # ctx.next_functions, which avoids building a view per parameter)
            with torch.enable_grad():
                node = p.view_as(p).grad_fn.next_functions[0][0]
        if not torch._C._will_engine_execute_node(node):
            return None, None
    except Exception:
        return None, None
    g = p.grad
    if g is None:
        return "new", owner
    # (a contiguous .grad, or a column block of a row-major gradient bucket: rows at a pitch, written in place)
    if (g.shape == p.shape and g.dtype == torch.float32 and g.device == p.device and not g.requires_grad
            and (g.is_contiguous() or _C.row_pitch_ok(g))):
        # the kernels store a rotation gradient row as one float4: its rows 16-B aligned, the pitch a multiple
        # of 4 (what gs_rasterize_backward_ex validates); any other .grad of that shape goes back to autograd
        if g.dim() == 2 and g.shape[1] == 4 and (g.stride(0) % 4 or g.data_ptr() % 16):
            return None, None
        return "add", owner
    return None, None


def _into_target(p, mode, direct, zero=False):
    """zero: the kernel writes only some rows (the index path), so a fresh .grad starts at zero."""
    if mode == "add":
        return (p.grad, True)
    t = (torch.zeros_like if zero else torch.empty_like)(p, memory_format=torch.contiguous_format)
    direct.append((p, t))
    return (t, False)


def rasterize_gaussian_model(xyz, means2D, features_dc, features_rest, colors_precomp, raw_opacity, raw_scaling,
                             raw_rotation, raster_settings, index=None, visible=None, prepared=None, recompute=False):
    """(color, radii, depth) of a GaussianModel given its raw tensors (_xyz, _features_dc, _features_rest or
    colors_precomp, _opacity, _scaling, _rotation); activations are applied in-kernel.  `index` (int32,
    ascending): render only those rows — the model's `localize` subset pc[mask] — gathering them
    in-kernel; the gradients land in the full-size tensors' rows (means2D/radii are per subset entry).
    prepared: this forward's first half from _C.rasterize_gaussians_fused_begin (same inputs)."""
    empty = torch.empty(0, dtype=torch.float32, device=xyz.device)
    return _RasterizeGaussiansFused.apply(
        xyz, means2D, empty if features_dc is None else features_dc, empty if features_rest is None else features_rest,
        empty if colors_precomp is None else colors_precomp, raw_opacity, raw_scaling, raw_rotation, raster_settings,
        index, visible, prepared, recompute)


class GaussianRasterizationSettings(NamedTuple):
    image_height: int
    image_width: int
    tanfovx: float
    tanfovy: float
    bg: torch.Tensor
    scale_modifier: float
    viewmatrix: torch.Tensor
    projmatrix: torch.Tensor
    sh_degree: int
    campos: torch.Tensor
    prefiltered: bool
    debug: bool


def _absent(like):
    return torch.empty(0, dtype=torch.float32, device=like.device)


class GaussianRasterizer(nn.Module):
    def __init__(self, raster_settings):
        super().__init__()
        self.raster_settings = raster_settings

    def markVisible(self, positions):
        with torch.no_grad():
            rs = self.raster_settings
            return _C.mark_visible(positions, rs.viewmatrix, rs.projmatrix)

    def forward(self, means3D, means2D, opacities, shs=None, colors_precomp=None, scales=None, rotations=None,
                cov3D_precomp=None):
        rs = self.raster_settings
        if (shs is None) == (colors_precomp is None):
            raise Exception("Please provide excatly one of either SHs or precomputed colors!")
        if ((scales is None or rotations is None) and cov3D_precomp is None) or (
                (scales is not None or rotations is not None) and cov3D_precomp is not None):
            raise Exception("Please provide exactly one of either scale/rotation pair or precomputed 3D covariance!")
        shs = _absent(means3D) if shs is None else shs
        colors_precomp = _absent(means3D) if colors_precomp is None else colors_precomp
        scales = _absent(means3D) if scales is None else scales
        rotations = _absent(means3D) if rotations is None else rotations
        cov3D_precomp = _absent(means3D) if cov3D_precomp is None else cov3D_precomp
        return rasterize_gaussians(means3D, means2D, shs, colors_precomp, opacities, scales, rotations, cov3D_precomp,
                                   rs)

    def apply_weights(self, means3D, means2D, opacities, shs=None, weights=None, scales=None, rotations=None,
                      cov3Ds_precomp=None, cnt=None, image_weights=None):
        assert weights is not None
        assert cnt is not None
        assert image_weights is not None
        rs = self.raster_settings
        shs = _absent(means3D) if shs is None else shs
        scales = _absent(means3D) if scales is None else scales
        rotations = _absent(means3D) if rotations is None else rotations
        cov3Ds_precomp = _absent(means3D) if cov3Ds_precomp is None else cov3Ds_precomp
        args = (rs.bg, means3D, weights, opacities, scales, rotations, rs.scale_modifier, cov3Ds_precomp,
                rs.viewmatrix, rs.projmatrix, rs.tanfovx, rs.tanfovy, rs.image_height, rs.image_width, shs,
                rs.sh_degree, rs.campos, rs.prefiltered, image_weights, cnt, rs.debug)
        _C.apply_weights(*args)


__all__ = ["GaussianRasterizationSettings", "GaussianRasterizer", "rasterize_gaussians", "_RasterizeGaussians"]
