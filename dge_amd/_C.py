"""Torch binding of the C ABI with the reference's ``_C`` surface.

Mirrors ``diff_gaussian_rasterization._C`` (ext.cpp:15-20) argument for
argument, so the Python wrapper in ``dge_amd.diff_gaussian_rasterization``
reads like the reference's:

  rasterize_gaussians            <- RasterizeGaussiansCUDA          rasterize_points.cu:35-95
  rasterize_gaussians_backward   <- RasterizeGaussiansBackwardCUDA  rasterize_points.cu:97-157
  mark_visible                   <- markVisible                     rasterize_points.cu:159-175
  apply_weights                  <- applyWeightsGaussiansCUDA       rasterize_points.cu:177-234

Empty tensors mean "absent" and become NULL pointers, as in the reference.
The opaque geometry/binning/image byte buffers are torch uint8 tensors
allocated through the C ABI's allocator callback (the reference's resize
functors, rasterize_points.cu:27-33) on the caller's current stream.
"""
from __future__ import annotations

import ctypes
import os
import threading
import weakref

import torch

from . import _native as N


def _ptr(t):
    """Device address of a tensor, or None for an absent (empty/None) one."""
    if t is None or t.numel() == 0:
        return None
    return t.data_ptr()


def _f32(t, name):
    """contiguous float32 view (the reference's .contiguous().data<float>())."""
    if t is None or t.numel() == 0:
        return t
    if t.dtype != torch.float32:
        raise RuntimeError(f"{name} must be float32 (got {t.dtype})")
    return t.contiguous()


def _sh_tensor(sh):
    """SH as the kernels take them: contiguous fp32, or contiguous fp16 (upcast in-kernel)."""
    if sh is None or sh.numel() == 0:
        return sh
    if sh.dtype == torch.float16:
        return sh.contiguous()
    return _f32(sh, "sh")


def _sh_params(P, M, means3D, sh, colors, opacity, scales, rotations, cov3D_precomp):
    """gs_params for the reference's (already activated) inputs, SH [P,M,3] in fp32 or fp16."""
    g = N.GsParams()
    g.P, g.M = P, M
    g.means3D = _ptr(means3D)
    half = M > 0 and sh.dtype == torch.float16
    if M:
        g.sh_dc = sh.data_ptr()
        g.sh_rest = sh.data_ptr() + 3 * sh.element_size() if M > 1 else None  # coefficient 1
        g.sh_dc_stride = g.sh_rest_stride = 3 * M
    g.colors_precomp = _ptr(colors)
    g.opacities = _ptr(opacity)
    g.scales, g.rotations, g.cov3D_precomp = _ptr(scales), _ptr(rotations), _ptr(cov3D_precomp)
    g.activation = 0
    g.sh_half = 1 if half else 0
    return g


_TLS = threading.local()
_EMPTY_U8 = {}  # device -> empty uint8 tensor (placeholder for buffers never allocated)


def _alloc_cb(ctx, which, nbytes):
    # this thread's current allocator (the C call that receives the callback runs on this thread); the
    # buffer is allocated on the current stream
    a = _TLS.alloc
    buf = torch.empty(int(nbytes), dtype=torch.uint8, device=a.device)
    a.buffers[which] = buf
    return buf.data_ptr() if nbytes else None


_ALLOC_CB = N.ALLOC_FN(_alloc_cb)  # one ctypes thunk for the process (building one per call is slow)


class _Allocator:
    """gs_alloc_fn backed by the torch caching allocator.  The C call that receives `fn` runs on this
    thread right after construction; the shared callback finds this object through a thread-local."""

    def __init__(self, device):
        self.device = device
        e = _EMPTY_U8.get(device)
        if e is None:
            e = _EMPTY_U8[device] = torch.empty(0, dtype=torch.uint8, device=device)
        self.buffers = [e, e, e]
        _TLS.alloc = self
        self.fn = _ALLOC_CB


_CONTIG = {}  # id(tensor) -> (weakref, _version, contiguous copy)


def _f32_cached(t, name):
    """_f32 for the small per-camera tensors (the reference's cameras keep transposed, non-contiguous
    matrices: .contiguous() would copy them on every forward and backward).  The copy is reused while
    the source tensor is alive and unmodified (same object, same version counter)."""
    if t is None or t.numel() == 0 or t.is_contiguous():
        return _f32(t, name)
    ent = _CONTIG.get(id(t))
    if ent is not None and ent[0]() is t and ent[1] == t._version:
        return ent[2]
    c = _f32(t, name)
    key = id(t)
    _CONTIG[key] = (weakref.ref(t, lambda _r, k=key: _CONTIG.pop(k, None)), t._version, c)
    return c


def _settings(bg, viewmatrix, projmatrix, campos, tanfovx, tanfovy, H, W, sh_degree, scale_modifier, prefiltered,
              debug):
    keep = [_f32(bg, "bg"), _f32_cached(viewmatrix, "viewmatrix"), _f32_cached(projmatrix, "projmatrix"),
            _f32_cached(campos, "campos")]
    s = N.GsSettings()
    s.image_height = int(H)
    s.image_width = int(W)
    s.tanfovx = float(tanfovx)
    s.tanfovy = float(tanfovy)
    s.bg = _ptr(keep[0])
    s.scale_modifier = float(scale_modifier)
    s.viewmatrix = _ptr(keep[1])
    s.projmatrix = _ptr(keep[2])
    s.sh_degree = int(sh_degree)
    s.campos = _ptr(keep[3])
    s.prefiltered = int(bool(prefiltered))
    s.debug = int(bool(debug))
    return s, keep


_RAW_STREAM = getattr(torch._C, "_cuda_getCurrentRawStream", None)

# The compiled binding (dge_amd/csrc/gs_torch.cpp -> dge_amd/lib/_gs_torch*.so) of the calls DGE's loop makes per
# view: the raw-parameter forward's halves and the recolor.  It drives the library instance loaded above (its
# entry points handed over as addresses); DGE_AMD_BINDING=ctypes keeps every call on the ctypes path below.
_GT = None


def _load_binding():
    global _GT
    if os.environ.get("DGE_AMD_BINDING", "torch") == "ctypes" or _RAW_STREAM is None:
        return None
    import glob
    import importlib.machinery
    import importlib.util

    found = glob.glob(os.path.join(os.path.dirname(N.LIB_PATH), "_gs_torch*.so")) or \
        glob.glob(os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib", "_gs_torch*.so"))
    if not found:
        return None
    loader = importlib.machinery.ExtensionFileLoader("_gs_torch", found[0])
    spec = importlib.util.spec_from_file_location("_gs_torch", found[0], loader=loader)
    mod = importlib.util.module_from_spec(spec)
    loader.exec_module(mod)
    L = N.lib()
    mod.bind({n: ctypes.cast(getattr(L, n), ctypes.c_void_p).value for n in (
        "gs_rasterize_forward_begin", "gs_rasterize_forward_end", "gs_rasterize_forward_release",
        "gs_render_recolor", "gs_image_buffer_size")})
    _GT = mod
    return mod


def _raw_stream(device) -> int:
    return _RAW_STREAM(device.index if device.index is not None else torch.cuda.current_device())


def _stream(device):
    """The device's current stream as a hipStream_t (the raw query: no Stream object per call)."""
    if _RAW_STREAM is not None:
        idx = device.index if device.index is not None else torch.cuda.current_device()
        return ctypes.c_void_p(_RAW_STREAM(idx))
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class _Same:
    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


_SAME = _Same()


def _on(dev):
    """torch.cuda.device(dev), or nothing when dev is already the current device (the common case: a context
    switch costs a device query and two sets per call)."""
    if dev.index is None or torch.cuda.current_device() == dev.index:
        return _SAME
    return torch.cuda.device(dev)


def rasterize_gaussians(background, means3D, colors, opacity, scales, rotations, scale_modifier, cov3D_precomp,
                        viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos,
                        prefiltered, debug):
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    N.require_gpu(means3D)
    dev = means3D.device
    P = means3D.size(0)
    H, W = int(image_height), int(image_width)
    with _on(dev):
        means3D = _f32(means3D, "means3D")
        colors, opacity = _f32(colors, "colors"), _f32(opacity, "opacity")
        scales, rotations = _f32(scales, "scales"), _f32(rotations, "rotations")
        cov3D_precomp, sh = _f32(cov3D_precomp, "cov3D_precomp"), _sh_tensor(sh)
        out_color = torch.empty((3, H, W), dtype=torch.float32, device=dev)
        out_depth = torch.empty((1, H, W), dtype=torch.float32, device=dev)
        radii = torch.empty((P,), dtype=torch.int32, device=dev)
        M = sh.size(1) if sh is not None and sh.numel() != 0 else 0
        s, keep = _settings(background, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, H, W, degree,
                            scale_modifier, prefiltered, debug)
        alloc = _Allocator(dev)
        nr = ctypes.c_int(0)
        if M and sh.dtype == torch.float16:  # fp16 SH storage: the _ex entry point upcasts in-kernel
            g = _sh_params(P, M, means3D, sh, colors, opacity, scales, rotations, cov3D_precomp)
            rc = N.lib().gs_rasterize_forward_ex(ctypes.byref(s), ctypes.byref(g), _ptr(out_color), _ptr(out_depth),
                                                 _ptr(radii), alloc.fn, None, _stream(dev), ctypes.byref(nr))
        else:
            rc = N.lib().gs_rasterize_forward(ctypes.byref(s), P, M, _ptr(means3D), _ptr(sh), _ptr(colors),
                                              _ptr(opacity), _ptr(scales), _ptr(rotations), _ptr(cov3D_precomp),
                                              _ptr(out_color), _ptr(out_depth), _ptr(radii), alloc.fn, None,
                                              _stream(dev), ctypes.byref(nr))
        N.check(rc, "rasterize_gaussians")
        if P == 0:
            radii.zero_()
        geom, binning, img = alloc.buffers
        del keep
        return nr.value, out_color, out_depth, radii, geom, binning, img


def rasterize_gaussians_backward(background, means3D, radii, colors, scales, rotations, scale_modifier, cov3D_precomp,
                                 viewmatrix, projmatrix, tan_fovx, tan_fovy, dL_dout_color, sh, degree, campos,
                                 geomBuffer, R, binningBuffer, imageBuffer, debug, dL_dconic=None):
    """rasterize_points.cu:97-157.  `dL_dconic` (not in the reference's API; parity tests): a [P,3]
    float32 tensor that receives each Gaussian's summed conic gradient (x, y, w of the reference's
    [P,2,2] dL_dconic2D)."""
    N.require_gpu(means3D)
    dev = means3D.device
    P = means3D.size(0)
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    M = sh.size(1) if sh is not None and sh.numel() != 0 else 0
    with _on(dev):
        opts = dict(dtype=torch.float32, device=dev)
        out = (torch.empty((P, 3), **opts), torch.empty((P, 3), **opts), torch.empty((P, 1), **opts),
               torch.empty((P, 3), **opts), torch.empty((P, 6), **opts), torch.empty((P, M, 3), **opts),
               torch.empty((P, 3), **opts), torch.empty((P, 4), **opts))
        if P == 0:
            return out
        means3D = _f32(means3D, "means3D")
        colors, sh = _f32(colors, "colors"), _sh_tensor(sh)
        scales, rotations = _f32(scales, "scales"), _f32(rotations, "rotations")
        cov3D_precomp = _f32(cov3D_precomp, "cov3D_precomp")
        radii = radii.contiguous()
        if radii.dtype != torch.int32:
            raise RuntimeError("radii must be int32")
        grad = _f32(dL_dout_color, "dL_dout_color")
        s, keep = _settings(background, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, H, W, degree,
                            scale_modifier, False, debug)
        dmeans2D, dcolors, dopac, dmeans3D, dcov, dsh, dscales, drot = out
        if (M and sh.dtype == torch.float16) or dL_dconic is not None:
            # _ex entry point: fp16 SH (fp32 SH gradients [P,M,3]) or the conic-gradient output
            g = _sh_params(P, M, means3D, sh, colors, None, scales, rotations, cov3D_precomp)
            o = N.GsGrads()
            o.dL_dmeans2D, o.dL_dcolors, o.dL_dopacity = _ptr(dmeans2D), _ptr(dcolors), _ptr(dopac)
            o.dL_dmeans3D, o.dL_dcov3D = _ptr(dmeans3D), _ptr(dcov)
            o.dL_dsh_dc = _ptr(dsh)
            o.dL_dsh_rest = dsh.data_ptr() + 12 if M > 1 else None
            o.dsh_dc_stride = o.dsh_rest_stride = 3 * M
            o.dL_dscales, o.dL_drotations = _ptr(dscales), _ptr(drot)
            if dL_dconic is not None:
                if dL_dconic.shape != (P, 3) or dL_dconic.dtype != torch.float32 or not dL_dconic.is_contiguous():
                    raise RuntimeError("dL_dconic must be a contiguous float32 [P,3] tensor")
                o.dL_dconic = _ptr(dL_dconic)
            rc = N.lib().gs_rasterize_backward_ex(ctypes.byref(s), ctypes.byref(g), int(R), _ptr(radii),
                                                  _ptr(geomBuffer), _ptr(binningBuffer), _ptr(imageBuffer),
                                                  _ptr(grad), ctypes.byref(o), _stream(dev))
            N.check(rc, "rasterize_gaussians_backward")
            del keep
            return out
        rc = N.lib().gs_rasterize_backward(
            ctypes.byref(s), P, M, int(R), _ptr(means3D), _ptr(sh), _ptr(colors), _ptr(scales), _ptr(rotations),
            _ptr(cov3D_precomp), _ptr(radii), _ptr(geomBuffer), _ptr(binningBuffer), _ptr(imageBuffer), _ptr(grad),
            _ptr(dmeans2D), _ptr(dcolors), _ptr(dopac), _ptr(dmeans3D), _ptr(dcov), _ptr(dsh), _ptr(dscales),
            _ptr(drot), _stream(dev))
        N.check(rc, "rasterize_gaussians_backward")
        del keep
        return out


def mark_visible(means3D, viewmatrix, projmatrix):
    N.require_gpu(means3D)
    dev = means3D.device
    P = means3D.size(0)
    with _on(dev):
        present = torch.zeros((P,), dtype=torch.bool, device=dev)
        if P == 0:
            return present
        m = _f32(means3D, "means3D")
        v = _f32(viewmatrix, "viewmatrix")
        p = _f32(projmatrix, "projmatrix")
        rc = N.lib().gs_mark_visible(P, _ptr(m), _ptr(v), _ptr(p), _ptr(present), _stream(dev))
        N.check(rc, "mark_visible")
        return present


def apply_weights(background, means3D, weights, opacity, scales, rotations, scale_modifier, cov3D_precomp, viewmatrix,
                  projmatrix, tan_fovx, tan_fovy, image_height, image_width, sh, degree, campos, prefiltered,
                  image_weights, cnt, debug):
    if means3D.ndimension() != 2 or means3D.size(1) != 3:
        raise RuntimeError("means3D must have dimensions (num_points, 3)")
    N.require_gpu(means3D)
    dev = means3D.device
    P = means3D.size(0)
    C = int(image_weights.size(0))
    if P == 0:
        return None
    if not (weights.is_contiguous() and cnt.is_contiguous()):
        raise RuntimeError("apply_weights updates weights and cnt in place: they must be contiguous")
    if weights.dtype != torch.float32 or cnt.dtype != torch.int32:
        raise RuntimeError("weights must be float32 and cnt int32")
    with _on(dev):
        means3D, opacity = _f32(means3D, "means3D"), _f32(opacity, "opacity")
        scales, rotations = _f32(scales, "scales"), _f32(rotations, "rotations")
        cov3D_precomp, sh = _f32(cov3D_precomp, "cov3D_precomp"), _f32(sh, "sh")
        iw = _f32(image_weights, "image_weights")
        M = sh.size(1) if sh is not None and sh.numel() != 0 else 0
        s, keep = _settings(background, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, image_height, image_width,
                            degree, scale_modifier, prefiltered, debug)
        alloc = _Allocator(dev)
        rc = N.lib().gs_apply_weights(ctypes.byref(s), P, M, _ptr(means3D), _ptr(weights), C, _ptr(opacity),
                                      _ptr(scales), _ptr(rotations), _ptr(cov3D_precomp), _ptr(sh), _ptr(iw),
                                      _ptr(cnt), alloc.fn, None, _stream(dev))
        N.check(rc, "apply_weights")
        del keep, alloc
        return None


# ---------------------------------------------------------------------------
# fused path: raw GaussianModel parameters, activations and SH split in-kernel
# (gs_rasterize_forward_ex / gs_rasterize_backward_ex)
# ---------------------------------------------------------------------------
def _params(P, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, index=None, visible=None,
            forward_only=False, aux_mask=None):
    """gs_params of the raw-parameter path; `index` (int32 [P], ascending): the localize subset's rows
    (gathered in-kernel); fp16 features are read as such (sh_half); forward_only: no backward will follow
    (the kernels skip the backward's scratch); aux_mask: a uint8 tensor over the parameter rows whose 0/1
    the blend composites beside the colour (gs_params.aux_mask, served to render_recolor)."""
    g = N.GsParams()
    g.P = P
    g.forward_only = 1 if forward_only else 0
    g.aux_mask = _ptr(aux_mask)
    g.index = _ptr(index)
    g.sh_half = 1 if f_dc is not None and f_dc.dtype == torch.float16 else 0
    have_sh = f_dc is not None and f_dc.numel() != 0
    Mr = f_rest.size(1) if have_sh and f_rest is not None and f_rest.numel() != 0 else 0
    g.M = (1 + Mr) if have_sh else 0
    g.means3D = _ptr(xyz)
    g.sh_dc = _ptr(f_dc) if have_sh else None
    g.sh_rest = _ptr(f_rest) if Mr else None
    g.sh_dc_stride = 3
    g.sh_rest_stride = 3 * Mr
    g.colors_precomp = None if have_sh else _ptr(colors)
    g.opacities = _ptr(raw_opacity)
    g.scales = _ptr(raw_scaling)
    g.rotations = _ptr(raw_rotation)
    g.cov3D_precomp = None
    g.activation = 1
    if visible is not None:
        if visible.dtype != torch.bool or visible.numel() != P or not visible.is_contiguous():
            raise ValueError("visible must be a contiguous bool tensor of P elements")
        g.visible_out = visible.data_ptr()
    return g


def _index32(index):
    if index is None:
        return None
    if index.dtype != torch.int32 or index.dim() != 1:
        raise RuntimeError("index must be a 1-D int32 tensor of parameter rows")
    return index.contiguous()


def _features(t, name):
    """fp32, or fp16 read as such (gs_params.sh_half); contiguous."""
    if t is None or t.numel() == 0 or t.dtype != torch.float16:
        return _f32(t, name)
    return t.contiguous()


class Prepared:
    """A raw-parameter forward between gs_rasterize_forward_begin and _end (see rasterize_gaussians_fused_begin):
    the native handle, the allocator that holds its buffers, its outputs so far and every input it reads."""

    def __init__(self, handle, alloc, radii, keep, H, W, P, dev):
        self.handle, self.alloc, self.radii, self.keep = handle, alloc, radii, keep
        self.H, self.W, self.P, self.dev = H, W, P, dev
        # a handle that is never ended gives back its read-back slot when this object goes away
        self._fin = weakref.finalize(self, N.lib().gs_rasterize_forward_release, handle)


def rasterize_gaussians_fused_begin(background, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation,
                                    scale_modifier, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height,
                                    image_width, degree, campos, prefiltered, debug, index=None, visible=None,
                                    forward_only=False, aux_mask=None):
    """First half of rasterize_gaussians_fused (gs_rasterize_forward_begin): enqueues the preprocess, the
    depth sort and the instance scan on the current stream without waiting; returns a Prepared for
    rasterize_gaussians_fused_end.  Rendering several views, begin them all first, then end each: the
    host then waits once for the first view's instance count instead of once per view with the GPU
    idle behind it."""
    N.require_gpu(xyz)
    dev = xyz.device
    if _GT is not None:
        p = _GT.fused_begin(background, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation,
                            float(scale_modifier), viewmatrix, projmatrix, float(tan_fovx), float(tan_fovy),
                            int(image_height), int(image_width), int(degree), campos, bool(prefiltered), bool(debug),
                            index, visible, bool(forward_only), aux_mask, _raw_stream(dev))
        if p.rc:
            N.check(p.rc, "rasterize_gaussians_fused")
        return p
    index = _index32(index)
    P = index.numel() if index is not None else xyz.size(0)
    H, W = int(image_height), int(image_width)
    with _on(dev):
        xyz = _f32(xyz, "xyz")
        f_dc, f_rest = _features(f_dc, "features_dc"), _features(f_rest, "features_rest")
        colors = _f32(colors, "colors")
        raw_opacity, raw_scaling = _f32(raw_opacity, "opacity"), _f32(raw_scaling, "scaling")
        raw_rotation = _f32(raw_rotation, "rotation")
        radii = torch.empty((P,), dtype=torch.int32, device=dev)
        if aux_mask is not None:
            if (aux_mask.dtype not in (torch.bool, torch.uint8) or aux_mask.device != dev or aux_mask.dim() != 1
                    or aux_mask.numel() != xyz.size(0)):
                raise ValueError("aux_mask must be a bool or uint8 tensor over the parameter rows, on the device")
            aux_mask = aux_mask.contiguous().view(torch.uint8)
        g = _params(P, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, index, visible,
                    forward_only, aux_mask)
        s, keep = _settings(background, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, H, W, degree,
                            scale_modifier, prefiltered, debug)
        keep += [xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, index, visible, aux_mask]
        alloc = _Allocator(dev)
        h = ctypes.c_void_p(None)
        rc = N.lib().gs_rasterize_forward_begin(ctypes.byref(s), ctypes.byref(g), _ptr(radii), alloc.fn, None,
                                                _stream(dev), ctypes.byref(h))
        N.check(rc, "rasterize_gaussians_fused")
        return Prepared(h.value, alloc, radii, keep, H, W, P, dev)


def rasterize_gaussians_fused_end(prep):
    """Second half (gs_rasterize_forward_end) on the current stream (the begin stream or one ordered after
    it): -> the (num_rendered, color, depth, radii, geom, binning, img) of rasterize_gaussians_fused."""
    if _GT is not None and isinstance(prep, _GT.Prepared):
        rc, nr, color, depth, radii, geom, binning, img = _GT.fused_end(prep, _raw_stream(prep.radii.device))
        if rc:
            N.check(rc, "rasterize_gaussians_fused")
        return nr, color, depth, radii, geom, binning, img
    dev = prep.dev
    with _on(dev):
        out_color = torch.empty((3, prep.H, prep.W), dtype=torch.float32, device=dev)
        out_depth = torch.empty((1, prep.H, prep.W), dtype=torch.float32, device=dev)
        _TLS.alloc = prep.alloc  # the binning buffer joins the geometry/image buffers of the begin
        nr = ctypes.c_int(0)
        prep._fin.detach()  # _end consumes the handle, also on error
        rc = N.lib().gs_rasterize_forward_end(prep.handle, _ptr(out_color), _ptr(out_depth), prep.alloc.fn, None,
                                              _stream(dev), ctypes.byref(nr))
        N.check(rc, "rasterize_gaussians_fused")
        radii = prep.radii
        if prep.P == 0:
            radii.zero_()
        geom, binning, img = prep.alloc.buffers
        return nr.value, out_color, out_depth, radii, geom, binning, img


def render_recolor(background, colors, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, image_height, image_width,
                   degree, scale_modifier, prefiltered, P, num_rendered, geomBuffer, binningBuffer, imgBuffer,
                   src_aux_mask=None):
    """gs_render_recolor: the blend of a finished forward (its geometry/binning/image buffers, num_rendered
    instances, with backward bookkeeping) again with colours `colors` [P,3] in place of its own -> (color
    [3,H,W], depth [1,H,W]), bit-identical to a full forward with colors_precomp = colors, on the current
    stream (which must be ordered after that forward).  src_aux_mask: the aux_mask that forward composited
    (unchanged since): colours equal to its 0/1 grey are then served from that forward's sums."""
    dev = colors.device
    if _GT is not None:
        rc, color, depth = _GT.render_recolor(background, colors, viewmatrix, projmatrix, campos, float(tan_fovx),
                                              float(tan_fovy), int(image_height), int(image_width), int(degree),
                                              float(scale_modifier), bool(prefiltered), int(P), int(num_rendered),
                                              geomBuffer, binningBuffer, imgBuffer, src_aux_mask, _raw_stream(dev))
        if rc:
            N.check(rc, "render_recolor")
        return color, depth
    H, W = int(image_height), int(image_width)
    with _on(dev):
        colors = _f32(colors, "colors")
        if colors.numel() < 3 * P:
            raise RuntimeError("colors must hold P x 3 values")
        s, keep = _settings(background, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, H, W, degree,
                            scale_modifier, prefiltered, False)
        out_color = torch.empty((3, H, W), dtype=torch.float32, device=dev)
        out_depth = torch.empty((1, H, W), dtype=torch.float32, device=dev)
        img_out = torch.empty(int(N.lib().gs_image_buffer_size(W, H)), dtype=torch.uint8, device=dev)
        src = None if src_aux_mask is None else src_aux_mask.contiguous().view(torch.uint8)
        if src is not None and src.numel() < P:
            raise RuntimeError("src_aux_mask must cover the P Gaussians")
        rc = N.lib().gs_render_recolor(ctypes.byref(s), int(P), int(num_rendered), _ptr(geomBuffer),
                                       _ptr(binningBuffer), _ptr(imgBuffer), _ptr(colors), _ptr(img_out),
                                       _ptr(out_color), _ptr(out_depth), _ptr(src), _stream(dev))
        N.check(rc, "render_recolor")
        del keep
        return out_color, out_depth


def rasterize_gaussians_fused(background, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation,
                              scale_modifier, viewmatrix, projmatrix, tan_fovx, tan_fovy, image_height, image_width,
                              degree, campos, prefiltered, debug, index=None, visible=None):
    """Forward on raw parameters: opacity = sigmoid, scale = exp, rotation = normalize applied in-kernel,
    SH read from _features_dc [P,1,3] and _features_rest [P,M-1,3] without concatenation (fp32 or fp16).
    index: optional int32 rows — render only those Gaussians (the `localize` subset), P = len(index).
    visible: optional bool [P] output, set to radii > 0 by the preprocess kernel."""
    return rasterize_gaussians_fused_end(rasterize_gaussians_fused_begin(
        background, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, scale_modifier, viewmatrix,
        projmatrix, tan_fovx, tan_fovy, image_height, image_width, degree, campos, prefiltered, debug, index=index,
        visible=visible))


def row_pitch_ok(t) -> bool:
    """t's rows (dim 0) may sit at any pitch, its trailing dims packed: a parameter-shaped gradient the kernels
    can write in place (a contiguous tensor, or a column block of a row-major gradient bucket)."""
    if t.dim() == 0 or t.stride(-1) != 1:
        return False
    expect = 1
    for d in range(t.dim() - 1, 0, -1):
        if t.size(d) > 1 and t.stride(d) != expect:
            return False
        expect *= t.size(d)
    return t.size(0) <= 1 or t.stride(0) >= expect


def set_grad_pitches(o, d_xyz, d_op, d_sc, d_rot, d_dc=None, d_rest=None):
    """gs_grads row pitches (ABI 17) and SH strides from the output tensors' row strides."""
    o.pitch_means3D, o.pitch_opacity = int(d_xyz.stride(0)), int(d_op.stride(0))
    o.pitch_scales, o.pitch_rotations = int(d_sc.stride(0)), int(d_rot.stride(0))
    o.dsh_dc_stride = int(d_dc.stride(0)) if d_dc is not None else 3
    o.dsh_rest_stride = int(d_rest.stride(0)) if d_rest is not None else 0


def rasterize_gaussians_fused_backward(background, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation,
                                       radii, scale_modifier, viewmatrix, projmatrix, tan_fovx, tan_fovy,
                                       dL_dout_color, degree, campos, geomBuffer, R, binningBuffer, imageBuffer,
                                       debug, into=None, index=None, writes_after=None, defer=False, stream=None):
    """-> (dL_dmeans2D [P,3], dL_dxyz, dL_dfeatures_dc, dL_dfeatures_rest, dL_dcolors, dL_dopacity_raw,
    dL_dscaling_raw, dL_drotation_raw), gradients w.r.t. the raw tensors.

    into: optional {"xyz"|"sh"|"opacity"|"scaling"|"rotation": (dest, accumulate)} — write that gradient
    into `dest` (for "sh" a (dc, rest) pair), adding to its contents when accumulate is true (the kernel's
    fused gradient accumulation, gs_grads.accumulate); the returned tuple then holds `dest`.
    index: the forward's rows; the parameter-shaped gradients are then full-size, zero outside them.
    writes_after: optional torch.cuda.Event the stream waits for before the first accumulated write
    (gs_grads.writes_after: after the replay, before the per-Gaussian pass).
    defer: enqueue only the gradient replay (gs_rasterize_backward_replay) and return (out, PendingBackward):
    the outputs are written when rasterize_backward_passes runs that pending pass (with others); `stream`
    (a torch.cuda.Stream ordered after the current one): where the replay runs (default: the current stream;
    the outputs are allocated on the current stream either way)."""
    N.require_gpu(xyz)
    dev = xyz.device
    index = _index32(index)
    Pp = xyz.size(0)  # parameter rows
    P = index.numel() if index is not None else Pp
    H, W = int(dL_dout_color.size(1)), int(dL_dout_color.size(2))
    with _on(dev):
        opts = dict(dtype=torch.float32, device=dev)
        have_sh = f_dc is not None and f_dc.numel() != 0
        into = into or {}
        acc_bits = 0

        def dest(name, make, bit):
            nonlocal acc_bits
            if name in into:
                t, acc = into[name]
                if acc:
                    acc_bits |= bit
                return t
            return make()

        # parameter-shaped outputs: only the index rows are written, so fresh ones start at zero
        new = torch.zeros if index is not None else torch.empty
        new_like = torch.zeros_like if index is not None else torch.empty_like
        d_m2 = torch.empty((P, 3), **opts)
        d_xyz = dest("xyz", lambda: new((Pp, 3), **opts), N.ACC_MEANS3D)
        if have_sh and "sh" in into:
            (d_dc, d_rest), acc = into["sh"]
            acc_bits |= N.ACC_SH if acc else 0
        else:
            d_dc = new_like(f_dc, **opts) if have_sh else None
            d_rest = new_like(f_rest, **opts) if have_sh and f_rest is not None else None
        d_col = None if have_sh else torch.empty((P, 3), **opts)  # not needed when colours come from SH
        d_op = dest("opacity", lambda: new_like(raw_opacity, **opts), N.ACC_OPACITY)
        d_sc = dest("scaling", lambda: new((Pp, 3), **opts), N.ACC_SCALES)
        d_rot = dest("rotation", lambda: new((Pp, 4), **opts), N.ACC_ROTATIONS)
        out = (d_m2, d_xyz, d_dc, d_rest, d_col, d_op, d_sc, d_rot)
        if P == 0:
            return (out, None) if defer else out
        xyz = _f32(xyz, "xyz")
        f_dc, f_rest = _features(f_dc, "features_dc"), _features(f_rest, "features_rest")
        colors = _f32(colors, "colors")
        raw_opacity, raw_scaling = _f32(raw_opacity, "opacity"), _f32(raw_scaling, "scaling")
        raw_rotation = _f32(raw_rotation, "rotation")
        g = _params(P, xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, index)
        o = N.GsGrads()
        o.dL_dmeans2D, o.dL_dcolors, o.dL_dopacity = _ptr(d_m2), _ptr(d_col), _ptr(d_op)
        o.dL_dmeans3D, o.dL_dcov3D = _ptr(d_xyz), None
        o.dL_dsh_dc = _ptr(d_dc) if have_sh else None
        o.dL_dsh_rest = _ptr(d_rest) if d_rest is not None else None
        o.dL_dscales, o.dL_drotations = _ptr(d_sc), _ptr(d_rot)
        set_grad_pitches(o, d_xyz, d_op, d_sc, d_rot, d_dc if have_sh else None, d_rest)
        o.accumulate = acc_bits
        if writes_after is not None:
            o.writes_after = writes_after.cuda_event
        gm = into.get("grad_mask")
        if gm is not None:
            mask_t, names = gm
            o.grad_mask = mask_t.data_ptr()
            o.mask_bits = sum({"xyz": N.ACC_MEANS3D, "sh": N.ACC_SH, "opacity": N.ACC_OPACITY,
                               "scaling": N.ACC_SCALES, "rotation": N.ACC_ROTATIONS}[n] for n in names)
        grad = _f32(dL_dout_color, "dL_dout_color")
        s, keep = _settings(background, viewmatrix, projmatrix, campos, tan_fovx, tan_fovy, H, W, degree,
                            scale_modifier, False, debug)
        radii = radii.contiguous()
        if defer:
            rc = N.lib().gs_rasterize_backward_replay(ctypes.byref(s), ctypes.byref(g), int(R), _ptr(radii),
                                                      _ptr(geomBuffer), _ptr(binningBuffer), _ptr(imageBuffer),
                                                      _ptr(grad), ctypes.byref(o),
                                                      _stream(dev) if stream is None else stream.cuda_stream)
            N.check(rc, "rasterize_gaussians_fused_backward (replay)")
            keep += [xyz, f_dc, f_rest, colors, raw_opacity, raw_scaling, raw_rotation, index, radii, grad,
                     geomBuffer, binningBuffer, imageBuffer, into, out]
            return out, PendingBackward(s, g, o, int(R), radii, geomBuffer, binningBuffer, keep)
        rc = N.lib().gs_rasterize_backward_ex(ctypes.byref(s), ctypes.byref(g), int(R), _ptr(radii),
                                              _ptr(geomBuffer), _ptr(binningBuffer), _ptr(imageBuffer), _ptr(grad),
                                              ctypes.byref(o), _stream(dev))
        N.check(rc, "rasterize_gaussians_fused_backward")
        del keep
        return out


class PendingBackward:
    """A view's backward whose gradient replay is enqueued (gs_rasterize_backward_replay) and whose
    per-Gaussian pass waits for rasterize_backward_passes; holds the native arguments and every tensor
    they point at."""

    def __init__(self, s, g, o, R, radii, geom, binning, keep):
        self.s, self.g, self.o, self.R, self.radii, self.geom, self.binning = s, g, o, R, radii, geom, binning
        self.keep = keep

    def set_writes_after(self, event):
        self.o.writes_after = event.cuda_event if event is not None else None


def rasterize_backward_passes(pending):
    """The per-Gaussian passes of the pending backwards (in order) on the current stream, which must be
    ordered after each one's replay: one merged pass when they render one scene into the same gradient
    outputs (gs_rasterize_backward_passes), else one pass per view; at most N.MAX_VIEWS per native call."""
    if not pending:
        return
    dev = pending[0].radii.device
    with _on(dev):
        for c0 in range(0, len(pending), N.MAX_VIEWS):
            chunk = pending[c0:c0 + N.MAX_VIEWS]
            n = len(chunk)
            sa = (ctypes.c_void_p * n)(*[ctypes.addressof(p.s) for p in chunk])
            ga = (ctypes.c_void_p * n)(*[ctypes.addressof(p.g) for p in chunk])
            oa = (ctypes.c_void_p * n)(*[ctypes.addressof(p.o) for p in chunk])
            ra = (ctypes.c_int * n)(*[p.R for p in chunk])
            rad = (ctypes.c_void_p * n)(*[_ptr(p.radii) for p in chunk])
            geo = (ctypes.c_void_p * n)(*[_ptr(p.geom) for p in chunk])
            binn = (ctypes.c_void_p * n)(*[_ptr(p.binning) for p in chunk])
            rc = N.lib().gs_rasterize_backward_passes(n, sa, ga, ra, rad, geo, binn, oa, _stream(dev))
            N.check(rc, "rasterize_backward_passes")


try:
    _load_binding()
except ImportError:  # (no libgs_raster.so yet: every native call raises when it is made; tests/test_c_abi.py)
    _GT = None
