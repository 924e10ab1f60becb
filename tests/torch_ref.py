"""Dense, differentiable PyTorch formulation of the reference rasterizer.

Test infrastructure: an INDEPENDENT derivation used to pin the oracle
(oracle/gs_oracle.c) — the oracle's backward is hand-derived like the
reference's (backward.cu), this module's gradients come from autograd.

Semantics follow forward.cu / auxiliary.h: near cull z <= 0.2, EWA cov2D with
the 1.3*tanfov clamp and +0.3, conic, 3-sigma radius, tile rects, SH->RGB with
clamp at 0, per-tile lists ordered by (depth, index), and per pixel the
front-to-back blend with the power > 0 / alpha < 1/255 skips and the
T < 1e-4 stop.  Discrete decisions (visibility, rects, skips, stop) are taken
in float32 like the kernels; values are recomputed in `dtype` (float64 by
default) so autograd gives the exact gradient of that piecewise function.

Autograd equals the reference's hand-written backward only where the
reference's gradient IS the derivative: callers must keep every Gaussian
inside the +-1.3*tanfov clamp (backward.cu:175-176 zeroes only x/y) and keep
opacity*G below the 0.99 alpha clamp (backward.cu:538-554 ignore it).
"""
from __future__ import annotations

import math

import numpy as np
import torch

SH_C0 = 0.28209479177387814
SH_C1 = 0.4886025119029199
SH_C2 = [1.0925484305920792, -1.0925484305920792, 0.31539156525252005, -1.0925484305920792, 0.5462742152960396]
SH_C3 = [-0.5900435899266435, 2.890611442640554, -0.4570457994644658, 0.3731763325901154, -0.4570457994644658,
         1.445305721320277, -0.5900435899266435]


def sh_rgb(deg, sh, d):
    x, y, z = d[:, 0:1], d[:, 1:2], d[:, 2:3]
    r = SH_C0 * sh[:, 0]
    if deg > 0:
        r = r - SH_C1 * y * sh[:, 1] + SH_C1 * z * sh[:, 2] - SH_C1 * x * sh[:, 3]
    if deg > 1:
        xx, yy, zz, xy, yz, xz = x * x, y * y, z * z, x * y, y * z, x * z
        r = (r + SH_C2[0] * xy * sh[:, 4] + SH_C2[1] * yz * sh[:, 5] + SH_C2[2] * (2 * zz - xx - yy) * sh[:, 6]
             + SH_C2[3] * xz * sh[:, 7] + SH_C2[4] * (xx - yy) * sh[:, 8])
    if deg > 2:
        r = (r + SH_C3[0] * y * (3 * xx - yy) * sh[:, 9] + SH_C3[1] * xy * z * sh[:, 10]
             + SH_C3[2] * y * (4 * zz - xx - yy) * sh[:, 11] + SH_C3[3] * z * (2 * zz - 3 * xx - 3 * yy) * sh[:, 12]
             + SH_C3[4] * x * (4 * zz - xx - yy) * sh[:, 13] + SH_C3[5] * z * (xx - yy) * sh[:, 14]
             + SH_C3[6] * x * (xx - 3 * yy) * sh[:, 15])
    return r + 0.5


def _geometry(means3D, scales, rots, cov3D, mod, view, proj, tanfovx, tanfovy, W, H, means2D_off=None):
    """Per-Gaussian projection; returns dict of tensors in the inputs' dtype."""
    V = view.reshape(4, 4)  # row-major memory of the column-major transform
    Pm = proj.reshape(4, 4)
    pv = means3D @ V[:3, :3] + V[3, :3]
    ph = means3D @ Pm[:3, :] + Pm[3, :]
    pw = 1.0 / (ph[:, 3] + 1e-7)
    pproj = ph[:, :2] * pw[:, None]
    if means2D_off is not None:
        pproj = pproj + means2D_off[:, :2]
    if cov3D is None:
        s = mod * scales
        r, x, y, z = rots[:, 0], rots[:, 1], rots[:, 2], rots[:, 3]
        R = torch.stack([1 - 2 * (y * y + z * z), 2 * (x * y - r * z), 2 * (x * z + r * y),
                         2 * (x * y + r * z), 1 - 2 * (x * x + z * z), 2 * (y * z - r * x),
                         2 * (x * z - r * y), 2 * (y * z + r * x), 1 - 2 * (x * x + y * y)], -1).reshape(-1, 3, 3)
        L = R * s[:, None, :]
        Sig = L @ L.transpose(1, 2)
    else:
        c = cov3D
        Sig = torch.stack([c[:, 0], c[:, 1], c[:, 2], c[:, 1], c[:, 3], c[:, 4], c[:, 2], c[:, 4], c[:, 5]],
                          -1).reshape(-1, 3, 3)
    fx = W / (2.0 * tanfovx)
    fy = H / (2.0 * tanfovy)
    limx, limy = 1.3 * tanfovx, 1.3 * tanfovy
    tz = pv[:, 2]
    tx = torch.clamp(pv[:, 0] / tz, -limx, limx) * tz
    ty = torch.clamp(pv[:, 1] / tz, -limy, limy) * tz
    zero = torch.zeros_like(tz)
    J = torch.stack([fx / tz, zero, -(fx * tx) / (tz * tz), zero, fy / tz, -(fy * ty) / (tz * tz)], -1).reshape(-1, 2, 3)
    Rv = V[:3, :3].T
    T = J @ Rv
    cov2 = T @ Sig @ T.transpose(1, 2)
    a = cov2[:, 0, 0] + 0.3
    b = cov2[:, 0, 1]
    c = cov2[:, 1, 1] + 0.3
    det = a * c - b * b
    conic = torch.stack([c / det, -b / det, a / det], -1)
    xy = torch.stack([((pproj[:, 0] + 1.0) * W - 1.0) * 0.5, ((pproj[:, 1] + 1.0) * H - 1.0) * 0.5], -1)
    return {"pv": pv, "xy": xy, "conic": conic, "a": a, "b": b, "c": c, "det": det}


def _rects(xy32, radius, W, H):
    gx, gy = (W + 15) // 16, (H + 15) // 16
    x = xy32[:, 0]
    y = xy32[:, 1]
    r = radius.astype(np.float32)
    f = lambda v: np.trunc(v).astype(np.int64)
    x0 = np.clip(f((x - r) / np.float32(16)), 0, gx)
    y0 = np.clip(f((y - r) / np.float32(16)), 0, gy)
    x1 = np.clip(f((((x + r) + np.float32(16)) - np.float32(1)) / np.float32(16)), 0, gx)
    y1 = np.clip(f((((y + r) + np.float32(16)) - np.float32(1)) / np.float32(16)), 0, gy)
    return x0, y0, x1, y1


def dense_render(means3D, opacities, settings, shs=None, colors=None, scales=None, rotations=None, cov3D=None,
                 means2D=None, dtype=torch.float64):
    """Returns (color [3,H,W], depth [1,H,W], radii np[P], n_contrib np[H,W]) differentiable in `dtype`."""
    s = settings
    W, H = int(s.image_width), int(s.image_height)
    view = torch.as_tensor(np.asarray(s.viewmatrix, np.float32).reshape(16))
    proj = torch.as_tensor(np.asarray(s.projmatrix, np.float32).reshape(16))
    campos = torch.as_tensor(np.asarray(s.campos, np.float32).reshape(3))
    bg = torch.as_tensor(np.asarray(s.bg, np.float32).reshape(3))
    P = means3D.shape[0]

    def cast(t):
        return None if t is None else t.to(dtype)

    # ---- float32 pass: discrete decisions ----
    with torch.no_grad():
        g32 = _geometry(means3D.detach().float(), None if scales is None else scales.detach().float(),
                        None if rotations is None else rotations.detach().float(),
                        None if cov3D is None else cov3D.detach().float(), float(s.scale_modifier), view, proj,
                        float(s.tanfovx), float(s.tanfovy), W, H)
        a, c, det = g32["a"].numpy(), g32["c"].numpy(), g32["det"].numpy()
        mid = np.float32(0.5) * (a + c)
        sq = np.sqrt(np.maximum(np.float32(0.1), mid * mid - det))
        lam = np.maximum(mid + sq, mid - sq)
        radius = np.ceil(np.float32(3.0) * np.sqrt(lam)).astype(np.int64)
        vis = (g32["pv"][:, 2].numpy() > np.float32(0.2)) & (det != 0)
        x0, y0, x1, y1 = _rects(g32["xy"].numpy().astype(np.float32), radius, W, H)
        vis &= (x1 - x0) * (y1 - y0) != 0
        radii = np.where(vis, radius, 0).astype(np.int32)
        depth32 = g32["pv"][:, 2].numpy().astype(np.float32)

    # ---- differentiable pass ----
    g = _geometry(cast(means3D), cast(scales), cast(rotations), cast(cov3D), float(s.scale_modifier), view.to(dtype),
                  proj.to(dtype), float(s.tanfovx), float(s.tanfovy), W, H, cast(means2D))
    op = cast(opacities).reshape(-1)
    if colors is None:
        d = cast(means3D) - campos.to(dtype)
        d = d / d.norm(dim=1, keepdim=True)
        rgb = torch.clamp_min(sh_rgb(int(s.sh_degree), cast(shs), d), 0.0)
    else:
        rgb = cast(colors)
    depth = g["pv"][:, 2]

    gx, gy = (W + 15) // 16, (H + 15) // 16
    order = np.lexsort((np.arange(P), depth32.view(np.uint32)))
    out_c = torch.zeros(3, H, W, dtype=dtype)
    out_d = torch.zeros(1, H, W, dtype=dtype)
    n_contrib = np.zeros((H, W), np.int64)
    xy, conic = g["xy"], g["conic"]
    xy32n, con32n = g32["xy"].numpy(), g32["conic"].numpy()
    op32 = opacities.detach().float().reshape(-1).numpy()
    rows = []
    for ty in range(gy):
        for tx in range(gx):
            ids = [i for i in order if vis[i] and x0[i] <= tx < x1[i] and y0[i] <= ty < y1[i]]
            px = np.arange(tx * 16, min(tx * 16 + 16, W))
            py = np.arange(ty * 16, min(ty * 16 + 16, H))
            if len(px) == 0 or len(py) == 0:
                continue
            PX, PY = np.meshgrid(px, py)
            PXf, PYf = PX.reshape(-1).astype(np.float32), PY.reshape(-1).astype(np.float32)
            npx = PXf.shape[0]
            if not ids:
                for ch in range(3):
                    out_c[ch, PY.reshape(-1), PX.reshape(-1)] = bg[ch].to(dtype)
                continue
            idt = torch.as_tensor(ids)
            # float32 decisions, sequential like the kernel
            dx32 = xy32n[ids, 0][:, None] - PXf[None, :]
            dy32 = xy32n[ids, 1][:, None] - PYf[None, :]
            cx, cy, cz = con32n[ids, 0][:, None], con32n[ids, 1][:, None], con32n[ids, 2][:, None]
            pw32 = np.float32(-0.5) * (cx * dx32 * dx32 + cz * dy32 * dy32) - cy * dx32 * dy32
            al32 = np.minimum(np.float32(0.99), op32[ids][:, None] * np.exp(pw32).astype(np.float32))
            valid = (pw32 <= 0) & (al32 >= np.float32(1.0 / 255.0))
            keep = np.zeros_like(valid)
            T = np.ones(npx, np.float32)
            alive = np.ones(npx, bool)
            last = np.zeros(npx, np.int64)
            for k in range(len(ids)):
                v = valid[k] & alive
                tT = T * (np.float32(1) - al32[k])
                stop = v & (tT < np.float32(0.0001))
                alive &= ~stop
                v &= ~stop
                keep[k] = v
                T = np.where(v, tT, T)
                last = np.where(v, k + 1, last)
            n_contrib[PY.reshape(-1), PX.reshape(-1)] = last
            # values
            dx = xy[idt, 0][:, None] - torch.as_tensor(PXf, dtype=dtype)[None, :]
            dy = xy[idt, 1][:, None] - torch.as_tensor(PYf, dtype=dtype)[None, :]
            con = conic[idt]
            power = -0.5 * (con[:, 0:1] * dx * dx + con[:, 2:3] * dy * dy) - con[:, 1:2] * dx * dy
            alpha = op[idt][:, None] * torch.exp(power)
            alpha = torch.where(torch.as_tensor(keep), alpha, torch.zeros_like(alpha))
            one_m = 1.0 - alpha
            Tb = torch.cumprod(torch.cat([torch.ones(1, npx, dtype=dtype), one_m[:-1]], 0), 0)
            wgt = alpha * Tb
            Tf = Tb[-1] * one_m[-1]
            col = wgt.T @ rgb[idt]  # [npx, 3]
            dep = wgt.T @ depth[idt]
            for ch in range(3):
                out_c[ch, PY.reshape(-1), PX.reshape(-1)] = col[:, ch] + Tf * bg[ch].to(dtype)
            out_d[0, PY.reshape(-1), PX.reshape(-1)] = dep
    return out_c, out_d, radii, n_contrib
