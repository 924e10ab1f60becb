"""Cache-line model of the per-Gaussian backward pass's memory traffic at c2 (dev tool, GPU).

Renders the bench's three c2 views through the reference ABI (forward + backward), reads back the
live sets, slot ranges and gradient-record flags, and counts for k_gauss_live + k_gauss_bwd_live
(gs_backward.hip), per phase, the bytes the pass needs (algorithmic) and the distinct 128-B lines
(reads) / 64-B segments (writes) those bytes fall in — what an L2 that keeps every line for the whole
launch would move.  The layout is the bench's: parameter gradients in one flat bucket of six
row-major tensors (GradBucket), accumulated by every view (the bucket is zeroed beforehand).
Prints one JSON line per phase and the totals, to set beside rocprofv3's FETCH_SIZE x 2 / WRITE_SIZE.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dge_amd import _C, _native  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import _settings  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402

RL, WL = 128, 64  # read line, write segment (bytes)


def lines(byte_offsets, nbytes, gran):
    """distinct gran-byte lines covered by [off, off + nbytes) for every offset (int64 tensor)"""
    first = byte_offsets // gran
    last = (byte_offsets + nbytes - 1) // gran
    span = int((last - first).max().item()) + 1 if byte_offsets.numel() else 1
    ids = torch.cat([torch.minimum(first + k, last) for k in range(span)])
    return int(torch.unique(ids).numel())


def main():
    dev = torch.device("cuda", 0)
    P, W, H, V = 1_000_000, 512, 512, 3
    sc = synthetic_scene(P, sh_degree=3, seed=0, device=dev)
    cams = [orbit_camera(k, V, W, H, device=dev) for k in range(V)]
    gen = torch.Generator(device="cpu").manual_seed(1)
    seeds = [(torch.randn(3, H, W, generator=gen) * 1e-3).to(dev) for _ in range(V)]
    bg = torch.zeros(3, device=dev)
    lib = _native.lib()
    views = []
    with torch.no_grad():
        for cam, g in zip(cams, seeds):
            s = _settings(cam, bg, 1.0, sc.active_sh_degree)
            K, color, depth, radii, geom, binning, img = _C.rasterize_gaussians(
                s.bg, sc.get_xyz, torch.empty(0, device=dev), sc.get_opacity, sc.get_scaling, sc.get_rotation, 1.0,
                torch.empty(0, device=dev), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, H, W, sc.get_features,
                sc.active_sh_degree, s.campos, False, False)
            _C.rasterize_gaussians_backward(
                s.bg, sc.get_xyz, radii, torch.empty(0, device=dev), sc.get_scaling, sc.get_rotation, 1.0,
                torch.empty(0, device=dev), s.viewmatrix, s.projmatrix, s.tanfovx, s.tanfovy, g, sc.get_features,
                sc.active_sh_degree, s.campos, geom, K, binning, img, False)
            off = lambda buf, f: lib.gs_buffer_offset(buf, f, P, W, H, K)  # noqa: E731
            touched = geom[off(b"geometry", b"touched"):][:P]
            tt = geom[off(b"geometry", b"tiles_touched"):][:4 * P].view(torch.int32)
            fs = geom[off(b"geometry", b"first_slot"):][:4 * P].view(torch.int32)
            flags = binning[off(b"binning", b"rec_flags"):][:4 * K].view(torch.uint8).view(-1, 4)
            live = (touched != 0) & (radii > 0)
            views.append({"K": int(K), "live": live, "tt": tt.long(), "fs": fs.long(), "flags": flags})
    torch.cuda.synchronize()
    union = torch.zeros(P, dtype=torch.bool, device=dev)
    for v in views:
        union |= v["live"]
    U = torch.nonzero(union).flatten().long()
    out = []

    def phase(name, alg_r, lines_r, alg_w=0, segs_w=0):
        out.append({"phase": name, "alg_read_MB": round(alg_r / 1e6, 2), "line_read_MB": round(lines_r * RL / 1e6, 2),
                    "alg_write_MB": round(alg_w / 1e6, 2), "seg_write_MB": round(segs_w * WL / 1e6, 2)})

    # k_gauss_live: per view touched (1 B) + radii (4 B) streamed over P; the live list (4 B per union
    # Gaussian, in its block's region) and per-block counts written; per view the Gaussian-indexed
    # 3-float outputs of its dead Gaussians zeroed (dL_dconic always; means2D/colors: accumulated in
    # the bench) -- streamed (dead = most of P)
    phase("live: flags read", V * 5 * P, V * 5 * P // RL)
    phase("live: list + conic zeros", 0, 0, 4 * U.numel() + V * 12 * P, (4 * U.numel()) // WL + V * 12 * P // WL)
    # k_gauss_bwd_live, per live (Gaussian, view)
    tot = {"params": [0, 0], "geom": [0, 0], "flags": [0, 0], "records": [0, 0], "sh_rest": [0, 0]}
    wr = {"means2D": [0, 0, 0], "param_grads": [0, 0, 0], "sh_rest_grad": [0, 0, 0]}
    param_rows = [("means3D", 12), ("scales", 12), ("rotations", 16), ("opacity", 4)]
    for v in views:
        L = torch.nonzero(v["live"]).flatten().long()
        n = L.numel()
        # parameters (one row per Gaussian in each of the four tensors; SH dc 12 B)
        for _, b in param_rows + [("sh_dc", 12)]:
            tot["params"][0] += b * n
            tot["params"][1] += lines(L * b, b, RL)
        # per-view geometry: clamped (1 B), tiles_touched (4), first_slot (4)
        for b in (1, 4, 4):
            tot["geom"][0] += b * n
            tot["geom"][1] += lines(L * b, b, RL)
        first, cnt = v["fs"][L], v["tt"][L]
        slots = torch.repeat_interleave(first, cnt) + (torch.arange(int(cnt.sum().item()), device=dev)
                                                         - torch.repeat_interleave(torch.cumsum(cnt, 0) - cnt, cnt))
        tot["flags"][0] += 4 * slots.numel()
        tot["flags"][1] += lines(slots * 4, 4, RL)
        fl = v["flags"][slots]  # [n_slots, 4]
        rec = (4 * slots[:, None] + torch.arange(4, device=dev)[None, :])[fl != 0]
        tot["records"][0] += 48 * rec.numel()
        tot["records"][1] += lines(rec * 48, 48, RL)
        tot["sh_rest"][0] += 180 * n
        tot["sh_rest"][1] += lines(L * 180, 180, RL)
        # writes (and the accumulated outputs' reads)
        for key, b, stride in [("means2D", 8, 12)] + [("param_grads", b, b) for _, b in param_rows + [("sh_dc", 12)]] \
                + [("sh_rest_grad", 180, 180)]:
            wr[key][0] += b * n
            wr[key][1] += lines(L * stride, b, RL)
            wr[key][2] += lines(L * stride, b, WL)
        out.append({"view": len(out), "live": n, "slots": int(slots.numel()), "records": int(rec.numel())})
    for k, (a, l) in tot.items():
        phase(f"bwd read: {k}", a, l)
    for k, (a, r, w) in wr.items():  # read-modify-write: the old value read (lines), the sum written (segments)
        phase(f"bwd rmw: {k}", a, r, a, w)
    for o in out:
        print(json.dumps(o))
    ph = [o for o in out if "phase" in o]
    print(json.dumps({"union_live": int(U.numel()),
                      "total_alg_read_MB": round(sum(o["alg_read_MB"] for o in ph), 1),
                      "total_line_read_MB": round(sum(o["line_read_MB"] for o in ph), 1),
                      "total_alg_write_MB": round(sum(o["alg_write_MB"] for o in ph), 1),
                      "total_seg_write_MB": round(sum(o["seg_write_MB"] for o in ph), 1)}))


if __name__ == "__main__":
    main()
