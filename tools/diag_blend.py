"""Blend-kernel timeline diagnostics (dev tool, GPU).

Renders the c2 workload once (forward + backward) with the library's per-wave
timestamps on and prints, for each blend kernel: the kernel span, the
distribution of per-wave/per-tile durations, the correlation with kept entries
and rounds, and how many waves are still running over time (tail shape).
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dge_amd import _native  # noqa: E402
from dge_amd.cameras import orbit_camera  # noqa: E402
from dge_amd.gaussian_renderer import PipelineParams, render  # noqa: E402
from dge_amd.scene import synthetic_scene  # noqa: E402




def summarize(name, d, nquads=None):
    """d: per-wave records; for the backward, rows are work-queue positions and word 6 holds
    (segment << 32 | quadrant index)."""
    if d.size == 0:
        print(name, "no data")
        return
    d = d.astype(np.int64)
    ids = np.arange(len(d))
    live = d[:, 1] > 0  # blocks that had work (segments past a window's end exit without a record)
    d, ids = d[live], ids[live]
    start, end, kept, rounds, cyc_loop, cyc_total = (d[:, i] for i in range(6))
    t0 = start.min()
    dur = (end - start) * 10e-3  # us (100 MHz)
    span = (end.max() - t0) * 10e-3
    clk = cyc_total.sum() / max(1, (end - start).sum()) / 10e-3 / 1e3  # GHz
    print(f"== {name}: {len(d)} waves, span {span:.1f} us, start spread {(start.max() - t0) * 10e-3:.1f} us, "
          f"shader clock ~{clk:.2f} GHz")
    for q in (50, 90, 99, 100):
        print(f"   wave dur p{q}: {np.percentile(dur, q):.2f} us")
    print(f"   kept/wave mean {kept.mean():.1f} max {kept.max()}  rounds mean {rounds.mean():.2f} max {rounds.max()}")
    print(f"   loop share of cycles {cyc_loop.sum() / max(1, cyc_total.sum()):.3f}; "
          f"loop cycles per kept entry (all) {cyc_loop.sum() / max(1, kept.sum()):.0f}")
    order = np.argsort(-dur)[:6]
    for i in order:
        extra = f" seg {int(d[i, 6]) >> 32} quad {int(d[i, 6]) & 0xFFFFFFFF}" if nquads else \
            f" cull+wait share {d[i, 6] / max(1, cyc_total[i]):.2f}"
        print(f"   slowest: wave {ids[i]} dur {dur[i]:.1f} us kept {kept[i]} rounds {rounds[i]} loop cyc/kept "
              f"{cyc_loop[i] / max(1, kept[i]):.0f} loop share {cyc_loop[i] / max(1, cyc_total[i]):.2f} "
              f"start {(start[i] - t0) * 10e-3:.1f}{extra}")
    # SIMD sharing: waves of one SIMD (word 7: HW_ID | XCC_ID << 32) compete for its issue slots
    loc = d[:, 7]
    simd = (loc >> 32) * 4096 + ((loc >> 8) & 0xF) * 256 + ((loc >> 12) & 0x1) * 128 + ((loc >> 13) & 0x7) * 16 \
        + ((loc >> 4) & 0x3)
    if loc.any():
        u, inv = np.unique(simd, return_inverse=True)
        busy = np.bincount(inv, weights=dur)
        print(f"   SIMDs used {len(u)}; summed wave-us per SIMD p50 {np.percentile(busy, 50):.0f} "
              f"p99 {np.percentile(busy, 99):.0f} max {busy.max():.0f}")
        for i in order[:3]:
            mates = np.nonzero((inv == inv[i]) & (np.arange(len(d)) != i))[0]
            ov = [min(end[i], end[j]) - max(start[i], start[j]) for j in mates]
            print(f"   slowest wave {ids[i]}: {len(mates)} SIMD mates, overlap-us {[round(o * 10e-3, 1) for o in ov]}, "
                  f"their durations {[round(float(dur[j]), 1) for j in mates]}")
    if loc.any():  # per XCD: its last wave's end, summed wave time and waves (balance across the 8 L2s)
        xcc = loc >> 32
        print("   per XCD end/us, wave-us, waves:", " ".join(
            f"{int(x)}:{(end[xcc == x].max() - t0) * 10e-3:.0f}/{dur[xcc == x].sum():.0f}/{int((xcc == x).sum())}"
            for x in np.unique(xcc)))
    ts = np.linspace(0, span, 11)
    alive = [int(((start - t0) * 10e-3 <= t).sum() - ((end - t0) * 10e-3 <= t).sum()) for t in ts]
    print("   waves running over time:", " ".join(f"{t:.0f}:{a}" for t, a in zip(ts, alive)))


def main():
    dev = torch.device("cuda", 0)
    P = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    W = H = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    scene = synthetic_scene(P, sh_degree=3, seed=0, device=dev).requires_grad_(True)
    V = int(sys.argv[3]) if len(sys.argv) > 3 else 1  # V > 1: the bench's batch (render_views, one merged pass)
    cams = [orbit_camera(k, 3, W, H, device=dev) for k in range(V)]
    gs = [(torch.randn(3, H, W, generator=torch.Generator().manual_seed(1 + k)) * 1e-3).to(dev) for k in range(V)]
    bg = torch.zeros(3, device=dev)

    def once():
        if V == 1:
            render(cams[0], scene, PipelineParams(), bg)["render"].backward(gs[0])
        else:
            from dge_amd.multiview import render_views
            outs = render_views(cams, scene, PipelineParams(), bg, streams=V)
            torch.autograd.backward([o["render"] for o in outs], gs)

    for _ in range(3):
        once()
    torch.cuda.synchronize()
    _native.diag_enable(True)
    once()
    torch.cuda.synchronize()
    _native.diag_enable(False)
    summarize("render_fwd", _native.diag_read(0))
    summarize("render_bwd", _native.diag_read(1), nquads=4 * ((W + 15) // 16) * ((H + 15) // 16))
    g = _native.diag_read(2).astype(np.int64)
    g = g[g[:, 0] > 0]
    if len(g):
        t0 = g[:, 0].min()
        names = ["params+ids", "records", "SH staged", "chain", "commit", "SH store+end"]
        cols = [1, 2, 3, 4, 5, 7]
        prev = g[:, 0]
        print(f"== gauss_bwd_live: {len(g)} waves, span {(g[:, 7].max() - t0) * 1e-2:.1f} us, "
              f"start spread {(g[:, 0].max() - t0) * 1e-2:.1f} us, live/workgroup mean {g[:, 6].mean():.0f}")
        for n, c in zip(names, cols):
            d = (g[:, c] - prev) * 1e-2
            print(f"   {n:>13}: mean {d.mean():6.2f} us  p90 {np.percentile(d, 90):6.2f}  max {d.max():6.2f}")
            prev = g[:, c]


if __name__ == "__main__":
    main()
