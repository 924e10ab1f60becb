"""Probe (GPU box): which float32 operation order does torch.optim.Adam's foreach
path compute on this ROCm build?  Runs one torch step on the GPU from known
(p, g, m, v) and counts bitwise mismatches against numpy emulations of candidate
orders (fma emulated in float64 and rounded once: exact product, one rounding)."""
import numpy as np
import torch

f32 = np.float32


def fma(a, b, c):
    return (a.astype(np.float64) * b.astype(np.float64) + c.astype(np.float64)).astype(f32)


def main():
    rng = np.random.default_rng(0)
    n = 1 << 20
    b1, b2, eps, lr = 0.9, 0.99, 1e-15, 0.0125
    for step in (1, 2, 5):
        p = rng.standard_normal(n).astype(f32)
        g = (rng.standard_normal(n) * 1e-2).astype(f32)
        m = (rng.standard_normal(n) * 1e-2).astype(f32)
        v = (rng.random(n) * 1e-4).astype(f32)
        P = torch.nn.Parameter(torch.from_numpy(p.copy()).cuda())
        opt = torch.optim.Adam([P], lr=lr, betas=(b1, b2), eps=eps, foreach=True)
        P.grad = torch.from_numpy(g.copy()).cuda()
        opt.step()  # initialises state (step 1), then overwrite and step again
        st = opt.state[P]
        with torch.no_grad():
            P.copy_(torch.from_numpy(p))
            st["exp_avg"].copy_(torch.from_numpy(m))
            st["exp_avg_sq"].copy_(torch.from_numpy(v))
            st["step"].fill_(step - 1)
        opt.step()
        torch.cuda.synchronize()
        tp = P.detach().cpu().numpy()
        tm = st["exp_avg"].cpu().numpy()
        tv = st["exp_avg_sq"].cpu().numpy()
        omb1, omb2 = f32(1 - b1), f32(1 - b2)
        bc1 = 1 - b1 ** step
        bc2s = (1 - b2 ** step) ** 0.5
        nstep = f32(-(lr / bc1))
        ms = {"plain": m + omb1 * (g - m), "fma": fma(np.full(n, omb1, f32), g - m, m)}
        vs = {"plain": v * f32(b2) + (omb2 * g) * g, "fma_gg": fma(np.full(n, omb2, f32), g * g, v * f32(b2)),
              "fma_sg": fma(omb2 * g, g, v * f32(b2)), "plain_gg": v * f32(b2) + omb2 * (g * g)}
        for k, mm in ms.items():
            print(f"step {step} m[{k}] mismatches {int((mm != tm).sum())}")
        for k, vv in vs.items():
            print(f"step {step} v[{k}] mismatches {int((vv != tv).sum())}")
        mm, vv = tm, tv
        sq = np.sqrt(vv)
        dens = {"div": sq / f32(bc2s) + f32(eps), "mulrcp32": sq * (f32(1) / f32(bc2s)) + f32(eps),
                "mulrcp64": sq * f32(1.0 / bc2s) + f32(eps)}
        for dk, d in dens.items():
            for pk, pp in {"plain": p + nstep * (mm / d), "fma": fma(np.full(n, nstep, f32), mm / d, p)}.items():
                print(f"step {step} p[{dk},{pk}] mismatches {int((pp != tp).sum())}")


if __name__ == "__main__":
    main()
