"""Per-step phase breakdown of a rocprofv3 kernel trace of the bench (dev tool).

For each of the last `--steps` steps of `--views` views: the forward phase (first k_preprocess start to
the last k_render_fwd end), the gap to the backward, the backward phase (first k_render_bwd start to the
last per-Gaussian pass end), the rest (bucket zero, next step's start), and the chip's busy fraction
(union of kernel intervals) inside each phase.  Usage: python tools/step_phases.py trace.csv[.gz]
"""
import argparse
import csv
import gzip


def union_len(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if ce is None or s > ce:
            if ce is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    if ce is not None:
        tot += ce - cs
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--views", type=int, default=3)
    a = ap.parse_args()
    op = gzip.open if a.csv.endswith(".gz") else open
    rows = []
    with op(a.csv, "rt") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    pre = [i for i, r in enumerate(rows) if "k_preprocess" in r[2]]
    starts = pre[::a.views]
    starts = starts[-(a.steps + 1):]
    tot = {"fwd": 0, "gap": 0, "bwd": 0, "rest": 0}
    for k in range(len(starts) - 1):
        seg = rows[starts[k]:starts[k + 1]]
        t0 = seg[0][0]
        t_next = rows[starts[k + 1]][0]
        fwd_end = max(e for s, e, n in seg if "k_render_fwd" in n)
        bwd = [(s, e) for s, e, n in seg if "k_render_bwd" in n or "k_gauss" in n]
        b0 = min(s for s, e in bwd)
        b1 = max(e for s, e in bwd)
        ph = {"fwd": (t0, fwd_end), "gap": (fwd_end, b0), "bwd": (b0, b1), "rest": (b1, t_next)}
        out = []
        for name, (x0, x1) in ph.items():
            iv = [(max(s, x0), min(e, x1)) for s, e, _ in seg + rows[starts[k + 1]:starts[k + 1] + 1]
                  if e > x0 and s < x1]
            busy = union_len(iv) / max(1, x1 - x0)
            out.append(f"{name} {(x1 - x0) / 1e3:7.1f} us (busy {busy:.2f})")
            tot[name] += x1 - x0
        names = sorted({n for s, e, n in seg if s >= b1})
        print(f"step {k}: total {(t_next - t0) / 1e3:7.1f} us | " + " | ".join(out) + f" | rest kernels {names}")
    n = max(1, len(starts) - 1)
    print("mean: " + ", ".join(f"{k} {v / n / 1e3:.1f} us" for k, v in tot.items()))
    # per-kernel durations inside the last step
    seg = rows[starts[-2]:starts[-1]]
    agg = {}
    for s, e, nme in seg:
        agg.setdefault(nme, []).append((e - s) / 1e3)
    for nme, d in sorted(agg.items(), key=lambda x: -sum(x[1])):
        print(f"  {sum(d):8.1f} us  x{len(d):3d}  {nme}")


if __name__ == "__main__":
    main()
