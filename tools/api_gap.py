"""Host issue vs device start of each step's phases (dev tool; rocprofv3 --kernel-trace --hip-runtime-trace).

For the last `--steps` steps: when the host called the launch of the step's first preprocess and first
k_render_bwd (HIP API start, matched to the dispatch by correlation id), when the device started them,
and when the kernel before each ended.  A launch issued after the previous kernel ended is a host-bound
gap; one issued before is a dependency-latency gap.  Usage:
  python tools/api_gap.py <dir with *_kernel_trace.csv and *_hip_api_trace.csv>
"""
import argparse
import csv
import glob
import os


def load(pattern):
    f = glob.glob(pattern, recursive=True)
    if not f:
        raise SystemExit(f"no file matches {pattern}")
    with open(f[0]) as fh:
        return list(csv.DictReader(fh))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--views", type=int, default=3)
    a = ap.parse_args()
    ks = load(os.path.join(a.dir, "**", "*kernel_trace.csv"))
    api = load(os.path.join(a.dir, "**", "*hip_api_trace.csv"))
    by_corr = {r["Correlation_Id"]: r for r in api}
    rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0],
                   r["Correlation_Id"]) for r in ks)
    pre = [i for i, r in enumerate(rows) if "k_preprocess" in r[2]]
    starts = pre[::a.views][-(a.steps + 1):]
    # HIP calls that can block the host, in time order
    blocking = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Function"]) for r in api
                      if any(x in r["Function"] for x in ("Synchronize", "Memcpy", "Query")))
    for k in range(len(starts) - 1):
        seg = rows[starts[k]:starts[k + 1]]
        t0 = seg[0][0]
        out = []
        for name in ("k_preprocess", "k_render_bwd"):
            i = next(j for j, r in enumerate(seg) if name in r[2])
            s, e, n, c = seg[i]
            prev_end = max((r[1] for r in rows[:starts[k] + i] if r[1] <= s), default=0)
            call = by_corr.get(c)
            issued = int(call["Start_Timestamp"]) if call else None
            out.append(f"{name}: start +{(s - t0) / 1e3:7.1f} prev-end gap {(s - prev_end) / 1e3:6.1f} "
                       f"issued {((issued - prev_end) / 1e3) if issued else float('nan'):+7.1f} us vs prev end")
        waits = [(b, e, f) for b, e, f in blocking if t0 <= b < rows[starts[k + 1]][0] and e - b > 20_000]
        w = "; ".join(f"{f} {(e - b) / 1e3:.0f}us@+{(b - t0) / 1e3:.0f}" for b, e, f in waits)
        print(f"step {k}: " + " | ".join(out) + (f" | host waits: {w}" if w else ""))


if __name__ == "__main__":
    main()
