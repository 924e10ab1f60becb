"""GPU idle gaps inside one iteration of a loop, from a rocprofv3 kernel trace (dev tool).

The iteration is the stretch between the last two dispatches of the marker kernel (default k_gauss_bwd_live,
the end of a backward).  Prints every kernel of it (start offset, duration) and each idle gap over
--min-gap us with the kernels around it, then the summed busy and idle time.
Usage: python tools/gap_trace.py trace.csv [--marker NAME] [--min-gap US]
"""
import argparse
import csv


def short(name):
    return name.split("(")[0].split("<")[0].replace("void ", "").split("::")[-1][:48]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="k_gauss_bwd_live")
    ap.add_argument("--min-gap", type=float, default=5.0)
    a = ap.parse_args()
    rows = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]))
            for r in csv.DictReader(open(a.csv))]
    rows.sort()
    marks = [i for i, r in enumerate(rows) if r[2] == a.marker]
    if len(marks) < 2:
        raise SystemExit(f"fewer than two {a.marker} dispatches")
    it = rows[marks[-2] + 1: marks[-1] + 1]
    t0 = rows[marks[-2]][1]
    busy_end, idle, busy = t0, 0.0, 0.0
    for s, e, n in it:
        gap = (s - busy_end) * 1e-3
        if gap > a.min_gap:
            print(f"   -- idle {gap:7.1f} us")
        if gap > 0:
            idle += gap
        busy += max(0, e - max(s, busy_end)) * 1e-3
        print(f"{(s - t0) * 1e-3:9.1f} {(e - s) * 1e-3:7.1f}  {n}")
        busy_end = max(busy_end, e)
    print(f"iteration {(busy_end - t0) * 1e-3:.1f} us: busy {busy:.1f}, idle {idle:.1f}")


if __name__ == "__main__":
    main()
