"""Timeline analysis of a rocprofv3 kernel trace (dev tool): over the bench's last `--steps` steps
(3 views each), the union of kernel intervals vs the wall span (GPU busy fraction), the summed kernel
time, each kernel's summed duration and how much of it ran while another kernel was also running."""
import argparse
import csv
import gzip
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--steps", type=int, default=12)
    ap.add_argument("--views", type=int, default=3)
    a = ap.parse_args()
    op = gzip.open if a.csv.endswith(".gz") else open
    rows = []
    with op(a.csv, "rt") as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    # the timed region: the last steps * views launches of k_preprocess onward
    pre = [i for i, r in enumerate(rows) if "k_preprocess" in r[2]]
    first = pre[-a.steps * a.views] if len(pre) >= a.steps * a.views else 0
    sel = rows[first:]
    t0, t1 = sel[0][0], max(r[1] for r in sel)
    busy, cur_s, cur_e = 0, None, None
    for s, e, _ in sel:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    total = sum(e - s for s, e, _ in sel)
    renders = a.steps * a.views
    print(f"span {(t1 - t0) / 1e3:.1f} us over {renders} renders: {(t1 - t0) / 1e3 / renders:.1f} us/render; "
          f"busy (union) {busy / 1e3 / renders:.1f} us/render ({busy / (t1 - t0):.3f}); "
          f"summed kernel time {total / 1e3 / renders:.1f} us/render (concurrency {total / busy:.2f})")
    per = defaultdict(lambda: [0, 0])
    for s, e, n in sel:
        per[n][0] += e - s
        per[n][1] += 1
    for n, (d, c) in sorted(per.items(), key=lambda kv: -kv[1][0])[:16]:
        print(f"  {n[:60]:60s} {d / 1e3 / renders:8.1f} us/render  {c / renders:5.2f} launches/render  avg {d / 1e3 / c:7.1f} us")


if __name__ == "__main__":
    main()
