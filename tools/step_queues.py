"""One bench step of a rocprofv3 kernel trace, kernel by kernel with its HW queue and stream (dev tool).

Steps are cut at every `--views`-th k_preprocess; prints each step's length, then the kernels of step `--step`
(start / end / duration in us from the step's first preprocess, queue, stream, correlation id, grid) — the
gaps between kernels on one queue are the stream operations' queue time (tools/probes/queue_gap.hip).
Usage: python tools/step_queues.py run_kernel_trace.csv --step 14
"""
import argparse
import csv
import re


def base_name(k):
    k = k.split("(")[0]
    m = re.search(r"(k_\w+|__amd_\w+|\w+_kernel\w*)", k)
    return (m.group(1) if m else k)[:28]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--step", type=int, default=None)
    ap.add_argument("--views", type=int, default=3)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), base_name(r["Kernel_Name"]),
                         r["Queue_Id"], r["Stream_Id"], int(r["Grid_Size_X"]), int(r["Correlation_Id"])))
    rows.sort()
    pre = [i for i, r in enumerate(rows) if r[2] == "k_preprocess"]
    starts = pre[::a.views]
    print("step lengths (us):", " ".join(f"{k}:{(rows[starts[k + 1]][0] - rows[starts[k]][0]) / 1e3:.0f}"
                                         for k in range(len(starts) - 1)))
    if a.step is None:
        return
    i0, i1 = starts[a.step], starts[a.step + 1]
    t0 = rows[i0][0]
    for s, e, n, q, st, g, c in rows[max(0, i0 - 4):i1 + 3]:
        print(f"{(s - t0) / 1e3:8.1f} {(e - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f} q{q} s{st} c{c:<7} {n} grid={g}")


if __name__ == "__main__":
    main()
