"""Summarise rocprofv3 --pmc passes per kernel (dev tool).

Reads gpurun_out/pmc/p*/.../*counter_collection.csv, takes every counter's median
over a kernel's dispatches (the steady-state launches of the timed step: the bench's
setup calls — reference-ABI backwards that overwrite every output — are outliers a mean
would mix in), prints a table and writes
gpurun_out/pmc/pmc_traffic.json (committed as profiles/pmc_traffic.json): per kernel the HBM bytes per launch from the
memory-side counters, corrected as MI355X_MICROARCH.md §HBM prescribes
(FETCH_SIZE reports half the bytes of wide coalesced reads on gfx950: x2;
WRITE_SIZE is taken as reported; both are in KiB).
"""
import collections
import csv
import glob
import json
import os
import sys

STAGE = {"k_preprocess": "preprocess", "k_render_fwd": "render_fwd", "k_render_bwd": "render_bwd",
         "k_gauss_live": "gauss_bwd", "k_gauss_bwd_live": "gauss_bwd", "k_render_apply_weights": "apply_weights",
         "k_ranges": "ranges", "k_scan_emit": "emit", "k_emit_tiles": "emit"}


def main(root):
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
    from dge_amd._native import source_stamp  # (the kernel sources of the build that was measured)

    stamp = source_stamp()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(root, "p*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r.get("Kernel_Name", r.get("Kernel-Name", ""))
            short = name.split("(")[0].split("::")[-1].split("<")[0].strip()  # (template arguments dropped)
            # one row per (dispatch, counter)
            vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    keys = sorted(vals, key=lambda k: -sum(vals[k].get("SQ_WAVE_CYCLES", [0])))
    for k in keys:
        c = {n: sorted(v)[len(v) // 2] for n, v in vals[k].items()}
        line = " ".join(f"{n}={c[n]:.4g}" for n in sorted(c))
        print(f"{k}: {line}")
        if k in STAGE and "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            rd = 2.0 * c["FETCH_SIZE"] * 1024.0
            wr = c["WRITE_SIZE"] * 1024.0
            e = out.setdefault(STAGE[k], {"kernel": [], "read_bytes_per_launch": 0, "write_bytes_per_launch": 0,
                                          "bytes_per_launch": 0,
                                          "method": "rocprofv3 --pmc FETCH_SIZE (x2, gfx950 correction) + "
                                                    "WRITE_SIZE, separate passes; median over the kernel's dispatches; "
                                                    "a stage's kernels summed"})
            e["kernel"].append(k)
            e["read_bytes_per_launch"] += int(rd)
            e["write_bytes_per_launch"] += int(wr)
            e["bytes_per_launch"] += int(rd + wr)
            if "SQ_INSTS_VALU" in c:
                e["valu_insts_per_launch"] = int(e.get("valu_insts_per_launch", 0) + c["SQ_INSTS_VALU"])
            e["build"] = os.environ.get("PMC_BUILD") or stamp
    if out:
        dst = os.path.join(root, "pmc_traffic.json")  # copied into profiles/ by hand after the run
        json.dump(out, open(dst, "w"), indent=1)
        print("wrote", dst)


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
