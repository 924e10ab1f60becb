#!/bin/bash
# DGE loop A/B of the in-tree library against dge_amd/lib/var/base.so (run via gpurun): per build the loop's
# views/s (tools/probes/dge_loop_profile.py) and, from a kernel trace, the mean of each of our kernels.
# usage: tools/gpu_dge_ab.sh <tag>
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for r in 1 2; do
  for v in new base; do
    L=""; [ $v = base ] && L=$PWD/dge_amd/lib/var/base.so
    DGE_AMD_LIB=$L timeout -k 10 200 python tools/probes/dge_loop_profile.py > $O/loop_$v$r.txt 2>&1 || { tail -5 $O/loop_$v$r.txt; exit 1; }
    echo "$v: $(grep 'dge loop' $O/loop_$v$r.txt)"
  done
done
for v in new base; do
  L=""; [ $v = base ] && L=$PWD/dge_amd/lib/var/base.so
  DGE_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $O/tr_$v -o t -- python tools/probes/dge_loop_profile.py > $O/tr_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
  python - $(find $O/tr_$v -name "*kernel_trace.csv" | head -1) $v <<'PY'
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").split("::")[-1]
    if n.startswith("k_"):
        d[n].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
big = [x for x in d.get("k_render_fwd", []) if x > 40]
print(sys.argv[2], "render_fwd (training, >40us) mean %.1f n %d" % (sum(big) / max(1, len(big)), len(big)),
      " ".join("%s %.1f" % (k, sum(v) / len(v)) for k, v in sorted(d.items()) if k != "k_render_fwd"))
PY
done
