#!/bin/bash
# DGE loop A/B of environment settings on one box (run via gpurun): alternating rounds of
# tools/probes/dge_loop_profile.py per setting, then a kernel trace per setting with the backward's GPU span
# (first k_render_bwd start -> last k_gauss_bwd_live end, per iteration).
# usage: SETS="label|ENV=1;label2|ENV=2" tools/gpu_dge_env_ab.sh <tag>
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
IFS=';' read -ra CS <<< "$SETS"
for r in $(seq ${ROUNDS:-3}); do
  for c in "${CS[@]}"; do
    label=${c%%|*}; envs=${c#*|}
    env $envs timeout -k 10 200 python tools/probes/dge_loop_profile.py > $O/loop_$label$r.txt 2>&1 || { tail -5 $O/loop_$label$r.txt; exit 1; }
    echo "$label: $(grep 'dge loop' $O/loop_$label$r.txt)"
  done
done
for c in "${CS[@]}"; do
  label=${c%%|*}; envs=${c#*|}
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d $O/tr_$label -o t -- python tools/probes/dge_loop_profile.py > $O/tr_$label.log 2>&1 || { echo "trace $label failed"; exit 1; }
  python - $(find $O/tr_$label -name "*kernel_trace.csv" | head -1) $label <<'PY'
import csv, sys
rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in csv.DictReader(open(sys.argv[1])))
spans, start = [], None
for s, e, n in rows:
    if "k_render_bwd" in n and start is None:
        start = s
    if "k_gauss_bwd_live" in n and start is not None:
        spans.append((e - start) * 1e-3)
        start = None
spans = spans[5:]
print(sys.argv[2], "backward GPU span per iteration: mean %.1f us, min %.1f (n %d)" % (sum(spans) / len(spans), min(spans), len(spans)))
PY
done
