#!/bin/bash
# Alternating A/B benches of configurations on one box (run via gpurun):
#   CFGS="label1|ENV=1 ENV2=x;label2|DGE_AMD_LIB=dge_amd/lib/var/head.so" ROUNDS=2 bash tools/gpu_ab_cfg.sh <outdir>
# each configuration's env assignments are applied to one `python bench.py` run per round
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=${1:-gpurun_out/abc}
mkdir -p $O
IFS=';' read -ra CS <<< "$CFGS"
for r in $(seq ${ROUNDS:-2}); do
  for c in "${CS[@]}"; do
    label=${c%%|*}; envs=${c#*|}
    env $envs timeout -k 10 240 python bench.py --steps ${STEPS:-40} --warmup 5 --no-side-legs --no-cpu-baseline \
        > $O/bench_$label$r.json 2> $O/bench_$label$r.err || { echo "bench $label failed $?"; tail -5 $O/bench_$label$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/bench_$label$r.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$label', d['value'], 'p50', d['step_ms']['p50'], 'iso', d['roofline_leg']['renders_per_s'], ' '.join(f'{k} {v*1e3:.1f}' for k, v in s.items()))"
  done
done
