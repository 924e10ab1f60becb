#!/bin/bash
# c4 A/B of library builds on one box (run via gpurun): alternating rounds of tools/bench_configs.py c4 per build.
# usage: LIBS="new ept16 ..." tools/gpu_c4_ab.sh <tag>   ("new": the in-tree library, else dge_amd/lib/var/NAME.so)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/$1
mkdir -p $O
for r in $(seq ${ROUNDS:-2}); do
  for v in $LIBS; do
    L=""; [ $v != new ] && L=$PWD/dge_amd/lib/var/$v.so
    DGE_AMD_LIB=$L timeout -k 10 200 python tools/bench_configs.py c4 --steps ${STEPS:-30} > $O/c4_$v$r.json 2> $O/c4_$v$r.err || { echo "c4 $v failed"; tail -5 $O/c4_$v$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/c4_$v$r.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$v', d['value'], ' '.join(f'{k} {v*1e3:.1f}' for k, v in s.items()))"
  done
done
