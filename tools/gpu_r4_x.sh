#!/bin/bash
# round 4, GPU call x: emission batch size (instances per thread) at c4 — in-tree (8) vs 16 vs 4, alternating
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4x
mkdir -p $O
for r in 1 2; do
  for v in new ept16 ept4; do
    lib=""; [ $v != new ] && lib=$PWD/dge_amd/lib/var/$v.so
    DGE_AMD_LIB=$lib timeout -k 10 300 python tools/bench_configs.py c4 > $O/c4_$v$r.json 2> $O/c4_$v$r.err || { tail -5 $O/c4_$v$r.err; exit 1; }
    echo "$v: $(tail -1 $O/c4_$v$r.json | cut -c60-330)"
  done
done
