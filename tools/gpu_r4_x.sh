#!/bin/bash
# round 4, GPU calls x, y: c4 A/B of library variants (VARS, default row32) against the in-tree build, alternating
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/${OUT:-r4x}
mkdir -p $O
for r in 1 2; do
  for v in new ${VARS:-row32}; do
    lib=""; [ $v != new ] && lib=$PWD/dge_amd/lib/var/$v.so
    DGE_AMD_LIB=$lib timeout -k 10 300 python tools/bench_configs.py c4 > $O/c4_$v$r.json 2> $O/c4_$v$r.err || { tail -5 $O/c4_$v$r.err; exit 1; }
    echo "$v: $(tail -1 $O/c4_$v$r.json | cut -c60-330)"
  done
done
