#!/bin/bash
# A/B bench of in-tree library variants (run via gpurun): default build vs each
# dge_amd/lib/var/*.so, alternating, c2 bench line per run into gpurun_out/ab.log
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
: > gpurun_out/ab.log
for rep in 1 2; do
  for lib in dge_amd/lib/libgs_raster.so dge_amd/lib/var/*.so; do
    DGE_AMD_LIB=$PWD/$lib timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/ab_one.json 2>> gpurun_out/ab.err || { echo "bench failed for $lib"; exit 1; }
    python - "$lib" >> gpurun_out/ab.log <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_one.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:45s} {d['value']:9.1f} renders/s", " ".join(f"{k}={v*1000:.1f}" for k, v in d["stages_ms"].items()))
PY
  done
done
cat gpurun_out/ab.log
