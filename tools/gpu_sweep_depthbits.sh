#!/bin/bash
# depth-sort digit layout sweep (bench only; env overrides read by libgs_raster)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
run() {
  env $1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_sw.log 2>/dev/null || exit 1
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_sw.log').read().strip().splitlines()[-1]); print('$1', d['value'], d['stages_ms']['depth_sort'], d['stages_ms']['preprocess'])"
}
run "DGE_AMD_DEPTH_SORT_BITS=27 DGE_AMD_DEPTH_PASS_BITS=9"
run "DGE_AMD_DEPTH_SORT_BITS=27 DGE_AMD_DEPTH_PASS_BITS=-8"
run "DGE_AMD_DEPTH_SORT_BITS=26 DGE_AMD_DEPTH_PASS_BITS=-8"
run "DGE_AMD_DEPTH_SORT_BITS=24 DGE_AMD_DEPTH_PASS_BITS=8"
run "DGE_AMD_DEPTH_SORT_BITS=32 DGE_AMD_DEPTH_PASS_BITS=8"
