#!/bin/bash
# round 4, GPU call w: u16 row-pass keys in the two-level binning — the GPU suite, then c4 three times
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4w
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for r in 1 2 3; do
  timeout -k 10 300 python tools/bench_configs.py c4 > $O/c4_$r.json 2> $O/c4_$r.err || { tail -5 $O/c4_$r.err; exit 1; }
  tail -1 $O/c4_$r.json | cut -c1-330
done
