#!/bin/bash
# round 4, GPU call l: tile-first binning (emission in Gaussian order, tile sort, per-tile depth sort) —
# the GPU suite under it, the depth-first binning's parity tests, the c2 A/B, c4 under both
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
VAR=DGE_AMD_BINNING VALS="depth" TESTS="tests/test_gpu_parity.py tests/test_gpu_multiview.py" ROUNDS=0 bash tools/gpu_env_ab.sh || exit 1
VAR=DGE_AMD_BINNING VALS="tile depth" NOTESTS=1 ROUNDS=3 bash tools/gpu_env_ab.sh || exit 1
for b in tile depth; do
  DGE_AMD_BINNING=$b timeout -k 10 300 python tools/bench_configs.py c4 > $O/c4_$b.json 2> $O/c4_$b.err || { tail -5 $O/c4_$b.err; exit 1; }
  echo "c4 $b: $(tail -1 $O/c4_$b.json | cut -c1-400)"
done
