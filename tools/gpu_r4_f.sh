#!/bin/bash
# round 4, GPU call f: parity, then A/B of the quadrant masks v4 (64-bit band words from the preprocess)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4f
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
VAR=DGE_AMD_QMASK VALS="1 0" NOTESTS=1 ROUNDS=2 bash tools/gpu_env_ab.sh || exit 1
