#!/bin/bash
# round 4, GPU call e: parity (the blend/binning/multiview suites), then A/B of the quadrant masks (v3: the
# preprocess's words + emission fallback for big rects, inputs prefetched) and of the XCD-aware backward lists
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4e
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
DGE_AMD_BWD_XCD=0 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_parity.py > $O/pytest_parity_noxcd.log 2>&1 || { tail -40 $O/pytest_parity_noxcd.log; exit 1; }
tail -1 $O/pytest_parity_noxcd.log
VAR=DGE_AMD_QMASK VALS="1 0" NOTESTS=1 ROUNDS=2 bash tools/gpu_env_ab.sh || exit 1
VAR=DGE_AMD_BWD_XCD VALS="1 0" NOTESTS=1 ROUNDS=2 bash tools/gpu_env_ab.sh || exit 1
