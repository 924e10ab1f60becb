#!/bin/bash
# round 4, GPU call aa: the per-Gaussian pass's live-set half behind view 0's replay — the GPU suite, then the
# c2 bench against the previous build (dge_amd/lib/var/prevtail.so), 3 alternating rounds
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4aa
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
NOTESTS=1 VARS=prevtail ROUNDS=3 bash tools/gpu_ab.sh || exit 1
