#!/bin/bash
# round 4, GPU call j: the batched blend launch (one k_render_fwd for a step's views): the GPU suite, A/B
# against per-view launches on the views' streams, and with the shared preprocess on top
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4j
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
VAR=DGE_AMD_VIEWS_FWD VALS="batch render streams" NOTESTS=1 ROUNDS=2 bash tools/gpu_env_ab.sh || exit 1
DGE_AMD_VIEWS_FWD=streams timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_multiview.py > $O/pytest_mv_streams.log 2>&1 || { tail -40 $O/pytest_mv_streams.log; exit 1; }
tail -1 $O/pytest_mv_streams.log
