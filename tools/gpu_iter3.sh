#!/bin/bash
# GPU suite + A/B bench of dge_amd/lib/var/*.so against the default build (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/gpu_tests.log | head; exit $rc; }
bash tools/gpu_ab.sh
