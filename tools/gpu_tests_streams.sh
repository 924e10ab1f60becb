#!/bin/bash
# GPU suite, then the stream sweep and the default bench line (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
STEPS=40 ./tools/gpu_streams.sh && ./tools/gpu_bench.sh
