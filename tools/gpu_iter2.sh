#!/bin/bash
# One iteration on the GPU box (run via gpurun): the whole GPU suite, blend diagnostics, side configs
# (c4/c5/Adam) and an A/B bench of dge_amd/lib/var/*.so against the default build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -4 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/gpu_tests.log | head; exit $rc; }
timeout -k 10 200 python tools/diag_blend.py > gpurun_out/diag.log 2>&1 || { echo "diag failed"; exit 1; }
grep -E "==|p50|p99|p100|kept/wave|running" gpurun_out/diag.log
timeout -k 10 300 python tools/bench_configs.py > gpurun_out/configs.jsonl 2> gpurun_out/configs.err || { echo "configs failed"; tail -5 gpurun_out/configs.err; exit 1; }
cut -c1-400 gpurun_out/configs.jsonl
bash tools/gpu_ab.sh
