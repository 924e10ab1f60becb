#!/bin/bash
# round 4, GPU call n: the round's evidence at the pruned build — tools/gpu_final.sh (GPU suite, side
# configs, default bench, rocprofv3 kernel stats 3-stream and 1-stream), then the PMC passes
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash tools/gpu_final.sh || exit $?
bash tools/gpu_pmc.sh || exit $?
