#!/bin/bash
# one-rank RCCL rehearsal, taken apart (run via gpurun): rocprofv3 kernel trace of the distributed bench
# step, then the host time per phase (tools/probes/dist_phases.py)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash tools/gpu_dist_prof.sh || exit $?
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533
timeout -k 10 200 python tools/probes/dist_phases.py > gpurun_out/distprof/phases.txt 2>&1 || { tail -5 gpurun_out/distprof/phases.txt; exit 1; }
cat gpurun_out/distprof/phases.txt | tail -12
