#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
DIST=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29517 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 timeout -k 10 200 python tools/host_timeline.py > gpurun_out/host.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/host.log; exit $rc
