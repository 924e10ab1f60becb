#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 200 python tools/host_timeline.py > gpurun_out/host.log 2>&1 && SERIAL_ZERO=1 timeout -k 10 200 python tools/host_timeline.py >> gpurun_out/host.log 2>&1 && CPROFILE=1 timeout -k 10 200 python tools/host_timeline.py > gpurun_out/host_prof.log 2>&1
rc=$?; grep -v amdgpu.ids gpurun_out/host.log; exit $rc
