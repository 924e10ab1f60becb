#!/bin/bash
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/r4t
PROBE3=1 timeout -k 10 200 python tools/probes/fused_accum_debug.py > gpurun_out/r4t/debug.txt 2>&1; rc=$?
grep -v amdgpu.ids gpurun_out/r4t/debug.txt; exit $rc
