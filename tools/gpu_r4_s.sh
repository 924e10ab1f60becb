#!/bin/bash
# round 4, GPU call s: the fused-accumulation mismatch under the speculated render, taken apart
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/r4s
timeout -k 10 200 python tools/probes/fused_accum_debug.py > gpurun_out/r4s/debug.txt 2>&1; rc=$?
cat gpurun_out/r4s/debug.txt | grep -v amdgpu.ids; exit $rc
