#!/bin/bash
# round 5: DGE's unchanged loop on the fused render(): wall time + cProfile, and a rocprofv3 kernel trace of
# the same loop (GPU busy / idle per view).  usage: tools/gpu_r5_dge.sh <tag>   (run via gpurun)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python tools/probes/dge_loop_profile.py > $O/dge_profile.txt 2>&1 || { tail -20 $O/dge_profile.txt; exit 1; }
head -3 $O/dge_profile.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof -o dge -- python tools/probes/dge_loop_profile.py > $O/dge_prof.log 2>&1 || { tail -20 $O/dge_prof.log; exit 1; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python tools/trace_busy.py $T --steps 20 --views 3 > $O/busy.txt 2>&1; tail -15 $O/busy.txt
