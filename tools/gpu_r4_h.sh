#!/bin/bash
# round 4, GPU call h: the GPU suite (quadrant masks removed, recolor), A/B of the views' issue order
# (every preprocess first vs view by view), a kernel trace of one steady step
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
VAR=DGE_AMD_VIEWS_ISSUE VALS="breadth view" NOTESTS=1 ROUNDS=3 bash tools/gpu_env_ab.sh || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --steps 12 --warmup 5 --no-cpu-baseline --no-side-legs --no-profile > $O/trace.log 2> $O/trace.err || { echo "rocprof failed $?"; tail -20 $O/trace.err; exit 1; }
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python tools/step_phases.py "$f" --steps 8 > $O/phases.txt; tail -3 $O/phases.txt
python tools/probes/step_timeline.py "$f" > $O/step.txt; tail -70 $O/step.txt | cut -c1-110
gzip -f "$f"
