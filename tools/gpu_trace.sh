#!/bin/bash
# rocprofv3 kernel trace of the default bench (no side legs / cpu baseline), for the timeline analysis
# of tools/trace_busy.py (GPU busy fraction, per-kernel overlap).  BENCH_ARGS: extra bench flags.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/trace
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace -o run -- python bench.py --steps 12 --warmup 3 --no-cpu-baseline --no-side-legs --no-profile ${BENCH_ARGS:-} > gpurun_out/trace_bench.log 2> gpurun_out/trace_bench.err || { echo "rocprof failed $?"; tail -20 gpurun_out/trace_bench.err; exit 1; }
cat gpurun_out/trace_bench.log
f=$(find gpurun_out/trace -name "*kernel_trace.csv" | head -1)
python tools/trace_busy.py "$f" --steps 12 --views 3 | tee gpurun_out/trace_busy.txt
gzip -f "$f"
