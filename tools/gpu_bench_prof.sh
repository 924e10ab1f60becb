#!/bin/bash
# bench + rocprofv3 kernel-trace stats on the GPU box (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed $?"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.log
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_prof.log 2> gpurun_out/bench_prof.err || { echo "rocprof failed $?"; tail -20 gpurun_out/bench_prof.err; exit 1; }
find gpurun_out/prof -name "*stats*" | head
