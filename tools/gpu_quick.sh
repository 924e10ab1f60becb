#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread ${PYTEST_EXTRA:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -30 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs > gpurun_out/bench_prof.log 2> gpurun_out/bench_prof.err || { echo "rocprof failed"; exit 1; }
head -25 gpurun_out/prof/run_kernel_stats.csv | cut -d, -f1-4
