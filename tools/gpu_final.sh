#!/bin/bash
# round-end evidence (run via gpurun): GPU suite, side configs, default bench, rocprofv3 kernel stats of the
# default bench and of the one-stream bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/final/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/final/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/final/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python tools/bench_configs.py > gpurun_out/final/configs.jsonl 2> gpurun_out/final/configs.err || { echo "configs failed"; tail -5 gpurun_out/final/configs.err; exit 1; }
cut -c1-300 gpurun_out/final/configs.jsonl
timeout -k 10 500 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || { echo "bench failed"; tail -5 gpurun_out/final/bench.err; exit 1; }
cut -c1-200 gpurun_out/final/bench.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/final/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs > gpurun_out/final/bench_prof.json 2> gpurun_out/final/bench_prof.err || { echo "rocprof failed"; tail -5 gpurun_out/final/bench_prof.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/final/prof1 -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs --streams 1 --per-view-backward > gpurun_out/final/bench_prof1.json 2> gpurun_out/final/bench_prof1.err || { echo "rocprof 1 failed"; tail -5 gpurun_out/final/bench_prof1.err; exit 1; }
head -12 gpurun_out/final/prof/run_kernel_stats.csv | cut -d, -f1-4
