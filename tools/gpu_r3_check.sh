#!/bin/bash
# round 3: GPU suite, then the driver-shaped bench (speculated batch, and --exact for comparison)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/r3
TESTS=${TESTS:-tests}
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/r3/pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/r3/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|error|FAILED|assert" gpurun_out/r3/pytest_gpu.log | head -30; exit $rc; }
[ -n "$NOBENCH" ] && exit 0
for m in ${MODES:-spec exact spec}; do
  args="--steps 20 --warmup 5"; [ $m = exact ] && args="$args --exact"; [ $m = serialzero ] && args="$args --serial-zero"
  timeout -k 10 240 python bench.py $args > gpurun_out/r3/bench_$m.json 2> gpurun_out/r3/bench_$m.err || { echo "bench $m failed $?"; tail -20 gpurun_out/r3/bench_$m.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r3/bench_$m.json').read().strip().splitlines()[-1])
print('$m', d['value'], 'iso', d['roofline_leg'], 'step', d['step_ms'], 'host', d['host_ms_per_step'], 'alloc', d['allocator_timed_region'], 'legs', {k: v['value'] for k, v in d['legs'].items()})"
done
