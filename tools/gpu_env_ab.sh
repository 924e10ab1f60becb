#!/bin/bash
# Parity tests and benches of one environment variable's values (run via gpurun):
#   VAR=NAME VALS="a b c" [TESTS=...] [ROUNDS=2] bash tools/gpu_env_ab.sh
# Each value: the GPU tests in $TESTS under it (a failing test is reported; a crash stops the run),
# then ROUNDS alternating benches of every value.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/env
TESTS=${TESTS:-tests/test_gpu_parity.py}
for v in $VALS; do
  if [ -z "$NOTESTS" ]; then
    env "$VAR=$v" timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread \
        -m gpu $TESTS > gpurun_out/env/pytest_$v.log 2>&1
    rc=$?; echo "$VAR=$v tests: $(tail -1 gpurun_out/env/pytest_$v.log)"
    [ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
    [ $rc -eq 0 ] || grep -E "Error|assert|FAILED" gpurun_out/env/pytest_$v.log | head -10
  fi
done
for r in $(seq ${ROUNDS:-2}); do
  for v in $VALS; do
    env "$VAR=$v" timeout -k 10 240 python bench.py --steps 40 --warmup 5 --no-side-legs --no-cpu-baseline ${BENCH_ARGS:-} \
        > gpurun_out/env/bench_$v$r.json 2> gpurun_out/env/bench_$v$r.err || { echo "bench $v failed $?"; tail -5 gpurun_out/env/bench_$v$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/env/bench_$v$r.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$VAR=$v', d['value'], 'step', d['step_ms']['p50'], 'iso', d['roofline_leg']['renders_per_s'], ' '.join(f'{k} {v*1e3:.1f}' for k, v in s.items()))"
  done
done
