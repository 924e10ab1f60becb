#!/bin/bash
# multiview GPU tests, then a bench with the side legs (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/mv
timeout -k 10 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_multiview.py} > gpurun_out/mv/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/mv/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/mv/pytest.log | head -20; exit $rc; }
[ -n "$NOBENCH" ] && exit 0
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/mv/bench.json 2> gpurun_out/mv/bench.err || { tail -5 gpurun_out/mv/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/mv/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['step_ms'], {k: v['value'] for k, v in d['legs'].items()})"
