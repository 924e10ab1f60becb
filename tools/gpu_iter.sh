#!/bin/bash
# One iteration on the GPU box (run via gpurun): parity tests, bench (+ per-stage times), blend diagnostics.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/parity.log 2>&1
rc=$?; tail -4 gpurun_out/parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench.log 2> gpurun_out/bench.err \
    || { echo "bench failed"; tail -20 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json; d = json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"]); print("stages", d.get("stages_ms"))
PY
timeout -k 10 200 python tools/diag_blend.py > gpurun_out/diag.log 2>&1 || { echo "diag failed"; exit 1; }
grep -E "==|p50|p99|p100|kept/wave|loop share|running" gpurun_out/diag.log
