#!/bin/bash
# GPU suite, then an A/B bench of one environment switch (run via gpurun):
#   AB_VAR=NAME AB_A=value AB_B=value bash tools/gpu_ab_env.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -2 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/gpu_tests.log | head; exit $rc; }
: > gpurun_out/ab_env.log
for rep in 1 2 3; do
  for val in "$AB_A" "$AB_B"; do
    env "$AB_VAR=$val" timeout -k 10 240 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-side-legs \
        > gpurun_out/ab_one.json 2>> gpurun_out/ab.err || { echo "bench failed for $val"; exit 1; }
    python - "$AB_VAR=$val" >> gpurun_out/ab_env.log <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_one.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:28s} {d['value']:9.1f} renders/s", " ".join(f"{k}={v*1000:.1f}" for k, v in d["stages_ms"].items()))
PY
  done
done
cat gpurun_out/ab_env.log
