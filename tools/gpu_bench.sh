#!/bin/bash
# the default bench line (run via gpurun); extra args in BENCH_ARGS
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench.log 2> gpurun_out/bench.err || { echo "bench failed $?"; tail -20 gpurun_out/bench.err; exit 1; }
python - <<'PY'
import json; d = json.loads(open("gpurun_out/bench.log").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"]); print("stages", d.get("stages_ms"))
for k, r in d.get("rooflines", {}).items(): print(k, r)
print("legs", d.get("legs")); print("cpu", d.get("cpu_baseline"))
PY
