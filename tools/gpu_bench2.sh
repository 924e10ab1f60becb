#!/bin/bash
# the default bench line twice, plus the allocator stats (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
for i in 1 2; do
timeout -k 10 500 python bench.py ${BENCH_ARGS:-} > gpurun_out/bench$i.log 2> gpurun_out/bench$i.err || { echo "bench failed $?"; tail -20 gpurun_out/bench$i.err; exit 1; }
python - $i <<'PY'
import json, sys; d = json.loads(open(f"gpurun_out/bench{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("value", d["value"], "ms/step", d["ms_per_step"], "alloc", d.get("allocator_timed_region"), "iso", d.get("roofline_leg"))
PY
done
