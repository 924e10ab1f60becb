#!/bin/bash
# rocprofv3 kernel trace of the default bench; per-step phases (tools/step_phases.py) and overlap
# (tools/trace_busy.py).  BENCH_ARGS: extra bench flags.  TAG: output name.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
TAG=${TAG:-trace}
rm -rf gpurun_out/r3/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3/$TAG -o run -- python bench.py --steps 12 --warmup 5 --no-cpu-baseline --no-side-legs --no-profile ${BENCH_ARGS:-} > gpurun_out/r3/$TAG.log 2> gpurun_out/r3/$TAG.err || { echo "rocprof failed $?"; tail -20 gpurun_out/r3/$TAG.err; exit 1; }
python -c "import json; d=json.loads(open('gpurun_out/r3/$TAG.log').read().strip().splitlines()[-1]); print(d['value'], d['step_ms'], d['host_ms_per_step'])"
f=$(find gpurun_out/r3/$TAG -name "*kernel_trace.csv" | head -1)
python tools/step_phases.py "$f" --steps 8 | tee gpurun_out/r3/${TAG}_phases.txt
gzip -f "$f"
