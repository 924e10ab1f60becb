#!/bin/bash
# Stream-overlap sweep on the GPU box (run via gpurun): the c2 bench at 1/2/3 streams, per-view
# forward+backward and batch-backward orders.  One line per run in gpurun_out/streams.log.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
: > gpurun_out/streams.log
run() {
    timeout -k 10 240 python bench.py --steps ${STEPS:-60} --warmup 5 --no-cpu-baseline --no-side-legs --no-profile "$@" \
        > gpurun_out/streams_one.json 2> gpurun_out/streams_one.err || { echo "bench $* failed"; tail -20 gpurun_out/streams_one.err; exit 1; }
    python - "$*" <<'PY' >> gpurun_out/streams.log
import json, sys
d = json.loads(open("gpurun_out/streams_one.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1] or 'default':40s} {d['value']:9.1f} renders/s  {d['ms_per_step']:.4f} ms/step")
PY
}
for rep in 1 2; do
run ${EXTRA_ARGS:-}
run --stagger ${EXTRA_ARGS:-}
run --serial-zero ${EXTRA_ARGS:-}
done
cat gpurun_out/streams.log
