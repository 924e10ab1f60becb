#!/bin/bash
# rocprofv3 kernel + HIP runtime trace of the default bench: host issue time vs device start of each
# step's phases (tools/api_gap.py).  BENCH_ARGS: extra bench flags.  TAG: output name.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
TAG=${TAG:-apitrace}
rm -rf gpurun_out/r3/$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --output-format csv -d gpurun_out/r3/$TAG -o run -- python bench.py --steps 12 --warmup 5 --no-cpu-baseline --no-side-legs --no-profile ${BENCH_ARGS:-} > gpurun_out/r3/$TAG.log 2> gpurun_out/r3/$TAG.err || { echo "rocprof failed $?"; tail -20 gpurun_out/r3/$TAG.err; exit 1; }
python tools/api_gap.py gpurun_out/r3/$TAG --steps 8 | tee gpurun_out/r3/${TAG}_gap.txt
python tools/step_phases.py $(find gpurun_out/r3/$TAG -name "*kernel_trace.csv" | head -1) --steps 8 | tee gpurun_out/r3/${TAG}_phases.txt
find gpurun_out/r3/$TAG -name "*.csv" -exec gzip -f {} \;
