#!/bin/bash
# round 3 evidence: rocprofv3 --stats of the default bench (kernel summary) + the one-stream bench, then
# the PMC passes (tools/gpu_pmc.sh).  PMC_BUILD: the git revision stamped into pmc_traffic.json.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/r3
export TMPDIR=/tmp
TAG=${TAG:-stats}
for s in 3 1; do
  rm -rf gpurun_out/r3/${TAG}_s$s
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3/${TAG}_s$s -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs --streams $s > gpurun_out/r3/${TAG}_s$s.log 2> gpurun_out/r3/${TAG}_s$s.err || { echo "rocprof failed $?"; tail -20 gpurun_out/r3/${TAG}_s$s.err; exit 1; }
  f=$(find gpurun_out/r3/${TAG}_s$s -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/r3/kernel_stats_${TAG}_s$s.csv
  head -12 "$f" | cut -d, -f1-8
  find gpurun_out/r3/${TAG}_s$s -name "*kernel_trace.csv" -exec gzip -f {} \;
done
[ -n "$NOPMC" ] && exit 0
bash tools/gpu_pmc.sh
