#!/bin/bash
# round 5: alternating A/B benches of $CFGS (tools/gpu_ab_cfg.sh), then rocprofv3 kernel stats of the in-tree
# library on ONE stream (every kernel in isolation).  usage: CFGS="..." tools/gpu_r5_ab3.sh <tag>  (gpurun)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ -n "$CFGS" ]; then
  timeout -k 10 1200 bash tools/gpu_ab_cfg.sh $O/ab > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
  cat $O/ab.txt
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof1 -o one -- python bench.py --streams 1 --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs --no-profile > $O/bench_prof1.log 2> $O/bench_prof1.err || { echo "rocprof failed $?"; tail -20 $O/bench_prof1.err; exit 1; }
S=$(find $O/prof1 -name "*kernel_stats.csv" | head -1)
head -24 $S | cut -d, -f1-6
