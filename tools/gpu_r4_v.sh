#!/bin/bash
# round 4, GPU call v: c4 (2.5M Gaussians, 1080p, forward only) kernel breakdown
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python tools/bench_configs.py c4 > $O/c4.json 2> $O/c4.err || { tail -5 $O/c4.err; exit 1; }
tail -1 $O/c4.json | cut -c1-300
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
head -20 $f | cut -d, -f1-4
