#!/bin/bash
# Kernel times of the c4 leg under rocprofv3 (DGE_AMD_BINNING in the environment picks the binning).
O=gpurun_out/c4prof
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python tools/bench_configs.py c4 --steps 10 --warmup 3 > $O/prof.log 2>&1 || { echo "prof rc=$?"; tail -20 $O/prof.log; exit 3; }
f=$(ls $O/prof/run_kernel_stats.csv $O/prof/*/run_kernel_stats.csv 2>/dev/null | head -1)
cut -d, -f1-4 "$f" | head -25
