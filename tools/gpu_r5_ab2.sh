#!/bin/bash
# round 5: a pytest selection, alternating A/B benches of $CFGS (tools/gpu_ab_cfg.sh), a rocprofv3 kernel
# trace of the default bench.  usage: CFGS="..." tools/gpu_r5_ab2.sh <tag> "<pytest -k expression>" (gpurun)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests -k "$2" > $O/pytest.log 2>&1 || { grep -E "parity|PASS|FAIL|Error" $O/pytest.log | tail -30; exit 1; }
  grep -E "passed|failed" $O/pytest.log | tail -1
fi
if [ -n "$CFGS" ]; then
  timeout -k 10 1200 bash tools/gpu_ab_cfg.sh $O/ab > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
  cat $O/ab.txt
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs > $O/bench_prof.log 2> $O/bench_prof.err || { echo "rocprof failed $?"; tail -20 $O/bench_prof.err; exit 1; }
S=$(find $O/prof -name "*kernel_stats.csv" | head -1)
head -24 $S | cut -d, -f1-6
