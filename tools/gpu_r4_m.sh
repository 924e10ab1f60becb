#!/bin/bash
# round 4, GPU call m: the pruned build (per-view streams only) — GPU suite, then the default bench line
# (side legs included: the AccumulateGrad warning check is its stderr)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -1 $O/bench.json | cut -c1-600
grep -c "AccumulateGrad" $O/bench.err || true
