#!/bin/bash
# round 4, GPU call d: the whole GPU suite (quadrant masks on), the parity suite with the masks off, A/B
# of the masks and of the staggered backward, rocPRIM's sort times, the full default bench, a kernel-stat
# profile of a short bench
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
grep -E "^\[(c2|overflow|deferred|parity c2)" $O/pytest_gpu.log | head -20
DGE_AMD_QMASK=0 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_parity.py > $O/pytest_parity_noqmask.log 2>&1 || { tail -40 $O/pytest_parity_noqmask.log; exit 1; }
tail -1 $O/pytest_parity_noqmask.log
VAR=DGE_AMD_QMASK VALS="1 0" NOTESTS=1 ROUNDS=2 bash tools/gpu_env_ab.sh || exit 1
timeout -k 10 400 python bench.py > $O/bench_full.json 2> $O/bench_full.err || { tail -20 $O/bench_full.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_full.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline'], d['stages_ms']); print(json.dumps(d['legs'])[:2500]); print(d['cpu_baseline'])"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 20 --warmup 5 --no-side-legs --no-cpu-baseline > $O/prof_bench.json 2> $O/prof_bench.err || { tail -20 $O/prof_bench.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -3
