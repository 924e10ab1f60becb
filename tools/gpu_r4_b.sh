#!/bin/bash
# round 4, GPU call b: the whole GPU suite, rocPRIM's sort times, A/B of the cull (lib) and of the staggered
# backward (env), the warning tracer, the bench-spawned 2-rank gloo rehearsal, the full default bench
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
grep -E "^\[(c2|overflow|deferred|parity c2)" $O/pytest_gpu.log | head -20
timeout -k 10 120 tools/probes/rocprim_sort_time > $O/rocprim_sort.txt 2>&1; cat $O/rocprim_sort.txt
DGE_AMD_VIEWS_BWD=merged VARS="base wfma" NOTESTS=1 ROUNDS=2 bash tools/gpu_ab.sh || exit 1
VAR=DGE_AMD_VIEWS_BWD VALS="merged stagger" NOTESTS=1 ROUNDS=2 bash tools/gpu_env_ab.sh || exit 1
timeout -k 10 300 python tools/warn_trace.py --steps 5 --warmup 3 --no-cpu-baseline > $O/warn.json 2> $O/warn.err || { tail -20 $O/warn.err; exit 1; }
grep -A25 "warn-trace" $O/warn.err | head -40
DGE_AMD_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { tail -20 $O/bench_gloo2.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_gloo2.json').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d.get('distributed'))"
timeout -k 10 400 python bench.py > $O/bench_full.json 2> $O/bench_full.err || { tail -20 $O/bench_full.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_full.json').read().strip().splitlines()[-1]); print(d['value'], d['roofline']['avg_ms'], d['stages_ms'], json.dumps(d['legs'])[:1500]); print(d['cpu_baseline'])"
