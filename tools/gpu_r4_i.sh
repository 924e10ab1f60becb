#!/bin/bash
# round 4, GPU call i: the batched-views tests with the shared preprocess (k_preprocess_views), A/B of it,
# the warning tracer, the bench-spawned 2-rank gloo run
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4i
mkdir -p $O
DGE_AMD_VIEWS_PRE=1 timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests/test_gpu_multiview.py > $O/pytest_mv_pre.log 2>&1 || { tail -40 $O/pytest_mv_pre.log; exit 1; }
tail -2 $O/pytest_mv_pre.log
VAR=DGE_AMD_VIEWS_PRE VALS="1 0" NOTESTS=1 ROUNDS=3 bash tools/gpu_env_ab.sh || exit 1
timeout -k 10 300 python tools/warn_trace.py --steps 5 --warmup 3 --no-cpu-baseline --no-side-legs > $O/warn.json 2> $O/warn.err || { tail -20 $O/warn.err; exit 1; }
grep -A30 "warn-trace" $O/warn.err | head -45
DGE_AMD_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-side-legs --no-cpu-baseline > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { tail -20 $O/bench_gloo2.err; exit 1; }
python -c "import json; d=json.loads(open('$O/bench_gloo2.json').read().strip().splitlines()[-1]); print(d['value'], d['n_gpus'], d.get('distributed'))"
timeout -k 10 300 python tools/probes/dge_loop_profile.py > $O/dge_loop_profile.txt 2>&1 || { tail -20 $O/dge_loop_profile.txt; exit 1; }
head -60 $O/dge_loop_profile.txt | cut -c1-150
