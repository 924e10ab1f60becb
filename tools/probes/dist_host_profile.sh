#!/bin/bash
# cProfile of the one-rank RCCL rehearsal's host side (run via gpurun): where the 1.5 ms/step goes
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/disthost
export RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29541 DGE_AMD_BENCH_DIST=1
timeout -k 10 300 python -m cProfile -o gpurun_out/disthost/prof.out bench.py --steps 200 --warmup 5 --no-cpu-baseline \
    --no-side-legs --no-profile > gpurun_out/disthost/out.json 2> gpurun_out/disthost/err.txt || { tail -5 gpurun_out/disthost/err.txt; exit 1; }
tail -1 gpurun_out/disthost/out.json | cut -c1-150
python - <<'PY'
import pstats
p = pstats.Stats("gpurun_out/disthost/prof.out")
p.sort_stats("tottime").print_stats(25)
PY
