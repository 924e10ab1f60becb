#!/bin/bash
# rocprofv3 kernel trace of the one-rank RCCL rehearsal (run via gpurun): the process group comes from
# the environment (RANK/WORLD_SIZE/MASTER_*), so the profiled program is python itself (no launcher)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/distprof
export TMPDIR=/tmp RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29531 DGE_AMD_BENCH_DIST=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/distprof/prof -o run -- \
    python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs --no-profile > gpurun_out/distprof/out.json 2> gpurun_out/distprof/err.txt \
    || { tail -5 gpurun_out/distprof/err.txt; exit 1; }
tail -1 gpurun_out/distprof/out.json | cut -c1-200
python3 - <<'PY'
import csv
r = list(csv.DictReader(open("gpurun_out/distprof/prof/run_kernel_stats.csv")))
for x in r[:24]:
    print(x["Name"][:90], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1), x["Percentage"])
PY
