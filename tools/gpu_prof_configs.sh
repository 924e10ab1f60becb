#!/bin/bash
# rocprofv3 kernel stats of one side config of tools/bench_configs.py (run via gpurun):
#   WORKLOAD=c4 bash tools/gpu_prof_configs.sh
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
W=${WORKLOAD:-c4}
mkdir -p gpurun_out/prof_$W
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d gpurun_out/prof_$W/prof -o run -- \
    python tools/bench_configs.py $W --steps 10 --warmup 3 > gpurun_out/prof_$W/out.txt 2>&1 || { tail -5 gpurun_out/prof_$W/out.txt; exit 1; }
python3 - "$W" <<'PY'
import csv, sys
w = sys.argv[1]
r = list(csv.DictReader(open(f"gpurun_out/prof_{w}/prof/run_kernel_stats.csv")))
for x in r[:20]:
    print(x["Name"][:110], x["Calls"], round(float(x["AverageNs"]) / 1e3, 1))
PY
