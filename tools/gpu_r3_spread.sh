#!/bin/bash
# round 3: the driver-shaped bench (--steps 20 --warmup 5) several times in a row on one box,
# per-step spread in each line; then one run without the side legs (is the AccumulateGrad
# stream-mismatch warning from the timed region or from the unfused side leg?)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/r3
N=${N:-4}
for i in $(seq 1 $N); do
  timeout -k 10 240 python bench.py --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/r3/spread_$i.json 2> gpurun_out/r3/spread_$i.err || { echo "bench $i failed $?"; tail -20 gpurun_out/r3/spread_$i.err; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/r3/spread_$i.json').read().strip().splitlines()[-1])
print($i, d['value'], 'iso', d['roofline_leg'], 'step', d['step_ms'], 'host', d['host_ms_per_step'], 'alloc', d['allocator_timed_region'])"
done
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-side-legs --no-cpu-baseline > gpurun_out/r3/nolegs.json 2> gpurun_out/r3/nolegs.err || exit 1
grep -c AccumulateGrad gpurun_out/r3/nolegs.err || true
python -c "
import json; d=json.loads(open('gpurun_out/r3/nolegs.json').read().strip().splitlines()[-1])
print('nolegs', d['value'], 'step', d['step_ms'], 'host', d['host_ms_per_step'])"
