#!/bin/bash
# round 6 (session 2): the bucket's sparse clear on the caller's stream before the forwards (--serial-zero) vs on
# a view stream beside them (default).  (via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/ab12; mkdir -p $O
for r in 1 2 3; do
  for cfg in side serial; do
    case $cfg in side) A="";; serial) A="--serial-zero";; esac
    timeout -k 10 240 python bench.py --steps 40 --warmup 5 --no-side-legs --no-cpu-baseline $A \
        > $O/bench_$cfg$r.json 2> $O/bench_$cfg$r.err || { echo "bench $cfg failed"; tail -5 $O/bench_$cfg$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/bench_$cfg$r.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$cfg', d['value'], 'step', d['step_ms']['p50'], 'host', d['host_ms_per_step']['busy'], d['host_ms_per_step']['wait'])"
  done
done
