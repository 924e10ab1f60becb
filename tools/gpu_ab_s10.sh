#!/bin/bash
# round 6 (session 2): the preprocess counters published by the depth sort's first kernel and polled by the host
# (default) vs the D2H copy + event (DGE_AMD_COUNT_COPY=1); the whole GPU suite first.  (via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/ab10; mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests \
    > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for cfg in pub copy; do
    case $cfg in pub) E="DGE_AMD_COUNT_COPY=0";; copy) E="DGE_AMD_COUNT_COPY=1";; esac
    env $E timeout -k 10 240 python bench.py --steps 40 --warmup 5 --no-side-legs --no-cpu-baseline \
        > $O/bench_$cfg$r.json 2> $O/bench_$cfg$r.err || { echo "bench $cfg failed"; tail -5 $O/bench_$cfg$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/bench_$cfg$r.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$cfg', d['value'], 'step', d['step_ms']['p50'], 'host', d['host_ms_per_step']['busy'], d['host_ms_per_step']['wait'])"
  done
done
