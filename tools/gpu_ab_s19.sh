#!/bin/bash
# round 6 (session 2): the merged per-Gaussian pass in batches of (Gaussian, view) pairs (k_gauss_bwd_mixed,
# default) vs view by view (DGE_AMD_GAUSS_MIX=0): the whole GPU suite under the default, then alternating benches
# with the high-live leg.  (via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/ab19; mkdir -p $O
DGE_AMD_GAUSS_MIX=1 timeout -k 10 900 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests \
    > $O/pytest.log 2>&1 || { grep -E "Error|assert|FAILED|passed|failed" $O/pytest.log | tail -20; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for cfg in mix view; do
    case $cfg in mix) E="DGE_AMD_GAUSS_MIX=1";; view) E="DGE_AMD_GAUSS_MIX=0";; esac
    env $E timeout -k 10 240 python bench.py --steps 40 --warmup 5 --no-side-legs --no-cpu-baseline \
        > $O/bench_$cfg$r.json 2> $O/bench_$cfg$r.err || { echo "bench $cfg failed"; tail -5 $O/bench_$cfg$r.err; exit 1; }
    env $E timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-side-legs --no-cpu-baseline --opacity-mean -2 --opacity-std 1 \
        > $O/hl_$cfg$r.json 2> $O/hl_$cfg$r.err || { echo "bench hl $cfg failed"; tail -5 $O/hl_$cfg$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/bench_$cfg$r.json').read().strip().splitlines()[-1]); s=d['stages_ms']
h=json.loads(open('$O/hl_$cfg$r.json').read().strip().splitlines()[-1])
print('$cfg', d['value'], 'step', d['step_ms']['p50'], 'gauss_bwd', s.get('gauss_bwd'), '| high-live', h['value'], 'gauss_bwd', h['stages_ms'].get('gauss_bwd'))"
  done
done
