#!/bin/bash
# round 6 (session 2): merged replay + fence-free pool events (new), system-fenced pool events (fence),
# per-view replays (new, DGE_AMD_REPLAY_MERGE=0), the live-set pass beside the merged replay (side); tests on
# new first.  (via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/ab8; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
    tests/test_gpu_multiview.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2 3; do
  for cfg in new fence merge0 side; do
    case $cfg in
      new) L=""; E="";;
      fence) L="$PWD/dge_amd/lib/var/fence.so"; E="";;
      merge0) L=""; E="DGE_AMD_REPLAY_MERGE=0";;
      side) L=""; E="DGE_AMD_LIVE_SIDE=1";;
    esac
    env DGE_AMD_LIB=$L $E timeout -k 10 240 python bench.py --steps 40 --warmup 5 --no-side-legs --no-cpu-baseline \
        > $O/bench_$cfg$r.json 2> $O/bench_$cfg$r.err || { echo "bench $cfg failed"; tail -5 $O/bench_$cfg$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/bench_$cfg$r.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$cfg', d['value'], 'step', d['step_ms']['p50'], 'host', d['host_ms_per_step']['busy'], d['host_ms_per_step']['wait'])"
  done
done
