#!/bin/bash
# round 4, GPU call r: render()'s speculated training render — the GPU suite, then DGE's unchanged loop
# (tools/probes/dge_loop_profile.py) with DGE_AMD_SPEC_RENDER 1 / 0 alternating, then the default bench line
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4r
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for r in 1 2; do
  for v in 1 0; do
    DGE_AMD_SPEC_RENDER=$v timeout -k 10 200 python tools/probes/dge_loop_profile.py > $O/loop_$v$r.txt 2>&1 || { tail -5 $O/loop_$v$r.txt; exit 1; }
    echo "spec $v: $(grep 'dge loop' $O/loop_$v$r.txt)"
  done
done
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], json.dumps(d['legs']['dge_loop_unchanged'])[:300])"
