#!/bin/bash
# A/B of two builds of the library on one box: the GPU suite on the in-tree build, then the default
# bench alternating the in-tree build (new) and dge_amd/lib/var/$v.so for v in VARS (default: base, a build of
# the commit compared against), ROUNDS times each.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/ab
if [ -z "$NOTESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests} > gpurun_out/ab/pytest.log 2>&1
  rc=$?; tail -3 gpurun_out/ab/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/ab/pytest.log | head -30; exit $rc; }
fi
for r in $(seq ${ROUNDS:-2}); do
  for v in new ${VARS:-base}; do
    lib=""; [ $v != new ] && lib=$PWD/dge_amd/lib/var/$v.so
    DGE_AMD_LIB=$lib timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-side-legs --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/ab/$v$r.json 2> gpurun_out/ab/$v$r.err || { echo "bench $v failed $?"; tail -5 gpurun_out/ab/$v$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/ab/$v$r.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$v', d['value'], 'step', d['step_ms']['p50'], 'iso', d['roofline_leg']['renders_per_s'], ' '.join(f'{k} {v*1e3:.1f}' for k, v in s.items()))"
  done
done
