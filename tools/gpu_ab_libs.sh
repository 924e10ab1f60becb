#!/bin/bash
# A/B of several builds of the library on one box (run via gpurun):
#   LIBS="new head pipe" bash tools/gpu_ab_libs.sh
# "new" is the in-tree dge_amd/lib/libgs_raster.so, any other name dge_amd/lib/var/NAME.so.
# Per build: the GPU parity tests in $TESTS (a failing test is reported, the next build still runs),
# then the blend diagnostics of one c2 render; then ROUNDS alternating benches of every build.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/abl
TESTS=${TESTS:-tests/test_gpu_parity.py}
libpath() { [ "$1" = new ] && echo "" || echo "$PWD/dge_amd/lib/var/$1.so"; }
for v in $LIBS; do
  if [ -z "$NOTESTS" ]; then
    DGE_AMD_LIB=$(libpath $v) timeout -k 10 400 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 \
        --timeout-method thread -m gpu $TESTS > gpurun_out/abl/pytest_$v.log 2>&1
    rc=$?; echo "$v tests: $(tail -1 gpurun_out/abl/pytest_$v.log)"
    [ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
  fi
  DGE_AMD_LIB=$(libpath $v) timeout -k 10 200 python tools/diag_blend.py > gpurun_out/abl/diag_$v.txt 2>&1 \
      || { echo "diag $v failed"; tail -5 gpurun_out/abl/diag_$v.txt; exit 1; }
  echo "$v diag: $(grep -A6 '== render_fwd' gpurun_out/abl/diag_$v.txt | grep -E 'span|p100|per kept' | tr '\n' ' ')"
done
for r in $(seq ${ROUNDS:-2}); do
  for v in $LIBS; do
    DGE_AMD_LIB=$(libpath $v) timeout -k 10 240 python bench.py --steps 40 --warmup 5 --no-side-legs --no-cpu-baseline \
        > gpurun_out/abl/bench_$v$r.json 2> gpurun_out/abl/bench_$v$r.err || { echo "bench $v failed $?"; tail -5 gpurun_out/abl/bench_$v$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('gpurun_out/abl/bench_$v$r.json').read().strip().splitlines()[-1]); s=d['stages_ms']
print('$v', d['value'], 'step', d['step_ms']['p50'], 'iso', d['roofline_leg']['renders_per_s'], ' '.join(f'{k} {v*1e3:.1f}' for k, v in s.items()))"
  done
done
