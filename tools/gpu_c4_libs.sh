#!/bin/bash
# c4 leg (tools/bench_configs.py c4) for several builds of the library (run via gpurun):
#   LIBS="new c4k ..." bash tools/gpu_c4_libs.sh   ("new" = in-tree, else dge_amd/lib/var/NAME.so)
# TESTS_LIB=NAME: the binning parity tests with that build first.
set -o pipefail
O=gpurun_out/c4libs
mkdir -p $O
libpath() { [ "$1" = new ] && echo "" || echo "$PWD/dge_amd/lib/var/$1.so"; }
if [ -n "$TESTS_LIB" ]; then
  DGE_AMD_LIB=$(libpath $TESTS_LIB) timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q \
      -p no:cacheprovider --timeout 200 --timeout-method thread -k "region_emission or two_level_binning or c4_hd" \
      > $O/tests_$TESTS_LIB.log 2>&1
  rc=$?; echo "$TESTS_LIB tests: $(tail -1 $O/tests_$TESTS_LIB.log)"
  [ $rc -le 1 ] || { echo "pytest rc $rc: stopping"; exit $rc; }
fi
for r in $(seq ${ROUNDS:-2}); do
  for v in $LIBS; do
    DGE_AMD_LIB=$(libpath $v) timeout -k 10 200 python tools/bench_configs.py c4 --steps 20 --warmup 3 \
        > $O/c4_$v$r.json 2> $O/c4_$v$r.err || { echo "c4 $v failed $?"; tail -5 $O/c4_$v$r.err; exit 1; }
    echo "$v $(tail -1 $O/c4_$v$r.json)"
  done
done
