#!/bin/bash
# Region emission check on one GPU: parity tests (region vs two-level vs two-pass vs oracle), then the c4 leg with
# the default (two-level) binning and with DGE_AMD_BINNING=region.  A step that faults, aborts or times out ends the script
# (pytest's exit 1 — failed tests — does not).
O=gpurun_out/r6region
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 200 --timeout-method thread \
    -p no:cacheprovider -k "region_emission or two_level_binning or c4_hd" > $O/tests.log 2>&1
rc=$?
tail -25 $O/tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests rc=$rc: stopping"; exit $rc; fi
timeout -k 10 200 python tools/bench_configs.py c4 > $O/c4.json 2> $O/c4.err || { echo "c4 rc=$?"; tail $O/c4.err; exit 3; }
cat $O/c4.json
DGE_AMD_BINNING=region timeout -k 10 200 python tools/bench_configs.py c4 > $O/c4_region.json 2> $O/c4_region.err \
    || { echo "c4 region rc=$?"; exit 3; }
cat $O/c4_region.json
exit $rc
