#!/bin/bash
# GPU suite, then the two traffic passes (FETCH_SIZE, WRITE_SIZE) and the VALU pass on a short default bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/r3 gpurun_out/pmc
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r3/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/r3/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/r3/pytest_gpu.log | head -20; exit $rc; }
rm -rf gpurun_out/pmc/p*
CMD="python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-profile --no-side-legs ${PMC_BENCH_ARGS:-}"
i=0
for group in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $group -d gpurun_out/pmc/p$i -o run --output-format csv -- $CMD > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i [$group] rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt 2>&1; grep -E "^k_render|^k_gauss|^k_preprocess|^k_scan_emit|^k_radix" gpurun_out/pmc/summary.txt | cut -c1-200
python -c "
import json; d=json.load(open('gpurun_out/pmc/pmc_traffic.json'))
for k,v in d.items(): print(k, v['read_bytes_per_launch']/1e6, v['write_bytes_per_launch']/1e6, v.get('valu_insts_per_launch'))"
