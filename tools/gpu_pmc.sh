#!/bin/bash
# PMC counters per kernel on the GPU box (run via gpurun): one rocprofv3 pass
# per counter group (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950),
# --kernel-trace only (no sys/runtime trace with --pmc).  Stops at the first
# crash/timeout; a pass that is merely rejected (unknown counter) is skipped.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CMD=${PMC_CMD:-"python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-profile --no-side-legs ${PMC_BENCH_ARGS:-}"}
OUT=${PMC_OUT:-gpurun_out/pmc}
mkdir -p $OUT
i=0
while read -r group; do
  [ -z "$group" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --pmc $group -d $OUT/p$i -o run --output-format csv -- $CMD \
      > $OUT/p$i.log 2>&1
  rc=$?
  echo "pass $i [$group] rc=$rc"
  case $rc in 0) ;; 124|134|137|139) echo "aborting after rc=$rc"; exit $rc ;; *) tail -5 $OUT/p$i.log ;; esac
done <<'GROUPS'
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_BRANCH
TCC_HIT_sum TCC_MISS_sum
GROUPS
python tools/pmc_summary.py $OUT > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
