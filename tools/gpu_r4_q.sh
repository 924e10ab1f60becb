#!/bin/bash
# round 4, GPU call q: kernel timelines of one steady step of the one-rank RCCL rehearsal, row chunks 4 vs 0
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4q
mkdir -p $O
export TMPDIR=/tmp RANK=0 LOCAL_RANK=0 WORLD_SIZE=1 MASTER_ADDR=127.0.0.1 DGE_AMD_BENCH_DIST=1
for c in 4 0; do
  DGE_AMD_ROWS_CHUNKS=$c MASTER_PORT=$((29640 + c)) timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof$c -o run -- \
      python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs --no-profile > $O/out$c.json 2> $O/err$c.txt \
      || { tail -5 $O/err$c.txt; exit 1; }
  f=$(ls $O/prof$c/run_kernel_trace.csv 2>/dev/null || find $O/prof$c -name "*kernel_trace.csv" | head -1)
  echo "== chunks $c: $(tail -1 $O/out$c.json | cut -c60-120)"
  python tools/probes/step_timeline.py $f k_gauss_live > $O/step$c.txt 2>&1
  tail -45 $O/step$c.txt
done
