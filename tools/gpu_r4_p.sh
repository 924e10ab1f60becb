#!/bin/bash
# round 4, GPU call p: where the host's time goes per step — cProfile (by own time) of the bench's one-GPU
# step and of the one-rank RCCL step with and without row chunks (200 steps dominate the profile)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4p
mkdir -p $O
A="--steps 200 --warmup 5 --no-cpu-baseline --no-side-legs --no-profile"
timeout -k 10 300 python -m cProfile -s tottime bench.py --gpus 1 $A > $O/prof_1gpu.txt 2> $O/prof_1gpu.err || { tail -5 $O/prof_1gpu.err; exit 1; }
for c in 0 4; do
  DGE_AMD_ROWS_CHUNKS=$c DGE_AMD_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29600 + c)) -m cProfile -s tottime bench.py --gpus 1 $A > $O/prof_dist_c$c.txt 2> $O/prof_dist_c$c.err || { tail -5 $O/prof_dist_c$c.err; exit 1; }
done
for f in $O/prof_1gpu.txt $O/prof_dist_c0.txt $O/prof_dist_c4.txt; do echo "== $f"; grep -m1 '"metric"' $f | cut -c1-120; grep -A28 "Ordered by" $f | cut -c1-160; done
