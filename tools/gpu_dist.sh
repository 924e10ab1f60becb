#!/bin/bash
# distributed rehearsals on a one-GPU box (run via gpurun): RCCL one-rank group (the whole sparse-row
# all-reduce protocol), and two gloo ranks sharing the card
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
DGE_AMD_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs > gpurun_out/dist1.log 2> gpurun_out/dist1.err || { echo "rccl one-rank failed"; tail -20 gpurun_out/dist1.err; exit 1; }
tail -1 gpurun_out/dist1.log | cut -c1-300
DGE_AMD_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29514 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs --scan-live > gpurun_out/dist1s.log 2> gpurun_out/dist1s.err || { echo "rccl one-rank scan failed"; tail -20 gpurun_out/dist1s.err; exit 1; }
tail -1 gpurun_out/dist1s.log | cut -c1-300
DGE_AMD_BENCH_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs > gpurun_out/dist2.log 2> gpurun_out/dist2.err || { echo "gloo two-rank failed"; tail -20 gpurun_out/dist2.err; exit 1; }
tail -1 gpurun_out/dist2.log | cut -c1-400
