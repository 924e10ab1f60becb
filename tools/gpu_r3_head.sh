#!/bin/bash
# round 3 re-entry check (run via gpurun): GPU suite + A/B bench of the in-tree build against
# dge_amd/lib/var/base.so (tools/gpu_ab.sh), then the one-rank RCCL rehearsal of the whole protocol
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
ROUNDS=${ROUNDS:-3} bash tools/gpu_ab.sh || exit $?
DGE_AMD_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs > gpurun_out/dist1.log 2> gpurun_out/dist1.err || { echo "rccl one-rank failed"; tail -20 gpurun_out/dist1.err; exit 1; }
tail -1 gpurun_out/dist1.log | cut -c1-300
