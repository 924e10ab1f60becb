#!/bin/bash
# the distributed step's stream -> hardware-queue mapping, then the one-rank RCCL rehearsal (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash tools/gpu_dist_prof.sh > /dev/null || exit $?
python3 tools/probes/step_timeline.py gpurun_out/distprof/prof/run_kernel_trace.csv > gpurun_out/distprof/step.txt
head -34 gpurun_out/distprof/step.txt; tail -1 gpurun_out/distprof/step.txt
mkdir -p gpurun_out/q2
for r in 1 2; do
DGE_AMD_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2956$r bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs > gpurun_out/q2/dist$r.json 2> gpurun_out/q2/dist$r.err || { echo "rccl failed"; tail -20 gpurun_out/q2/dist$r.err; exit 1; }
cut -c1-170 gpurun_out/q2/dist$r.json
done
