#!/bin/bash
# stream -> hardware-queue mapping of the distributed and the one-GPU bench step (run via gpurun): kernel
# traces, one steady step of each taken apart (tools/probes/step_timeline.py), then plain benches
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
bash tools/gpu_dist_prof.sh > /dev/null || exit $?
python3 tools/probes/step_timeline.py gpurun_out/distprof/prof/run_kernel_trace.csv > gpurun_out/distprof/step.txt
head -30 gpurun_out/distprof/step.txt; tail -1 gpurun_out/distprof/step.txt
mkdir -p gpurun_out/q1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -T --output-format csv -d gpurun_out/q1/prof -o run -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs --no-profile > gpurun_out/q1/out.json 2> gpurun_out/q1/err.txt || { tail -5 gpurun_out/q1/err.txt; exit 1; }
python3 tools/probes/step_timeline.py gpurun_out/q1/prof/run_kernel_trace.csv > gpurun_out/q1/step.txt
head -30 gpurun_out/q1/step.txt; tail -1 gpurun_out/q1/step.txt
for r in 1 2; do
DGE_AMD_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2955$r bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs > gpurun_out/q1/dist$r.json 2> gpurun_out/q1/dist$r.err || { echo "rccl failed"; tail -20 gpurun_out/q1/dist$r.err; exit 1; }
cut -c1-170 gpurun_out/q1/dist$r.json
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-side-legs --no-cpu-baseline > gpurun_out/q1/single$r.json 2> gpurun_out/q1/single$r.err || { echo "bench failed"; tail -5 gpurun_out/q1/single$r.err; exit 1; }
cut -c1-170 gpurun_out/q1/single$r.json
done
