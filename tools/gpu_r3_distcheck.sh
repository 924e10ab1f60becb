#!/bin/bash
# GPU suite, then the one-rank RCCL rehearsal three times and the one-GPU bench twice (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/dc
timeout -k 10 600 python -u -m pytest tests -x -q -m gpu -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/dc/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/dc/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/dc/pytest_gpu.log | head -20; exit $rc; }
for r in 1 2 3; do
DGE_AMD_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 2957$r bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs > gpurun_out/dc/dist$r.json 2> gpurun_out/dc/dist$r.err || { echo "rccl failed"; tail -20 gpurun_out/dc/dist$r.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/dc/dist$r.json').read().strip().splitlines()[-1]); print('dist', d['value'], d['step_ms'])"
done
for r in 1 2; do
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-side-legs --no-cpu-baseline > gpurun_out/dc/single$r.json 2> gpurun_out/dc/single$r.err || { echo "bench failed"; tail -5 gpurun_out/dc/single$r.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/dc/single$r.json').read().strip().splitlines()[-1]); print('single', d['value'], d['step_ms'])"
done
