#!/bin/bash
# round 4, last GPU call: the GPU suite, the default bench line, the self-spawned two-rank rehearsal (gloo on
# the one card) and the one-rank RCCL rehearsal of the distributed step
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4final
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(d['value'], d['step_ms']['p50'], d['roofline']['frac'])"
DGE_AMD_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs > $O/gloo2.log 2> $O/gloo2.err || { echo "gloo two-rank failed"; tail -20 $O/gloo2.err; exit 1; }
tail -1 $O/gloo2.log | cut -c1-200
DGE_AMD_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29712 bench.py --gpus 1 --steps 30 --warmup 5 --no-cpu-baseline --no-side-legs > $O/dist1.log 2> $O/dist1.err || { echo "rccl one-rank failed"; tail -20 $O/dist1.err; exit 1; }
tail -1 $O/dist1.log | cut -c1-200
