#!/bin/bash
# round 4, GPU call o: the row-chunked multi-GPU gradient SUM — the GPU suite (with the
# two-rank chunked test), then one-rank RCCL rehearsals of the bench's distributed step with and without
# chunks (alternating), and the self-spawned two-rank gloo rehearsal
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
grep "row chunks\]" $O/pytest_gpu.log | head -2
for r in 1 2; do
  for c in 4 0; do
    DGE_AMD_ROWS_CHUNKS=$c DGE_AMD_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $((29520 + r * 10 + c)) bench.py --gpus 1 --steps 30 --warmup 5 --no-cpu-baseline --no-side-legs > $O/dist1_c${c}_$r.log 2> $O/dist1_c${c}_$r.err || { echo "rccl one-rank chunks=$c failed"; tail -20 $O/dist1_c${c}_$r.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/dist1_c${c}_$r.log').read().strip().splitlines()[-1])
print('chunks $c round $r', d['value'], 'step', d['step_ms']['p50'], 'coll', d.get('collective_ms'), d.get('collective_share_p50'))"
  done
done
DGE_AMD_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs > $O/gloo2.log 2> $O/gloo2.err || { echo "gloo two-rank failed"; tail -20 $O/gloo2.err; exit 1; }
tail -1 $O/gloo2.log | cut -c1-300
