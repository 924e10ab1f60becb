#!/bin/bash
# deferred union check (run via gpurun): the multiview/bucket GPU tests, then the one-rank RCCL rehearsal
# A/B: deferred (default) vs --sync-union, and the plain one-GPU bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/defer
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -m gpu tests/test_gpu_multiview.py tests/test_gpu_bucket.py -s > gpurun_out/defer/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/defer/pytest.log; grep "\[deferred\]" gpurun_out/defer/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|FAILED|assert" gpurun_out/defer/pytest.log | head -30; exit $rc; }
p=29540
for r in 1 2; do
  for m in defer sync; do
    a=""; [ $m = sync ] && a="--sync-union"; p=$((p+1))
    DGE_AMD_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port $p bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs $a > gpurun_out/defer/$m$r.json 2> gpurun_out/defer/$m$r.err || { echo "rccl $m failed"; tail -20 gpurun_out/defer/$m$r.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/defer/$m$r.json').read().strip().splitlines()[-1])
print('$m', d['value'], 'step', d['step_ms'], 'host', d.get('host_ms_per_step'))"
  done
done
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-side-legs --no-cpu-baseline > gpurun_out/defer/single.json 2> gpurun_out/defer/single.err || { echo "bench failed"; tail -5 gpurun_out/defer/single.err; exit 1; }
cut -c1-160 gpurun_out/defer/single.json
