#!/bin/bash
# Forward-kernel A/B on the GPU box (run via gpurun): parity suite with the
# pipelined forward, then bench + blend diagnostics for both forward variants.
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiview.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
    > gpurun_out/parity.log 2>&1
rc=$?; tail -4 gpurun_out/parity.log; [ $rc -eq 0 ] || exit $rc
for v in 1 0 1; do
  DGE_AMD_FWD=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-side-legs > gpurun_out/bench_fwd$v.log 2> gpurun_out/bench_fwd$v.err \
      || { echo "bench failed"; tail -20 gpurun_out/bench_fwd$v.err; exit 1; }
  python - "$v" <<'PY'
import json, sys; d = json.loads(open(f"gpurun_out/bench_fwd{sys.argv[1]}.log").read().strip().splitlines()[-1])
print("fwd variant", sys.argv[1], "value", d["value"], "ms/step", d["ms_per_step"]); print("  stages", d.get("stages_ms"))
PY
done
for v in 1 0; do
  DGE_AMD_FWD=$v timeout -k 10 200 python tools/diag_blend.py > gpurun_out/diag_fwd$v.log 2>&1 || { echo "diag failed"; exit 1; }
  echo "== variant $v"; grep -A14 "== render_fwd" gpurun_out/diag_fwd$v.log
done
