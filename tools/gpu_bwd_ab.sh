#!/bin/bash
# merged (per-tile) vs per-quadrant backward: parity tests, then interleaved bench A/B (run via gpurun)
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_multiview.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > gpurun_out/pytest_bwd.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_bwd.log; [ $rc -eq 0 ] || { grep -E "Error|FAIL|assert" gpurun_out/pytest_bwd.log | head -20; exit $rc; }
: > gpurun_out/bwd_ab.log
for rep in 1 2; do for mode in tile quad; do
DGE_AMD_BWD=$mode timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-side-legs > gpurun_out/ab.json 2> gpurun_out/ab.err || { echo "bench $mode failed"; tail -5 gpurun_out/ab.err; exit 1; }
python - $mode <<'PY' >> gpurun_out/bwd_ab.log
import json, sys
d = json.loads(open("gpurun_out/ab.json").read().strip().splitlines()[-1])
print(f"{sys.argv[1]:5s} {d['value']:8.1f} renders/s  render_bwd {d['stages_ms'].get('render_bwd')} gauss_bwd {d['stages_ms'].get('gauss_bwd')} iso {d['roofline_leg']}")
PY
done; done
cat gpurun_out/bwd_ab.log
