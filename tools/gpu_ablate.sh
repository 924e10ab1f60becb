#!/bin/bash
# Marginal cost of each stage inside the concurrent 3-view step: the default bench with a probe build
# of the library (tools/build_variant.sh ablate -DGS_ABLATE -> dge_amd/lib/var/ablate.so) that skips the named stages (outputs meaningless).
set -o pipefail
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out/ablate
for a in none depth gauss rbwd fwd fwd,rbwd none; do
  DGE_AMD_LIB=$PWD/dge_amd/lib/var/ablate.so DGE_AMD_ABLATE=$a timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-side-legs --no-cpu-baseline --no-profile > gpurun_out/ablate/$a.json 2> gpurun_out/ablate/$a.err || { echo "ablate $a failed $?"; tail -5 gpurun_out/ablate/$a.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/ablate/$a.json').read().strip().splitlines()[-1]); print('$a', d['value'], 'step', d['step_ms']['p50'], 'host busy', d['host_ms_per_step']['busy'])"
done
