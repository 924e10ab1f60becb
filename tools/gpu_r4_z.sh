#!/bin/bash
# round 4, GPU call z: vectorized histogram loads — the GPU suite, then c4 and the c2 bench against the
# previous histogram (dge_amd/lib/var/oldhist.so), alternating
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4z
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
OUT=r4z VARS=oldhist bash tools/gpu_r4_x.sh || exit 1
NOTESTS=1 VARS=oldhist ROUNDS=2 bash tools/gpu_ab.sh || exit 1
