#!/bin/bash
# round 4: smoke() and the non-headline configs on the committed tree
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4smoke
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -30 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python -u tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cut -c1-220 $O/configs.jsonl
