#!/bin/bash
# round 5 validation call: the whole GPU suite, the default bench line (side legs included) and the side
# configs (c4, c5, adam).  usage: tools/gpu_r5_full.sh <tag>   (run via gpurun)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest.log 2>&1 || { grep -E "parity|PASS|FAIL|Error" $O/pytest.log | tail -30; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'p50', d['step_ms']['p50'], 'frac', d['roofline']['frac'], 'stages', d.get('stages_ms'))
print('legs', json.dumps(d.get('legs'))[:1500])"
timeout -k 10 300 python -u tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cut -c1-400 $O/configs.jsonl
