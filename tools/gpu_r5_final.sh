#!/bin/bash
# round 5 validation + evidence call: the whole GPU suite, the default bench line (side legs included), the
# side configs, and rocprofv3 kernel stats of the bench at 3 streams and at one stream (their summaries are
# what profiles/r05/final holds).  usage: tools/gpu_r5_final.sh <tag>   (run via gpurun)
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
print('dge', d['legs']['dge_loop_unchanged']['value'], 'cpu', d['cpu_baseline']['value'] if d.get('cpu_baseline') else None)"
timeout -k 10 300 python -u tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
cut -c1-300 $O/configs.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof3 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs > $O/prof3.log 2>&1 || { echo "rocprof failed $?"; tail -20 $O/prof3.log; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof1 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs --streams 1 --no-profile > $O/prof1.log 2>&1 || { echo "rocprof failed $?"; tail -20 $O/prof1.log; exit 1; }
for d in prof3 prof1; do S=$(find $O/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; head -14 $S | cut -d, -f1-6; done
