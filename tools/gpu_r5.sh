#!/bin/bash
# round 5 working GPU call: a pytest selection, the default bench line, a rocprofv3 kernel trace of the
# bench (3-stream step) with its stats, and one steady step's timeline.
# usage: tools/gpu_r5.sh <tag> [pytest -k expression | -]   (run via gpurun)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
if [ "${2:--}" != "-" ]; then
  timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests -k "$2" > $O/pytest.log 2>&1 || { grep -E "parity|PASS|FAIL|Error" $O/pytest.log | tail -30; exit 1; }
  grep -E "passed|failed" $O/pytest.log | tail -1
fi
timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print('value', d['value'], 'p50', d['step_ms']['p50'], 'frac', d['roofline']['frac'], 'stages', d.get('stages_ms'))"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs > $O/bench_prof.log 2> $O/bench_prof.err || { echo "rocprof failed $?"; tail -20 $O/bench_prof.err; exit 1; }
T=$(find $O/prof -name "*kernel_trace.csv" | head -1)
S=$(find $O/prof -name "*kernel_stats.csv" | head -1)
python tools/probes/step_timeline.py $T > $O/timeline.txt 2>&1; tail -3 $O/timeline.txt
head -25 $S | cut -d, -f1-6
