#!/bin/bash
# round 4, GPU call g: c4/c5 with the quadrant masks on and off; a rocprofv3 kernel trace of the default
# bench, its per-step phases and one steady step taken apart
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4g
mkdir -p $O
export TMPDIR=/tmp
for q in 1 0 1 0; do
  DGE_AMD_QMASK=$q timeout -k 10 300 python tools/bench_configs.py c4 c5 > $O/configs_q$q.jsonl 2> $O/configs_q$q.err || { tail -20 $O/configs_q$q.err; exit 1; }
  echo "QMASK=$q"; cut -c1-400 $O/configs_q$q.jsonl
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --steps 12 --warmup 5 --no-cpu-baseline --no-side-legs --no-profile > $O/trace.log 2> $O/trace.err || { echo "rocprof failed $?"; tail -20 $O/trace.err; exit 1; }
python -c "import json; d=json.loads(open('$O/trace.log').read().strip().splitlines()[-1]); print(d['value'], d['step_ms'], d['host_ms_per_step'])"
f=$(find $O/trace -name "*kernel_trace.csv" | head -1)
python tools/step_phases.py "$f" --steps 8 > $O/phases.txt; cat $O/phases.txt | tail -15
python tools/probes/step_timeline.py "$f" > $O/step.txt; cat $O/step.txt | tail -70
gzip -f "$f"
