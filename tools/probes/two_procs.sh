#!/bin/bash
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
mkdir -p gpurun_out
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-side-legs --no-profile > gpurun_out/one.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/one.json'));print('single', d['value'])"
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-side-legs --no-profile > gpurun_out/p1.json 2>/dev/null &
p1=$!
timeout -k 10 300 python bench.py --steps 200 --warmup 10 --no-cpu-baseline --no-side-legs --no-profile > gpurun_out/p2.json 2>/dev/null &
p2=$!
wait $p1 || exit 1
wait $p2 || exit 1
python -c "import json;a=json.load(open('gpurun_out/p1.json'));b=json.load(open('gpurun_out/p2.json'));print('two procs', a['value'], b['value'], 'sum', a['value']+b['value'])"
