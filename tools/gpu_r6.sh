#!/bin/bash
# round 6 GPU call: stages picked by name.  usage (via gpurun): tools/gpu_r6.sh <tag> <stage>...
#   tests      the whole -m gpu suite            bench     the default bench line
#   configs    tools/bench_configs.py            prof      rocprofv3 kernel stats, 3 streams and 1 stream
#   parity     the fp64-truth gradient tests only (-k truth)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for st in "$@"; do
  case $st in
  tests)
    timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest.log 2>&1 || { grep -E "parity|PASS|FAIL|Error" $O/pytest.log | tail -30; exit 1; }
    grep -E "passed|failed" $O/pytest.log | tail -1 ;;
  parity)
    mkdir -p $O/dump; DGE_AMD_TRUTH_DUMP=$O/dump timeout -k 10 900 python -u -m pytest -v -s --timeout 600 --timeout-method thread -m gpu -k "truth or deferred" -p no:cacheprovider tests > $O/parity.log 2>&1 || { grep -E "truth|PASS|FAIL|Error" $O/parity.log | tail -30; exit 1; }
    grep -E "truth|passed|failed" $O/parity.log | tail -20 ;;
  bench)
    timeout -k 10 600 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
    python -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('value', d['value'], 'p50', d['step_ms']['p50'], 'frac', d['roofline']['frac'], 'stages', d.get('stages_ms'))
print('host', d.get('host_ms_per_step'))
print('legs', {k: v.get('value') if isinstance(v, dict) else v for k, v in d.get('legs', {}).items()})" ;;
  configs)
    timeout -k 10 300 python -u tools/bench_configs.py > $O/configs.jsonl 2> $O/configs.err || { tail -20 $O/configs.err; exit 1; }
    cut -c1-300 $O/configs.jsonl ;;
  prof)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof3 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs > $O/prof3.log 2>&1 || { echo "rocprof failed $?"; tail -20 $O/prof3.log; exit 1; }
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof1 -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs --streams 1 --no-profile > $O/prof1.log 2>&1 || { echo "rocprof failed $?"; tail -20 $O/prof1.log; exit 1; }
    for d in prof3 prof1; do S=$(find $O/$d -name "*kernel_stats.csv" | head -1); echo "== $d"; head -14 $S | cut -d, -f1-6; done ;;
  dist)
    # the RCCL protocol on a one-rank group (torch.distributed.run), then 4 ranks sharing the card over gloo
    DGE_AMD_BENCH_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
        --master-addr 127.0.0.1 --master-port 29511 bench.py --steps 20 --warmup 5 --no-side-legs --no-cpu-baseline \
        > $O/rccl1.json 2> $O/rccl1.err || { tail -20 $O/rccl1.err; exit 1; }
    DGE_AMD_BENCH_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 4 --steps 10 --warmup 3 --no-side-legs \
        --no-cpu-baseline > $O/gloo4.json 2> $O/gloo4.err || { tail -20 $O/gloo4.err; exit 1; }
    for f in rccl1 gloo4; do python -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
print('$f', d['value'], d['n_gpus'], 'p50', d['step_ms']['p50'], json.dumps(d.get('distributed')))"; done ;;
  *) echo "unknown stage $st"; exit 2 ;;
  esac
done
