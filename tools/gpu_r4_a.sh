#!/bin/bash
# round 4, first GPU call: the new tests first, then the whole GPU suite, the default bench, a short bench
# under the warning tracer, and the 2-rank bench spawned by bench.py itself (gloo on one card)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/r4a
mkdir -p $O
python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)), 'cpu_count', os.cpu_count(), 'OMP', os.environ.get('OMP_NUM_THREADS')); print(open('/sys/fs/cgroup/cpu.max').read() if os.path.exists('/sys/fs/cgroup/cpu.max') else 'no cpu.max')" > $O/host.txt 2>&1
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider -s \
  tests/test_gpu_multiview.py -k "overflow or c2_timed or c2_speculated" > $O/pytest_new.log 2>&1 || { tail -30 $O/pytest_new.log; exit 1; }
tail -3 $O/pytest_new.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider tests > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
tail -c 600 $O/bench.json
timeout -k 10 300 python tools/warn_trace.py --steps 5 --warmup 3 --no-cpu-baseline > $O/warn.json 2> $O/warn.err || { tail -20 $O/warn.err; exit 1; }
DGE_AMD_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_gloo2.json 2> $O/bench_gloo2.err || { tail -20 $O/bench_gloo2.err; exit 1; }
tail -c 800 $O/bench_gloo2.json
