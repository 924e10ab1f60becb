#!/bin/bash
# round 5: a kernel change against the committed build (dge_amd/lib/var/base.so, tools/build_base.sh):
# the GPU parity tests of $TESTS with the in-tree library, alternating benches of both builds, a FETCH_SIZE /
# WRITE_SIZE PMC pass of each, and one-stream kernel stats of the new build.
# usage: TESTS="tests/..." tools/gpu_r5_ab4.sh <tag>   (run via gpurun)
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -m gpu \
    ${TESTS:-tests/test_gpu_parity.py} > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
CFGS="new|GS_AB=new;base|DGE_AMD_LIB=$PWD/dge_amd/lib/var/base.so" ROUNDS=${ROUNDS:-3} \
    timeout -k 10 1200 bash tools/gpu_ab_cfg.sh $O/ab > $O/ab.txt 2>&1 || { tail -20 $O/ab.txt; exit 1; }
cat $O/ab.txt
CMD="python bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-profile --no-side-legs"
for v in new base; do
  L=""; [ $v = base ] && L=$PWD/dge_amd/lib/var/base.so
  i=0
  for g in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    DGE_AMD_LIB=$L timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $g -d $O/pmc_$v/p$i -o run --output-format csv -- $CMD \
        > $O/pmc_$v.log 2>&1 || { echo "pmc $v $g failed $?"; tail -5 $O/pmc_$v.log; exit 1; }
  done
  echo "== pmc $v"; python tools/pmc_summary.py $O/pmc_$v 2>&1 | head -20
done
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d $O/prof1 -o one -- python bench.py --streams 1 --steps 10 --warmup 3 --no-cpu-baseline --no-side-legs --no-profile > $O/bench_prof1.log 2> $O/bench_prof1.err || { echo "rocprof failed $?"; tail -20 $O/bench_prof1.err; exit 1; }
S=$(find $O/prof1 -name "*kernel_stats.csv" | head -1)
head -16 $S | cut -d, -f1-6
