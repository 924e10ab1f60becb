#!/bin/bash
# one GPU call: the named pytest selection (-k expression or node ids) -> gpurun_out/<tag>/pytest.log
# usage: tools/gpu_test.sh <tag> <pytest args...>
cd "$GRAFT_REPO_ROOT" 2>/dev/null || cd /root/repo
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread -m gpu -p no:cacheprovider "$@" > $O/pytest.log 2>&1
rc=$?
grep -E "parity|PASS|FAIL|Error|passed|failed" $O/pytest.log | tail -40
exit $rc
