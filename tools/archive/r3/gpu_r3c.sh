#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r3c}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 300 python -u tools/r3/dbg_dp.py > $O/dbg_dp.log 2>&1; rc=$?; echo "dbg rc=$rc"; grep variant $O/dbg_dp.log | cut -c1-300; fatal $rc dbg
timeout -k 10 600 python -u -m pytest -v -s -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_dp.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; grep -E "PASSED|FAILED|Error|DP loss|buckets per" $O/tests.log | head -20; fatal $rc tests
