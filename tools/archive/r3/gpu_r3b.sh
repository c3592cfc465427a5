#!/bin/bash
# DP debug, Q-Former GEMM diagnostics + PMC, then the round-3 tests again.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r3b}; O=gpurun_out/$TAG; mkdir -p $O
export GVL_MARGINS_DIR=$O/parity_margins
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 300 python -u tools/r3/dbg_dp.py > $O/dbg_dp.log 2>&1; rc=$?; echo "dbg rc=$rc"; grep variant $O/dbg_dp.log; fatal $rc dbg
timeout -k 10 300 python -u tools/r3/gemm_diag.py > $O/gemm_diag.log 2>&1; rc=$?; echo "diag rc=$rc"; cat $O/gemm_diag.log | tail -9; fatal $rc diag
bash tools/r3/pmc_qf.sh $TAG > $O/pmc.log 2>&1; rc=$?; echo "pmc rc=$rc"; fatal $rc pmc
timeout -k 10 900 python -u -m pytest -v -s -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity_bench.py tests/test_gpu_boundary.py tests/test_gpu_parity_full.py > $O/tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/tests.log; fatal $rc tests
