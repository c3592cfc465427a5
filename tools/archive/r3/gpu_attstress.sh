#!/bin/bash
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-attstress}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u tools/r3/attn_stress.py 40 > $O/stress.log 2>&1; rc=$?; echo "stress rc=$rc"; tail -5 $O/stress.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py > $O/kernels.log 2>&1; rc=$?; echo "kernels rc=$rc: $(tail -1 $O/kernels.log)"; grep FAILED $O/kernels.log | head
