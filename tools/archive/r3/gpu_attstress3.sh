#!/bin/bash
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-attstress3}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 300 python -u tools/r3/attn_stress.py 60 > $O/stress.log 2>&1; rc=$?
echo "stress rc=$rc: $(grep -c BAD $O/stress.log) bad; $(tail -1 $O/stress.log)"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "attention or attn" > $O/tests.log 2>&1; rc=$?; echo "attention tests rc=$rc: $(tail -1 $O/tests.log)"
exit $rc
