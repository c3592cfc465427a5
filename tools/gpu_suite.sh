#!/bin/bash
# GPU suite + smoke only (the first two steps of gpu_full.sh).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-suite}; O=gpurun_out/$TAG; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -2 $O/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; exit $rc
