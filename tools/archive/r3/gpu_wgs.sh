#!/bin/bash
# Concurrent batched weight-gradient launches (GVL_WGRAD_STREAMS): deferral / DP / parity
# tests, then the LM step with the side streams on and off, alternated.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-wgs}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py tests/test_gpu_parity_bench.py tests/test_gpu_dp.py tests/test_gpu_parity_full.py tests/test_gpu_boundary.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
for v in 1 0 1 0; do
  GVL_WGRAD_STREAMS=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$v.json 2> $O/lm_$v.err; rc=$?; fatal $rc lm
  python -c "
import json
d=json.loads(open('$O/lm_$v.json').read().strip().splitlines()[-1]); print('lm WGRAD_STREAMS=$v', d['value'], d['ms_per_step'], d['loss'])"
done
