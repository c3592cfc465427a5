#!/bin/bash
# train_step seeding backward with a cached 1/accum scalar: model-level parity / DP / graph
# tests, then the Q-Former and LM bench steps.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-seed}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 700 python -u -m pytest -q -x --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity_full.py tests/test_gpu_parity_bench.py tests/test_gpu_dp.py tests/test_gpu_boundary.py \
  tests/test_gpu_decode.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --workload qformer --steps 20 --warmup 5 --no-cpu-baseline > $O/qf.json 2> $O/qf.err; fatal $? qf
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm.json 2> $O/lm.err; fatal $? lm
for w in qf lm; do python -c "
import json
d=json.loads(open('$O/$w.json').read().strip().splitlines()[-1]); print('$w', d['value'], d['ms_per_step'], d['loss'])"; done
