#!/bin/bash
# Batched weight gradients with the two-way in-launch K split (GVL_BATCHED_SPLIT): parity of
# the batched tests and the bench-shape model steps, then the LM step alternated 1 / 0.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-bsplit}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "batched" tests/test_gpu_parity_bench.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
show() { python -c "
import json
d=json.loads(open('$1').read().strip().splitlines()[-1]); r=d['roofline']
print('$2', d['value'], d['ms_per_step'], d['loss'], [(g['kernel'], g['launches_per_step'], g['avg_us']) for g in r['top_gemms'] if 'true, true' in g['kernel']])"; }
for v in 1 0 1 0; do
  GVL_BATCHED_SPLIT=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$v.json 2> $O/lm_$v.err; fatal $? lm; [ -s $O/lm_$v.json ] || exit 1
  show $O/lm_$v.json "LM SPLIT=$v"
done
