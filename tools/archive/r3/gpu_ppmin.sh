#!/bin/bash
# Persistent-kernel work-item floor (GVL_PP3_MIN, default 160) on the caption steps: which of
# the bridge's small GEMMs leave the split-K 128x128 ring for the persistent kernel.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-ppmin}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
for v in 160 64 96 160 64 96; do
  for w in qformer cross; do
    GVL_PP3_MIN=$v timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/${w}_$v.json 2> $O/${w}_$v.err; fatal $? $w
    python -c "
import json
d=json.loads(open('$O/${w}_$v.json').read().strip().splitlines()[-1]); print('$w MIN=$v', d['value'], d['ms_per_step'])"
  done
done
