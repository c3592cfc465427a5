#!/bin/bash
# Tile walk of the 128-row four-wave kernel (gemm_w4m): GVL_W4_GROUP=1 vs the default group.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-w4mgrp}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
for v in 0 1 0 1; do
  for w in cross qformer; do
    GVL_W4_GROUP=$v timeout -k 10 300 python bench.py --workload $w --steps 20 --warmup 5 --no-cpu-baseline > $O/${w}_$v.json 2> $O/${w}_$v.err; fatal $? $w
    python -c "
import json
d=json.loads(open('$O/${w}_$v.json').read().strip().splitlines()[-1]); print('$w W4_GROUP=$v', d['value'], d['ms_per_step'])"
  done
done
