#!/bin/bash
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-ggrp2}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
for v in 8 4 2 8 4 2 8 4; do
  GVL_GEMM_GROUP=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$v.json 2> $O/lm_$v.err; fatal $? lm
  python -c "
import json
d=json.loads(open('$O/lm_$v.json').read().strip().splitlines()[-1]); print('lm GROUP=$v', d['value'], d['ms_per_step'])"
done
