#!/bin/bash
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-ggrp4}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
W=gpt2-vision-language_amd/gvl/libgvl_wr2.so
for v in base rule2 env4 base rule2 env4; do
  case $v in base) E="";; rule2) E="GVL_LIB=$W";; env4) E="GVL_GEMM_GROUP=4";; esac
  env $E timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$v.json 2> $O/lm_$v.err; fatal $? lm
  python -c "
import json
d=json.loads(open('$O/lm_$v.json').read().strip().splitlines()[-1]); print('lm $v', d['value'], d['ms_per_step'])"
done
for v in base rule2 base rule2; do
  case $v in base) E="";; rule2) E="GVL_LIB=$W";; esac
  env $E timeout -k 10 300 python bench.py --workload qformer --steps 20 --warmup 5 --no-cpu-baseline > $O/qf_$v.json 2> $O/qf_$v.err; fatal $? qf
  python -c "
import json
d=json.loads(open('$O/qf_$v.json').read().strip().splitlines()[-1]); print('qf $v', d['value'], d['ms_per_step'])"
done
