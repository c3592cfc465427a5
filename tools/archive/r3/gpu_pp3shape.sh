#!/bin/bash
# Persistent-kernel tile shape on the Q-Former step's wide GEMMs (M = 8064): planner default vs
# forced 256-wide (GVL_PP3_BN=256) vs forced 128-row (GVL_PP3_BM=128) tiles.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-pp3shape}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
for v in def bn256 bm128 def bn256 bm128; do
  case $v in def) E="";; bn256) E="GVL_PP3_BN=256";; bm128) E="GVL_PP3_BM=128";; esac
  env $E timeout -k 10 300 python bench.py --workload qformer --steps 20 --warmup 5 --no-cpu-baseline > $O/qf_$v.json 2> $O/qf_$v.err; fatal $? qf
  python -c "
import json
d=json.loads(open('$O/qf_$v.json').read().strip().splitlines()[-1]); print('qf $v', d['value'], d['ms_per_step'], [(g['kernel'], g['avg_us']) for g in d['roofline']['top_gemms'][2:5]])"
done
