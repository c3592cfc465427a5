#!/bin/bash
# Round-2 closing run: full confirmation of the head (tests, bench, smoke, rocprof), then A/B of
# the head against the previous build (LN gamma/beta prefetch + short attention occupancy) and
# the four-wave tile-walk knob.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r2k}
bash tools/gpu_final.sh $TAG || exit $?
bash tools/gpu_lnattn.sh $TAG || exit $?
O=gpurun_out/grp_$TAG; mkdir -p $O
for g in 1 0; do
  for w in qformer cross; do
    GVL_W4_GROUP=$g timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/${w}_$g.json 2>> $O/bench.err || exit $?
    tail -1 $O/${w}_$g.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w group=$g', d['value'], d['ms_per_step'])" >> $O/summary.txt
  done
done
