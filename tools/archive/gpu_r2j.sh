#!/bin/bash
# Round-2 closing run: full confirmation (tests, bench, smoke, rocprof), then the four-wave
# tile-walk A/B (GVL_W4_GROUP=1: all column tiles of a row block on one XCD).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r2j}
bash tools/gpu_final.sh $TAG || exit $?
O=gpurun_out/grp_$TAG; mkdir -p $O
for g in 1 0 1 0; do
  for w in qformer cross; do
    GVL_W4_GROUP=$g timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/${w}_$g.json 2>> $O/bench.err || exit $?
    tail -1 $O/${w}_$g.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$w group=$g', d['value'], d['ms_per_step'])" >> $O/summary.txt
  done
done
