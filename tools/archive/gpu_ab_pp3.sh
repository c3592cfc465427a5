#!/bin/bash
# A/B of the persistent-kernel work-item floor (GVL_PP3_MIN) on the LM step (no graph capture
# change: the same shapes route to the 256x256 persistent kernel instead of the 128x128 ring).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
for v in 160 96 48; do
  GVL_PP3_MIN=$v timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --caption-steps 10 > gpurun_out/abpp3_${TAG}_$v.json 2> gpurun_out/abpp3_${TAG}_$v.err || exit $?
done
