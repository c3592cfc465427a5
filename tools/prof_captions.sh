#!/bin/bash
# rocprofv3 kernel-trace + stats of the linear and cross-att caption steps (bench workloads).
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
for w in cross linear; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_${w}_$TAG" -o $w -- \
    python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > "gpurun_out/prof_${w}_$TAG.json" 2> "gpurun_out/prof_${w}_$TAG.err"
done
