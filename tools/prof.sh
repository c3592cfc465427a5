#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench workloads (run on the GPU box via gpurun).
# Each profiled run has its own time limit; the script stops at the first failing step.
set -e
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
TAG=${1:-r1}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_qf_$TAG" -o qf -- \
  python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > "gpurun_out/prof_qf_$TAG.json" 2> "gpurun_out/prof_qf_$TAG.err"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_lm_$TAG" -o lm -- \
  python bench.py --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > "gpurun_out/prof_lm_$TAG.json" 2> "gpurun_out/prof_lm_$TAG.err"
