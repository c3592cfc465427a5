#!/bin/bash
# Round-2 late session: short-K four-wave A/B, cross-att GEMM shape table, PMC traffic passes.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-a}
bash tools/gpu_w4s.sh $TAG || exit $?
timeout -k 10 200 python tools/gemm_shapes.py xa 3:-1,3:10,2:-1 > gpurun_out/xa_shapes_$TAG.txt 2>&1 || exit $?
bash tools/pmc_traffic.sh r2h
