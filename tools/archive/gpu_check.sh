#!/bin/bash
# GPU tests + GEMM shape table (each step time-limited; stop at the first failure)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/gemm_shapes.py all -1,4,2,0 > gpurun_out/gemm_shapes_$TAG.log 2>&1
