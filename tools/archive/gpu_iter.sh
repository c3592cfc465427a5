#!/bin/bash
# quick GPU iteration: kernel tests, attention timing, GEMM PMC passes
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -rf -p no:cacheprovider > gpurun_out/kern_$TAG.log 2>&1 || exit $?
timeout -k 10 120 python tools/attn_one.py > gpurun_out/attn_$TAG.log 2>&1 || exit $?
bash tools/pmc_gemm.sh $TAG "8192 8192 8192 0 0 1 0" "8192 8192 8192 0 0 2 4" "8192 8192 8192 0 0 3 -1" "8192 8192 8192 0 0 2 0"
