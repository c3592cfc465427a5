#!/bin/bash
# ring GEMM: correctness probe + kernel tests under the ring impl
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
PROBE_ONLY_RING=1 timeout -k 10 300 python tools/gpu_probe_gemm.py > gpurun_out/probe_$TAG.log 2>&1 || exit $?
GVL_GEMM_IMPL=ring timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -rf -p no:cacheprovider > gpurun_out/kern_$TAG.log 2>&1 || exit $?
GVL_GEMM_IMPL=ring GVL_GEMM_CFG=4 timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -rf -p no:cacheprovider -k gemm > gpurun_out/kern_pp_$TAG.log 2>&1
