#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
GVL_GEMM_CFG=6 timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -rf -p no:cacheprovider -k gemm > gpurun_out/kern_$TAG.log 2>&1 || exit $?
OUT=gpurun_out/sweep_$TAG.log; : > $OUT
for spec in "8192 8192 8192 0 0" "16384 2304 768 0 0" "16384 3072 768 0 0" "16384 3072 768 0 1" "16384 50304 768 0 0" "8064 50304 768 0 0" "50304 768 16384 1 1" "4096 4096 4096 0 0"; do
  for ic in "2 4" "2 6"; do
    timeout -k 10 60 python tools/gemm_one.py $spec $ic 10 2>/dev/null >> $OUT || exit $?
  done
done
