#!/bin/bash
# GEMM timing sweep over L2 group sizes and kernel configs (single process per setting)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
OUT=gpurun_out/sweep_$TAG.log; : > $OUT
for grp in 1 4 8 16; do
  for spec in "8192 8192 8192 0 0" "16384 2304 768 0 0" "16384 3072 768 0 0" "16384 768 3072 0 1" "16384 50304 768 0 0" "8064 2304 768 0 0" "8064 768 3072 0 0"; do
    for ic in "1 0" "1 2" "2 2" "2 4"; do
      echo -n "group=$grp " >> $OUT
      GVL_GEMM_GROUP=$grp timeout -k 10 60 python tools/gemm_one.py $spec $ic 10 2>/dev/null >> $OUT || exit $?
    done
  done
done
for spec in "8192 8192 8192 0 0" "16384 2304 768 0 0" "16384 3072 768 0 0" "16384 768 3072 0 1" "16384 50304 768 0 0" "8064 2304 768 0 0" "8064 768 3072 0 0"; do
  timeout -k 10 60 python tools/gemm_one.py $spec 3 -1 10 2>/dev/null >> $OUT || exit $?
done
