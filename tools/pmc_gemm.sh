#!/bin/bash
# PMC passes (kernel-trace only, no sys/runtime trace) over single-GEMM runs.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}; shift
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE"
i=0
for spec in "$@"; do
  i=$((i+1))
  for pn in 1 2 3; do
    eval "CTRS=\$P$pn"
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $OUT/c${i}_p$pn -o run -- python tools/gemm_one.py $spec 5 ${EPI:-plain} > $OUT/c${i}_p$pn.log 2>&1 || exit $?
  done
  timeout -k 10 120 python tools/gemm_one.py $spec 20 ${EPI:-plain} >> $OUT/times.log 2>&1 || exit $?
done
