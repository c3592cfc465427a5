#!/bin/bash
# PMC passes over the Q-Former decoder GEMM shapes (M = 8064) with their model epilogues:
# one rocprofv3 --kernel-trace --pmc pass per counter group, each time-limited.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
OUT=gpurun_out/pmc_$TAG; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
SPECS=("8064 3072 768 0 0 3 -1 20 act" "8064 2304 768 0 0 3 -1 20 bias" "8064 768 3072 0 0 3 -1 20 bias_res"
       "8064 768 2304 0 1 3 -1 20 plain" "8064 3072 768 0 1 3 -1 20 dact" "8064 768 768 0 1 3 -1 20 plain")
i=0
for spec in "${SPECS[@]}"; do
  i=$((i+1))
  timeout -k 10 120 python tools/gemm_one.py $spec >> $OUT/times.log 2>&1 || exit $?
  for pn in 1 2 3 4; do
    eval "CTRS=\$P$pn"
    timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $OUT/c${i}_p$pn -o run -- python tools/gemm_one.py $spec > $OUT/c${i}_p$pn.log 2>&1 || exit $?
  done
done
