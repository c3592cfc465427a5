#!/bin/bash
# PMC passes over the attention timing script (kernel-trace + counters only)
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
OUT=gpurun_out/pmca_$TAG; mkdir -p $OUT
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU"
P2="GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM"
for pn in 1 2; do
  eval "CTRS=\$P$pn"
  timeout -k 10 120 rocprofv3 --kernel-trace --pmc $CTRS --output-format csv -d $OUT/p$pn -o run -- python tools/attn_one.py 3 > $OUT/p$pn.log 2>&1 || exit $?
done
