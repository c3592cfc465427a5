#!/bin/bash
# dQ kernel computing D = rowsum(dO * O) itself (no attn_bwd_pre_kernel): attention + model
# parity tests, then the LM step (GVL_DQ_DMA=0 restores pre + register-staged dQ: not an A/B of
# this change alone, so the comparison is against the previous commit's numbers on record).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-attnD}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest -q -x --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "attention or attn" tests/test_gpu_parity_full.py tests/test_gpu_parity_bench.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$i.json 2> $O/lm_$i.err; rc=$?; fatal $rc lm
  python -c "
import json
d=json.loads(open('$O/lm_$i.json').read().strip().splitlines()[-1]); print('lm', d['value'], d['ms_per_step'], d['loss'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lm -o lm -- \
  python bench.py --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > $O/prof_lm.json 2> $O/prof_lm.err; rc=$?; fatal $rc prof_lm
f=$(find $O/prof_lm -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 30 > $O/lm_table.txt; grep -E "attn|emb_" $O/lm_table.txt
