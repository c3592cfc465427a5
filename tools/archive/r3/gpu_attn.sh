#!/bin/bash
# attention v2 forward: tests with the default library, then timing A/B against the old forward
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-attn}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "attention or attn" > $O/tests.log 2>&1; rc=$?; echo "tests rc=$rc: $(tail -1 $O/tests.log)"; fatal $rc tests
grep -E "^FAILED|Error" $O/tests.log | head
for round in 1 2; do
  for v in base av0; do
    L=gpt2-vision-language_amd/gvl/libgvl_$v.so; [ "$v" = base ] && L=gpt2-vision-language_amd/gvl/libgvl.so
    GVL_LIB=$L timeout -k 10 200 python -u tools/attn_one.py 20 > $O/t_${v}_$round.log 2>&1; rc=$?; fatal $rc attn_$v
    echo "== $v $round"; grep "fwd" $O/t_${v}_$round.log | sed 's/causal=//; s/drop=//'
  done
done
