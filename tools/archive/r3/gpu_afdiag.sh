#!/bin/bash
# Attention forward timing-only builds (af0 shipped, af1 no exp, af2 no K/V loads, af3 no
# barrier), then the full parity set of the shipped library (fused D in the dQ kernel).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-afdiag}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
for round in 1 2; do
  for v in af0 af1 af2 af3; do
    GVL_LIB=gpt2-vision-language_amd/gvl/libgvl_$v.so timeout -k 10 120 python -u tools/attn_one.py 20 > $O/${v}_$round.log 2>&1; rc=$?; fatal $rc $v
    echo "== $v round $round: $(grep -m1 '1024' $O/${v}_$round.log)"
  done
done
timeout -k 10 700 python -u -m pytest -q -x --timeout 200 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity_full.py tests/test_gpu_parity_bench.py tests/test_gpu_decode.py > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && grep -E "FAIL|Error|assert" $O/tests.log | head -20
exit $rc
