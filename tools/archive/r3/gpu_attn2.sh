#!/bin/bash
# dK/dV on the LDS-DMA kernel with 32 keys per wave (G = 2): attention tests, timing vs
# GVL_DKDV_G=1; the G = 4 forward at 2 blocks per CU (libgvl_g4o2) vs the shipped G = 2 forward.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-attn2}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "attention" > $O/tests.log 2>&1; rc=$?; echo "attention tests rc=$rc: $(tail -1 $O/tests.log)"
[ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head; exit $rc; }
L=gpt2-vision-language_amd/gvl/libgvl_g4o2.so
GVL_LIB=$L GVL_ATTN_FWD_G=4 timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "attention" > $O/tests_g4.log 2>&1; rc=$?; echo "g4o2 attention tests rc=$rc: $(tail -1 $O/tests_g4.log)"; fatal $rc tests_g4
for round in 1 2; do
  timeout -k 10 120 python -u tools/attn_one.py 20 > $O/g2_$round.log 2>&1; fatal $? g2
  GVL_DKDV_G=1 timeout -k 10 120 python -u tools/attn_one.py 20 > $O/g1_$round.log 2>&1; fatal $? g1
  GVL_LIB=$L GVL_ATTN_FWD_G=4 timeout -k 10 120 python -u tools/attn_one.py 20 > $O/g4_$round.log 2>&1; fatal $? g4
  echo "round $round dkdv G=2: $(grep -m1 1024 $O/g2_$round.log)"
  echo "round $round dkdv G=1: $(grep -m1 1024 $O/g1_$round.log)"
  echo "round $round fwd G=4 (old bwd): $(grep -m1 1024 $O/g4_$round.log)"
done
