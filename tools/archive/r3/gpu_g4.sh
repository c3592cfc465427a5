#!/bin/bash
# G = 4 forward compiled for 2 blocks per CU (libgvl_g4o2) vs the shipped G = 2 forward, then
# the attention PMC passes of the shipped build.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-g4}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
L=gpt2-vision-language_amd/gvl/libgvl_g4o2.so
GVL_LIB=$L GVL_ATTN_FWD_G=4 timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "attention" > $O/tests.log 2>&1; rc=$?; echo "g4o2 attention tests rc=$rc: $(tail -1 $O/tests.log)"; fatal $rc tests
for round in 1 2; do
  timeout -k 10 120 python -u tools/attn_one.py 20 > $O/base_$round.log 2>&1; fatal $? base
  GVL_LIB=$L GVL_ATTN_FWD_G=4 timeout -k 10 120 python -u tools/attn_one.py 20 > $O/g4_$round.log 2>&1; fatal $? g4
  echo "round $round base: $(grep -m1 1024 $O/base_$round.log)"; echo "round $round g4o2: $(grep -m1 1024 $O/g4_$round.log)"
done
bash tools/pmc_attn.sh r3 || exit $?
echo pmc done
