#!/bin/bash
# A/B of w4 kernel variants: correctness (w4 GEMM tests) then the Q-Former GEMM diagnostics,
# interleaved by library.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-w4ab}; O=gpurun_out/$TAG; mkdir -p $O
shift
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
for v in "$@"; do
  L=gpt2-vision-language_amd/gvl/libgvl_$v.so; [ "$v" = base ] && L=gpt2-vision-language_amd/gvl/libgvl.so
  GVL_LIB=$L timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_kernels.py -k "w4" > $O/tests_$v.log 2>&1; rc=$?; echo "$v tests rc=$rc: $(tail -1 $O/tests_$v.log)"; fatal $rc tests_$v
done
for round in 1 2; do
  for v in "$@"; do
    L=gpt2-vision-language_amd/gvl/libgvl_$v.so; [ "$v" = base ] && L=gpt2-vision-language_amd/gvl/libgvl.so
    GVL_LIB=$L timeout -k 10 200 python -u tools/r3/gemm_diag.py > $O/diag_${v}_$round.log 2>&1; rc=$?; fatal $rc diag_$v
    echo "== $v round $round"; grep "N=" $O/diag_${v}_$round.log | awk '{print $1, $4, $5}'
  done
done
