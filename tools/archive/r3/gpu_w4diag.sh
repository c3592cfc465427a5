#!/bin/bash
# timing-only diagnostic builds of the w4 kernel (wrong results): no barrier (d1), no LDS
# writes + no global loads (d2) vs the shipped kernel
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-w4d}; O=gpurun_out/$TAG; mkdir -p $O
shift
for round in 1 2; do
  for v in "$@"; do
    L=gpt2-vision-language_amd/gvl/libgvl_$v.so; [ "$v" = base ] && L=gpt2-vision-language_amd/gvl/libgvl.so
    GVL_LIB=$L timeout -k 10 200 python -u tools/r3/gemm_diag.py > $O/diag_${v}_$round.log 2>&1 || exit $?
    echo "== $v round $round"; grep "N=" $O/diag_${v}_$round.log | sed 's/  */ /g' | awk '{print $1, $6}'
  done
done
