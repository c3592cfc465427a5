#!/bin/bash
# Timing-only w4d diagnostic builds (tools/r3/build_variant2.sh): base / no A loads / no B
# staging / no barrier, N = 768 shapes of the Q-Former step, two interleaved rounds.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-wdiag}; O=gpurun_out/$TAG; mkdir -p $O
shift
for round in 1 2; do
  for v in "$@"; do
    GVL_LIB=gpt2-vision-language_amd/gvl/libgvl_$v.so timeout -k 10 200 python -u tools/r3/gemm_diag.py > $O/diag_${v}_$round.log 2>&1 || exit $?
    echo "== $v round $round"; grep "N=  768" $O/diag_${v}_$round.log | sed -E 's/ +/ /g' | cut -d' ' -f1,5,6,7
  done
done
