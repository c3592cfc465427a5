#!/bin/bash
# Round-4 GPU sessions (run on the GPU box through gpurun): bash tools/r4_sessions.sh <name>.
# Every GPU step has its own time limit; a session stops at the first failing step.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; S=${1:?session}; O=gpurun_out/$S; mkdir -p $O
LIBDIR=gpt2-vision-language_amd/gvl
fatal() { [ "$1" -eq 0 ] || { echo "fatal rc $1 at $2"; exit $1; }; }
suite() {  # GPU suite (margins recorded) + smoke
  GVL_MARGINS_DIR=$O/parity_margins timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log; fatal $rc suite
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; fatal $rc smoke
}
diag() {  # diag <lib-suffix|base> <M> <set> <cols>
  local L=$LIBDIR/libgvl_$1.so; [ "$1" = base ] && L=$LIBDIR/libgvl.so
  GVL_LIB=$L GVL_DIAG_COLS=$4 timeout -k 10 240 python -u tools/gemm_diag.py $2 $3 > $O/diag_$1_$2_$3.log 2>&1
  rc=$?; echo "== $1 M=$2 $3"; cat $O/diag_$1_$2_$3.log | grep "N=" ; fatal $rc diag
}
case $S in
r4a)  # HEAD check + epilogue share of the short-K wide GEMMs (timing-only pp3 builds)
  suite
  diag base 8064 all all
  diag base 16384 wide all
  for v in pp3d1 pp3d2 base; do diag $v 8064 wide epi; diag $v 16384 wide epi; done
  ;;
*) echo "unknown session $S"; exit 2;;
esac
