#!/bin/bash
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-attstress2}; O=gpurun_out/$TAG; mkdir -p $O
for v in prev cur; do
  L=gpt2-vision-language_amd/gvl/libgvl.so; [ $v = prev ] && L=gpt2-vision-language_amd/gvl/libgvl_attprev.so
  GVL_LIB=$L timeout -k 10 300 python -u tools/r3/attn_stress.py 40 > $O/stress_$v.log 2>&1; rc=$?
  echo "$v rc=$rc: $(grep -c BAD $O/stress_$v.log) bad; $(tail -1 $O/stress_$v.log)"; [ $rc -ne 0 ] && exit $rc
done
exit 0
