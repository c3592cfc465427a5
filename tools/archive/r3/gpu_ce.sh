#!/bin/bash
# Cross-entropy with 1024 threads per row (libgvl_ce1024) vs 512: CE tests, then the LM step
# alternated.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-ce}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
L=gpt2-vision-language_amd/gvl/libgvl_ce1024.so
GVL_LIB=$L timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "cross_entropy or ce_" > $O/tests.log 2>&1; rc=$?; echo "ce1024 tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && exit $rc
for v in base ce1024 base ce1024; do
  LL=gpt2-vision-language_amd/gvl/libgvl.so; [ $v = ce1024 ] && LL=$L
  GVL_LIB=$LL timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$v.json 2> $O/lm_$v.err; fatal $? lm
  python -c "
import json
d=json.loads(open('$O/lm_$v.json').read().strip().splitlines()[-1]); print('lm $v', d['value'], d['ms_per_step'], d['loss'])"
done
