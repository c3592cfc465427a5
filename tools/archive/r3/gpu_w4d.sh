#!/bin/bash
# Direct-A four-wave GEMM (gemm_w4d.h): GEMM parity tests, then the Q-Former-shape GEMM
# diagnostics and the caption steps with GVL_W4D=1 (default) vs 0, alternated.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-w4d}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "w4 or tile128x192 or dropout_residual" > $O/tests.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
for round in 1 2; do
  for v in 1 0; do
    GVL_W4D=$v timeout -k 10 200 python -u tools/r3/gemm_diag.py > $O/diag_${v}_$round.log 2>&1; rc=$?; fatal $rc diag
    echo "== W4D=$v round $round"; grep "N=" $O/diag_${v}_$round.log | sed -E 's/ +/ /g' | cut -d' ' -f1,5,6
  done
done
for v in 1 0 1 0; do
  GVL_W4D=$v timeout -k 10 300 python bench.py --workload qformer --steps 20 --warmup 5 --no-cpu-baseline > $O/qf_$v.json 2> $O/qf_$v.err; rc=$?; fatal $rc qf
  GVL_W4D=$v timeout -k 10 300 python bench.py --workload cross --steps 20 --warmup 5 --no-cpu-baseline > $O/xa_$v.json 2> $O/xa_$v.err; rc=$?; fatal $rc xa
  python -c "
import json
for w in ('qf','xa'):
    d=json.loads(open('$O/'+w+'_$v.json').read().strip().splitlines()[-1]); print(w, 'W4D=$v', d['value'], d['roofline']['kernel'], d['roofline']['avg_launch_us'])"
done
