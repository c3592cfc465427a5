#!/bin/bash
# Short-K wide outputs on the four-wave kernel (GVL_W4=3) vs the default pick (GVL_W4=1):
# GEMM parity tests under GVL_W4=3, per-shape timing, Q-Former and LM bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-a}
O=gpurun_out/w4s_$TAG; mkdir -p $O
GVL_W4=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gemm and not tile192 and not tile128x192 and not bias_dropout_residual" > $O/tests.log 2>&1 || exit $?
for spec in "8064 2304 768 0 0" "8064 3072 768 0 0" "8064 3072 768 0 1" "16384 2304 768 0 0" "16384 3072 768 0 0" "16384 3072 768 0 1"; do
  for w in 1 3; do
    GVL_W4=$w timeout -k 10 60 python tools/gemm_one.py $spec 3 -1 50 2>/dev/null | sed "s/^/w4=$w /" >> $O/shapes.txt || exit $?
  done
done
for w in 1 3 1 3; do
  GVL_W4=$w timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_$w.json 2>> $O/qf.err || exit $?
  tail -1 $O/qf_$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('qf w4=$w', d['value'], d['ms_per_step'])" >> $O/shapes.txt
done
for w in 1 3; do
  GVL_W4=$w timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$w.json 2>> $O/lm.err || exit $?
  tail -1 $O/lm_$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lm w4=$w', d['value'], d['ms_per_step'])" >> $O/shapes.txt
done
