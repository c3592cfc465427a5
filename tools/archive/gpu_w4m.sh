#!/bin/bash
# 128-row four-wave tiles (gemm_w4m_kernel) where 192-row tiles fill < 3/4 of the CUs:
# GEMM parity tests, cross-att / Q-Former model tests, shape table, cross + Q-Former bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-a}
O=gpurun_out/w4m_$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gemm" > $O/tests_gemm.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_parity_full.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "cross or qformer" > $O/tests_models.log 2>&1 || exit $?
timeout -k 10 200 python tools/gemm_shapes.py xa 3:-1,2:-1 > $O/xa_shapes.txt 2>&1 || exit $?
for w in 1 0 1 0; do
  GVL_W4_BM128=$w timeout -k 10 300 python bench.py --workload cross --steps 10 --warmup 3 --no-cpu-baseline > $O/cross_$w.json 2>> $O/bench.err || exit $?
  tail -1 $O/cross_$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cross bm128=$w', d['value'], d['ms_per_step'])" >> $O/summary.txt
  GVL_W4_BM128=$w timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_$w.json 2>> $O/bench.err || exit $?
  tail -1 $O/qf_$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('qformer bm128=$w', d['value'], d['ms_per_step'])" >> $O/summary.txt
done
