#!/bin/bash
# 128-row four-wave tiles for the linear caption decoder's 8192-row N = 768 GEMMs (192-row tiles
# overflow one round: 258): GEMM + linear-model parity tests, shape timing, linear bench A/B
# (GVL_W4=4 turns the partial-fill / overflow routes off).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-a}
O=gpurun_out/w4l_$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gemm" > $O/tests_gemm.log 2>&1 || exit $?
timeout -k 10 400 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_parity_full.py tests/test_gpu_graph.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "linear or edge or cls" > $O/tests_models.log 2>&1 || exit $?
for spec in "8192 768 3072 0 0" "8192 768 768 0 0" "8192 768 3072 0 1" "8192 768 2304 0 1"; do
  for w in 1 4; do
    GVL_W4=$w timeout -k 10 60 python tools/gemm_one.py $spec 3 -1 50 2>/dev/null | sed "s/^/w4=$w /" >> $O/shapes.txt || exit $?
  done
done
for w in 1 4 1 4; do
  GVL_W4=$w timeout -k 10 300 python bench.py --workload linear --steps 10 --warmup 3 --no-cpu-baseline > $O/lin_$w.json 2>> $O/bench.err || exit $?
  tail -1 $O/lin_$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('linear w4=$w', d['value'], d['ms_per_step'])" >> $O/summary.txt
done
