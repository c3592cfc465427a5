# 128x192 persistent tiles: GEMM parity, per-shape A/B (GVL_PP3_BM=256 vs planner), Q-Former bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-b}
O=gpurun_out/bm128_$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gemm" > $O/tests.log 2>&1 || exit $?
for spec in "8064 768 3072 0 0" "8064 768 3072 0 1" "8064 768 768 0 0" "8064 768 768 0 1" "8064 768 2304 0 1" "8064 2304 768 0 0" "8064 3072 768 0 0" "8064 3072 768 0 1" "16384 768 3072 0 0" "16384 2304 768 0 0"; do
  for bm in 0 256; do
    GVL_PP3_BM=$bm timeout -k 10 60 python tools/gemm_one.py $spec 3 -1 50 2>/dev/null | sed "s/^/bm=$bm /" >> $O/shapes.txt || exit $?
  done
done
for bm in 0 256 0; do
  GVL_PP3_BM=$bm timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_$bm.json 2>> $O/qf.err || exit $?
  tail -1 $O/qf_$bm.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bm=$bm', d['value'], d['ms_per_step'])" >> $O/shapes.txt
done
