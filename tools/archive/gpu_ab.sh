#!/bin/bash
# A/B of a GEMM tile rule on the caption step: GEMM kernel parity first, then the Q-Former
# caption bench with GVL_RING_SMALLunset (128x128), =6 (64x128) and =1 (256x128).
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k gemm --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/ab_tests_$TAG.log 2>&1 || exit $?
for v in 0 6 1; do
  GVL_RING_SMALL=$v timeout -k 10 200 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_qf_${TAG}_$v.json 2> gpurun_out/ab_qf_${TAG}_$v.err || exit $?
done
for w in linear cross; do
  timeout -k 10 200 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_${w}_${TAG}.json 2> gpurun_out/ab_${w}_${TAG}.err || exit $?
done
