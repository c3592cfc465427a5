#!/bin/bash
# Cross-att kv_proj batched over the 12 blocks (Fn.CrossKVFn, GVL_XKV_BATCH=1) vs per-block:
# model / full-size / graph / boundary tests touching the cross-att model, then bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-a}
O=gpurun_out/xkv_$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gemm" > $O/tests_gemm.log 2>&1 || exit $?
timeout -k 10 500 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_parity_full.py tests/test_gpu_graph.py tests/test_gpu_boundary.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "cross" > $O/tests.log 2>&1 || exit $?
for x in 1 0 1 0; do
  GVL_XKV_BATCH=$x timeout -k 10 300 python bench.py --workload cross --steps 10 --warmup 3 --no-cpu-baseline > $O/cross_$x.json 2>> $O/bench.err || exit $?
  tail -1 $O/cross_$x.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cross xkv=$x', d['value'], d['ms_per_step'])" >> $O/summary.txt
done
for w in 1 4 1 4; do
  GVL_W4=$w timeout -k 10 300 python bench.py --workload cross --steps 10 --warmup 3 --no-cpu-baseline > $O/cross_w4_$w.json 2>> $O/bench.err || exit $?
  tail -1 $O/cross_w4_$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cross w4=$w', d['value'], d['ms_per_step'])" >> $O/summary.txt
done
timeout -k 10 200 python tools/gemm_shapes.py xa 3:-1,3:11,2:-1 > $O/xa_shapes.txt 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf.json 2>> $O/bench.err || exit $?
tail -1 $O/qf.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('qformer', d['value'], d['ms_per_step'])" >> $O/summary.txt
