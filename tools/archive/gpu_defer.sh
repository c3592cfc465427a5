# Deferred + batched weight gradients: GEMM/model/graph/full-parity tests, LM + Q-Former bench A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-a}
O=gpurun_out/defer_$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py tests/test_gpu_graph.py tests/test_gpu_parity_full.py tests/test_gpu_boundary.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gemm or colsum or models or graph or parity or boundary or ddp or accum or train" > $O/tests.log 2>&1 || exit $?
for d in 1 0 1; do
  GVL_DEFER_WGRAD=$d timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$d.json 2>> $O/bench.err || exit $?
  tail -1 $O/lm_$d.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lm defer=$d', d['value'], d['ms_per_step'])" >> $O/summary.txt
done
for d in 1 0 1; do
  GVL_DEFER_WGRAD=$d timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_$d.json 2>> $O/bench.err || exit $?
  tail -1 $O/qf_$d.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('qf defer=$d', d['value'], d['ms_per_step'])" >> $O/summary.txt
done
