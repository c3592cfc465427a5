# New epilogue / LN-residual tests + Q-Former and LM bench (default lib)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-a}
O=gpurun_out/step2_$TAG; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "dropout or layernorm or w4 or tile128 or qformer or caption or cross" > $O/tests.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf.json 2>> $O/bench.err || exit $?
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm.json 2>> $O/bench.err || exit $?
for f in qf lm; do tail -1 $O/$f.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$f', d['value'], d['ms_per_step'])" >> $O/summary.txt; done
