#!/bin/bash
# LayerNorm forward with gamma/beta prefetched + 4-waves/SIMD short attention forward, against
# the previous build (gvl/libgvl_base.so via GVL_LIB): attention / LN / model tests, bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-a}
O=gpurun_out/lnattn_$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "attn or layernorm or ln_ or models or qformer or cross" > $O/tests.log 2>&1 || exit $?
B=gpt2-vision-language_amd/gvl/libgvl_base.so
for v in new base new base; do
  if [ $v = base ]; then export GVL_LIB=$R/$B; else unset GVL_LIB; fi
  timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_$v.json 2>> $O/bench.err || exit $?
  tail -1 $O/qf_$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('qformer $v', d['value'], d['ms_per_step'])" >> $O/summary.txt
done
for v in new base; do
  if [ $v = base ]; then export GVL_LIB=$R/$B; else unset GVL_LIB; fi
  timeout -k 10 400 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$v.json 2>> $O/bench.err || exit $?
  tail -1 $O/lm_$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lm $v', d['value'], d['ms_per_step'])" >> $O/summary.txt
done
