# In-launch split-K combine: parity tests, per-shape A/B (GVL_PP3_COMBINE=0|1), Q-Former bench A/B.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-c}
O=gpurun_out/combine_$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "combined_in_launch or ring_band or tile192 or splitk_epilogue or wgrad or persistent_epilogues" > $O/tests.log 2>&1 || exit $?
for spec in "8064 768 3072 0 0" "8064 768 3072 0 1" "8064 768 768 0 0" "8064 768 768 0 1" "8064 768 2304 0 1" "16384 768 3072 0 0"; do
  for c in 0 1; do
    GVL_PP3_COMBINE=$c timeout -k 10 60 python tools/gemm_one.py $spec 3 -1 50 2>/dev/null | sed "s/^/combine=$c /" >> $O/shapes.txt || exit $?
  done
done
for c in 1 0 1; do
  GVL_PP3_COMBINE=$c timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_$c.json 2>> $O/qf.err || exit $?
  tail -1 $O/qf_$c.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('combine=$c', d['value'], d['ms_per_step'])" >> $O/shapes.txt
done
