# Four-wave 192x128 deep-ring GEMM (gemm_w4.hip): parity tests, per-shape timing next to the
# previous default and hipBLASLt, Q-Former bench A/B (GVL_W4=0|1).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-a}
O=gpurun_out/w4_$TAG; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "test_gemm_w4 or tile128x192" > $O/tests.log 2>&1 || exit $?
for spec in "8064 768 3072 0 0" "8064 768 3072 0 1" "8064 768 2304 0 1" "8064 768 768 0 0" "8064 768 768 0 1"; do
  for w in 0 1; do
    GVL_W4=$w timeout -k 10 60 python tools/gemm_one.py $spec 3 -1 50 2>/dev/null | sed "s/^/w4=$w /" >> $O/shapes.txt || exit $?
  done
  timeout -k 10 60 python tools/gemm_one.py $spec 9 0 50 2>/dev/null | sed "s/^/blaslt /" >> $O/shapes.txt || exit $?
done
for w in 1 0 1; do
  GVL_W4=$w timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_$w.json 2>> $O/qf.err || exit $?
  tail -1 $O/qf_$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('w4=$w', d['value'], d['ms_per_step'])" >> $O/shapes.txt
done
