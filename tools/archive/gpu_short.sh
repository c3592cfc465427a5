# Short-sequence fused attention backward: attention + model parity, Q-Former bench A/B (GVL_ATTN_SHORT).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-s}
O=gpurun_out/short_$TAG; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "attention or qformer or caption or cross or combined_in_launch" > $O/tests.log 2>&1 || exit $?
for c in 1 0 1 0; do
  GVL_ATTN_SHORT=$c timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_$c.json 2>> $O/qf.err || exit $?
  tail -1 $O/qf_$c.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('short=$c', d['value'], d['ms_per_step'])" >> $O/ab.txt
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o qf -- \
  python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_qf.json 2> $O/prof_qf.err || exit $?
