# Attention occupancy A/B on the LM shape (B=16, H=12, T=1024): GVL_ATTN_G=1|default; parity first.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
O=gpurun_out/attn_$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "attention" > $O/tests.log 2>&1 || exit $?
GVL_ATTN_G=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "attention" >> $O/tests.log 2>&1 || exit $?
for g in 0 1; do
  GVL_ATTN_G=$g timeout -k 10 120 python tools/attn_one.py > $O/one_$g.txt 2>&1 || exit $?
done
for g in 0 1 0 1; do
  GVL_ATTN_G=$g timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $O/lm_$g.json 2>> $O/lm.err || exit $?
  tail -1 $O/lm_$g.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lm G=$g', d['value'], d['ms_per_step'])" >> $O/ab.txt
done
