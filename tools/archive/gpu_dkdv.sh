# LDS-DMA pipelined dK/dV: attention parity (both paths), kernel timing and LM bench A/B (GVL_DKDV_DMA).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
O=gpurun_out/dkdv_$TAG; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_models.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "attention or full" > $O/tests.log 2>&1 || exit $?
for d in 1 0 1; do
  GVL_DKDV_DMA=$d timeout -k 10 120 python tools/attn_one.py 20 > $O/one_$d.txt 2>&1 || exit $?
done
for d in 1 0 1 0; do
  GVL_DKDV_DMA=$d timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $O/lm_$d.json 2>> $O/lm.err || exit $?
  tail -1 $O/lm_$d.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lm dma=$d', d['value'], d['ms_per_step'])" >> $O/ab.txt
done
