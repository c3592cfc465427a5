# dQ DMA A/B on one box: kernel trace of tools/attn_one.py with GVL_DQ_DMA=1|0, then LM bench.
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
O=gpurun_out/dq_$TAG; mkdir -p $O
for d in 1 0; do
  GVL_DQ_DMA=$d timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p$d -o run -- python tools/attn_one.py 20 > $O/one_$d.txt 2>&1 || exit $?
done
for d in 1 0 1 0; do
  GVL_DQ_DMA=$d timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $O/lm_$d.json 2>> $O/lm.err || exit $?
  tail -1 $O/lm_$d.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lm dq_dma=$d', d['value'], d['ms_per_step'])" >> $O/ab.txt
done
find $O -name "*.db" -delete
