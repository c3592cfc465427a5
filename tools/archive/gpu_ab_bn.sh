# A/B of the persistent GEMM's tile width on the LM step and the Q-Former step: default
# planner (192-wide tiles where they fill CUs better) vs GVL_PP3_BN=256, alternated twice.
set -o pipefail
mkdir -p gpurun_out/ab_bn
O=gpurun_out/ab_bn
for i in 1 2; do
  for v in 256 auto; do
    if [ $v = auto ]; then unset GVL_PP3_BN; else export GVL_PP3_BN=$v; fi
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-secondary --no-cpu-baseline --no-kernel-pass > $O/lm_${v}_$i.json 2>$O/lm_${v}_$i.err || exit 1
    timeout -k 10 300 python -u bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-pass > $O/qf_${v}_$i.json 2>$O/qf_${v}_$i.err || exit 1
    echo "$v $i: $(python3 -c "import json,sys; print(json.loads(open('$O/lm_${v}_$i.json').read().strip().splitlines()[-1])['value'])") $(python3 -c "import json,sys; print(json.loads(open('$O/qf_${v}_$i.json').read().strip().splitlines()[-1])['value'])")"
  done
done
