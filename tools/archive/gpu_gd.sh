set -o pipefail
mkdir -p gpurun_out/gd
O=gpurun_out/gd
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for i in 1 2; do
  for v in 0 1; do
    export GVL_GELU_DERIV=$v
    timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --no-secondary --no-cpu-baseline --no-kernel-pass > $O/lm_${v}_$i.json 2>$O/lm_${v}_$i.err || exit 1
    timeout -k 10 300 python -u bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-pass > $O/qf_${v}_$i.json 2>$O/qf_${v}_$i.err || exit 1
    echo "deriv=$v run $i: $(python3 -c "import json; print(json.loads(open('$O/lm_${v}_$i.json').read().strip().splitlines()[-1])['value'])") $(python3 -c "import json; print(json.loads(open('$O/qf_${v}_$i.json').read().strip().splitlines()[-1])['value'])")"
  done
done
