set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -v -s --timeout 300 --timeout-method thread > gpurun_out/r2c.log 2>&1
echo "tests rc=$?"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r2c_bench.json 2> gpurun_out/r2c_bench.err
echo "bench rc=$?"
