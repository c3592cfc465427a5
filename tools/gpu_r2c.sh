set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode.py -v -s --timeout 200 --timeout-method thread -k "sampler" > gpurun_out/r2c.log 2>&1
echo "rc=$?"
