set -o pipefail
mkdir -p gpurun_out
GVL_DKDV_G=2 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attention" > gpurun_out/attn_g2_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/attn_one.py 20 > gpurun_out/attn_g1.log 2>&1 && \
GVL_DKDV_G=2 timeout -k 10 120 python -u tools/attn_one.py 20 > gpurun_out/attn_g2.log 2>&1
