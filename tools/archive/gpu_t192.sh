set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "tile192 or persistent or splitk or wgrad or layouts" > gpurun_out/t192.log 2>&1 && \
GVL_PP3_BN=256 timeout -k 10 300 python -u tools/gemm_shapes.py all 3:-1 > gpurun_out/shapes_bn256.log 2>&1 && \
timeout -k 10 300 python -u tools/gemm_shapes.py all 3:-1 > gpurun_out/shapes_bn192.log 2>&1
