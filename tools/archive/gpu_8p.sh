set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/gemm_shapes.py all 3:-1,5:-1 > gpurun_out/shapes_w4.log 2>&1 && \
GVL_W4_NS=4 timeout -k 10 120 python -u tools/gemm_shapes.py big 5:-1 > gpurun_out/shapes_w4ns4.log 2>&1
