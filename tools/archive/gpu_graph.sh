#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_graph.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/graph_tests_$TAG.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_qf_$TAG.json 2> gpurun_out/bench_qf_$TAG.err || exit $?
timeout -k 10 300 python -u bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline --no-graph > gpurun_out/bench_qf_eager_$TAG.json 2>> gpurun_out/bench_qf_$TAG.err || exit $?
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
