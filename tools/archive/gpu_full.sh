#!/bin/bash
# full GPU suite + default bench (each step time-limited; stop at the first failure)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
timeout -k 10 600 python -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
