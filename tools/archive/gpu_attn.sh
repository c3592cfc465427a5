#!/bin/bash
# kernel tests + bench (each step time-limited; stop on a non-test failure)
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -rf -p no:cacheprovider > gpurun_out/kern_$TAG.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
