#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
timeout -k 10 600 python -m pytest tests -m gpu -q -x -rf -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1 || exit $?
bash tools/prof.sh $TAG
