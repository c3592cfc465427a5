#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
timeout -k 10 300 python -m pytest tests/test_gpu_kernels.py -q -x -rf -p no:cacheprovider -k attention > gpurun_out/kern_$TAG.log 2>&1 || exit $?
timeout -k 10 120 python tools/attn_one.py > gpurun_out/attn_$TAG.log 2>&1 || exit $?
bash tools/pmc_attn.sh $TAG
