#!/bin/bash
# Round-end confirmation: GPU suite, default bench (with PMC traffic from profiles/), smoke, and
# rocprofv3 kernel stats of both bench workloads. Each step time-limited; stop at the first failure.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x -rf --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/final_tests_$TAG.log 2>&1 || exit $?
timeout -k 10 400 python bench.py > gpurun_out/final_bench_$TAG.json 2> gpurun_out/final_bench_$TAG.err || exit $?
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke_$TAG.log 2>&1 || exit $?
bash tools/prof.sh $TAG
