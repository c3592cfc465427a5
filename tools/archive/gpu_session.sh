#!/bin/bash
# One GPU session: gpu tests (rc 0/1 both continue: failures are read from the log),
# then the default bench, then rocprof kernel traces.  Any other exit status (timeout,
# abort, fault) ends the session immediately.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r1}
timeout -k 10 600 python -m pytest tests -m gpu -q -rf -s -p no:cacheprovider > gpurun_out/gpu_tests_$TAG.log 2>&1
rc=$?; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit $?
bash tools/prof.sh $TAG
