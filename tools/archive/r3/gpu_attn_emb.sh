#!/bin/bash
# Embedding backward tests + timing; attention tests and timing with the G=4 forward.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/${1:-ae}; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
#timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "embedding or attention" -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 $O/t.log; fatal $rc tests
#GVL_ATTN_FWD_G=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -k "attention" -q -x --timeout 120 --timeout-method thread -p no:cacheprovider > $O/t4.log 2>&1; rc=$?; echo "tests G4 rc=$rc"; tail -3 $O/t4.log; fatal $rc testsG4
#timeout -k 10 120 python tools/r3/emb_one.py; fatal $? emb
for g in 0 4 0 4; do echo "== GVL_ATTN_FWD_G=$g"; GVL_ATTN_FWD_G=$g timeout -k 10 120 python tools/attn_one.py 20 2>/dev/null; fatal $? attn; done
