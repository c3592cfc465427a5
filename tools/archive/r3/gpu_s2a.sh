#!/bin/bash
# Session-2 opener: w4 diagnostics (base / no-barrier / no-memory builds) at M = 8064, then the
# full check of the head (suite, smoke, bench; no profile).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
bash tools/r3/gpu_w4diag.sh w4d base d1 d2 || exit $?
bash tools/r3/gpu_full.sh r3s2a noprof
