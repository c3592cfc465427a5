#!/bin/bash
# Round 3, first GPU session: the new tests (bench-shape parity, DP overlap, deferral safety,
# CrossAttention.forward, feature shards) verbose, then the full GPU suite, then the bench.
# Stops after any time-out / crash (124, 134, 137, 139); test failures continue.
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r3a}; O=gpurun_out/$TAG; mkdir -p $O
export GVL_MARGINS_DIR=$O/parity_margins
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest -v -s -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_parity_bench.py tests/test_gpu_dp.py \
  "tests/test_gpu_boundary.py::test_cross_attention_module_forward" \
  "tests/test_gpu_boundary.py::test_feature_shard_loader_feeds_caption_step" \
  "tests/test_gpu_boundary.py::test_deferred_wgrad_survives_failed_backward" > $O/new_tests.log 2>&1
rc=$?; echo "new tests rc=$rc"; fatal $rc new_tests
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_gpu_parity_bench.py --deselect tests/test_gpu_dp.py > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log; fatal $rc suite
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; fatal $rc bench
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r3a/bench.json").read().strip().splitlines()[-1])
print("LM", d["value"], d["step_mfma_frac"], d["loss"])
for k in ("caption_qformer", "caption_linear", "caption_cross", "caption_linear_pixels"):
    if k in d: print(k, d[k]["value"], d[k].get("step_mfma_frac"), d[k].get("loss"))
PY
