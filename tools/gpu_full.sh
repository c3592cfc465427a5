#!/bin/bash
# Full round-3 check: GPU suite (margins recorded), smoke, default bench, rocprof stats of the
# LM and Q-Former bench steps.  Stops after any time-out / crash.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r3full}; O=gpurun_out/$TAG; mkdir -p $O
export GVL_MARGINS_DIR=$O/parity_margins
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
rc=$?; echo "suite rc=$rc"; tail -4 $O/suite.log; fatal $rc suite
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; fatal $rc smoke
timeout -k 10 500 python bench.py > $O/bench.json 2> $O/bench.err; rc=$?; echo "bench rc=$rc"; fatal $rc bench
python - <<PY
import json
d = json.loads(open("$O/bench.json").read().strip().splitlines()[-1])
print("LM", d["value"], d["step_mfma_frac"], d["loss"], d["roofline"]["kernel"], d["roofline"]["frac"])
for k in ("caption_qformer", "caption_linear", "caption_cross", "caption_linear_pixels"):
    if k in d: print(k, d[k]["value"], d[k].get("step_mfma_frac"), d[k].get("loss"))
PY
[ "${2:-}" = noprof ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_qf -o qf -- \
  python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_qf.json 2> $O/prof_qf.err; rc=$?; fatal $rc prof_qf
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lm -o lm -- \
  python bench.py --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > $O/prof_lm.json 2> $O/prof_lm.err; rc=$?; fatal $rc prof_lm
for w in qf lm; do f=$(find $O/prof_$w -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 30 > $O/${w}_table.txt; echo "== $w"; head -22 $O/${w}_table.txt; done
