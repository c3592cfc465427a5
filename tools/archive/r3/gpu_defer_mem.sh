#!/bin/bash
# Deferred weight gradients on/off (GVL_DEFER_WGRAD): LM tokens/s and peak HBM (graphed and
# eager steps), alternated; then the HBM traffic of both steps with the current tile walk.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-defer}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
show() { python -c "
import json
d=json.loads(open('$1').read().strip().splitlines()[-1]); print('$2', d['value'], d['ms_per_step'], 'peak GiB', d['peak_hbm_gib'])"; }
for v in 1 0 1 0; do
  GVL_DEFER_WGRAD=$v timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-secondary --no-cpu-baseline > $O/g_$v.json 2> $O/g_$v.err; fatal $? lm_g; [ -s $O/g_$v.json ] || exit 1
  show $O/g_$v.json "graphed DEFER=$v"
done
for v in 1 0; do
  GVL_DEFER_WGRAD=$v timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline --no-graph --no-kernel-pass > $O/e_$v.json 2> $O/e_$v.err; fatal $? lm_e; [ -s $O/e_$v.json ] || exit 1
  show $O/e_$v.json "eager DEFER=$v"
done
timeout -k 10 900 bash tools/pmc_traffic.sh $TAG || exit $?
python - <<EOF
import json
d = json.load(open("gpurun_out/pmc_traffic_$TAG.json"))["workloads"]
for w in ("lm", "qf"):
    for k, v in sorted(d[w].items(), key=lambda kv: -kv[1]["hbm_bytes"] * kv[1]["launches"])[:8]:
        print(w, k[:60], v["launches"], round(v["hbm_bytes"] / 1e6, 1), "MB/launch")
EOF
