#!/bin/bash
# Rehearsal of the bench's N > 1 path on a one-GPU box: two ranks on cuda:0 over gloo
# (GVL_BENCH_ONE_DEVICE=1), graphed (segmented DP graphs) and eager, LM and Q-Former workloads.
# The numbers are not bench lines (two processes share one GPU; gloo, not RCCL).
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 GVL_BENCH_ONE_DEVICE=1
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-dp2}; O=gpurun_out/$TAG; mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --gpus 2 "$@" > $O/$n.json 2> $O/$n.err; local rc=$?
  echo "$n rc=$rc: $(tail -1 $O/$n.json | cut -c1-400)"
  case $rc in 0) ;; *) tail -5 $O/$n.err; exit $rc;; esac
}
run lm_graph --steps 2 --warmup 1 --no-secondary --no-cpu-baseline
run qf_graph --workload qformer --steps 3 --warmup 2 --no-cpu-baseline
run lm_eager --steps 1 --warmup 1 --no-secondary --no-cpu-baseline --no-graph
