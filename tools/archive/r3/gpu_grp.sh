#!/bin/bash
# Tile walk of the four-wave kernels: GVL_W4_GROUP=1 (all column tiles of a row block on one XCD)
# vs the default L2-grouped walk — Q-Former step alternated, then the HBM traffic of both.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-grp}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
for v in 0 1 0 1; do
  GVL_W4_GROUP=$v timeout -k 10 300 python bench.py --workload qformer --steps 20 --warmup 5 --no-cpu-baseline > $O/qf_$v.json 2> $O/qf_$v.err; fatal $? qf
  python -c "
import json
d=json.loads(open('$O/qf_$v.json').read().strip().splitlines()[-1]); print('qf GROUP=$v', d['value'], d['ms_per_step'], [(g['kernel'], g['avg_us']) for g in d['roofline']['top_gemms'][:2]])"
done
for v in 0 1; do
  for c in FETCH_SIZE WRITE_SIZE; do
    GVL_W4_GROUP=$v timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/g${v}/qf_$c -o run -- \
      python bench.py --workload qformer --steps 2 --warmup 0 --no-cpu-baseline --no-graph > $O/pmc_${v}_$c.log 2>&1 || exit $?
  done
  python tools/pmc_traffic.py $O/g$v > $O/traffic_$v.json
  python -c "
import json
d=json.load(open('$O/traffic_$v.json'))['workloads']['qf']
for k in ('gemm_w4d_kernel<true, 0>', 'gemm_w4d_kernel<false, 2>'): print('GROUP=$v', k, d.get(k, {}).get('hbm_bytes'))"
done
