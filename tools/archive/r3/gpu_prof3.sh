#!/bin/bash
# Round-3 profiles: DP overlap traces (world-1 RCCL, forced buckets), rocprofv3 stats of the
# Q-Former and LM bench steps.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-r3p}; O=gpurun_out/$TAG; mkdir -p $O
for mode in eager graph; do
  GVL_TRACE_BUCKETS=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv -d $O/dp_$mode -o dp -- \
    python tools/r3/dp_overlap_trace.py $mode > $O/dp_$mode.log 2>&1 || exit $?
  python tools/r3/dp_overlap_report.py $O/dp_$mode > $O/dp_overlap_$mode.txt 2>&1; cat $O/dp_overlap_$mode.txt | head -20
done
[ "${2:-}" = dp ] && exit 0
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_qf -o qf -- \
  python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_qf.json 2> $O/prof_qf.err || exit $?
f=$(find $O/prof_qf -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 40 > $O/qf_table.txt; head -45 $O/qf_table.txt
