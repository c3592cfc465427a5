#!/bin/bash
# Copy a head-check session's evidence from gpurun_out/<S> into profiles/r6 (CPU side):
# suite log, smoke line, bench line, kernel tables + stats CSVs of the four steps, parity margins.
set -e
S=${1:?session}; O=gpurun_out/$S; P=profiles/r6
cp $O/suite.log $P/gpu_suite_$S.txt
cp $O/smoke.log $P/smoke_$S.txt
cp $O/bench.json $P/bench_$S.json
for w in qf lm cross linear; do
  n=$w; [ $w = qf ] && n=qformer
  cp $O/${w}_table.txt $P/${n}_step_kernel_table_$S.txt
  f=$(find $O/prof_$w -name "*kernel_stats.csv" | head -1); cp $f $P/${n}_step_kernel_stats_$S.csv
done
python3 - "$O/parity_margins" "$P/parity_margins_$S.json" <<'PY'
import glob, json, os, sys
d = {os.path.basename(f)[:-5]: json.load(open(f)) for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json")))}
json.dump(d, open(sys.argv[2], "w"), indent=1)
print(len(d), "margin records")
PY
