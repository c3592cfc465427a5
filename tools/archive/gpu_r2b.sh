# bench (default) + rocprofv3 kernel stats of each workload (no kernel pass, no CPU
# baseline), to check the dispatch-timed roofline against rocprof's per-kernel averages
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${TAG:-r2b}
mkdir -p $O
if [ -z "$NOBENCH" ]; then
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
echo "bench rc=$?"
fi
cd /tmp && export TMPDIR=/tmp
for w in ${WORKLOADS:-lm qformer linear cross}; do
  extra="--workload $w --steps 10 --warmup 3"
  [ $w = lm ] && extra="--no-secondary --steps 5 --warmup 2"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o run -- python3 $R/bench.py $extra --no-kernel-pass --no-cpu-baseline > $O/prof_$w.json 2> $O/prof_$w.err || { echo "prof $w failed rc=$?"; exit 1; }
  # keep only the summaries (the full traces exceed gpurun's 64 MiB return limit)
  find $O/prof_$w -type f ! -name '*stats.csv' -delete
  echo "prof $w ok"
done
cd $R
[ -z "$NOSHAPES" ] && timeout -k 10 300 python -u tools/gemm_shapes.py qf > $O/gemm_shapes_qf.log 2>&1 && echo "shapes ok"
true
