# Which hipBLASLt kernels torch.mm picks for the caption / LM N=768 shapes (names encode the
# macro tile, MFMA shape, workgroup and stream-K), kernel-trace only.  Also times the same
# shapes with gvl's default routing.  args: spec list "M N K a_mn b_mn" ...
set -o pipefail
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
OUT=gpurun_out/blaslt; mkdir -p $OUT
i=0
for spec in "8064 768 3072 0 0" "8064 768 3072 0 1" "8064 768 768 0 0" "8064 768 2304 0 1" "8064 2304 768 0 0" "8064 3072 768 0 0" "16384 768 3072 0 0" "768 3072 16384 1 1"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/s$i -o run -- \
    python tools/gemm_one.py $spec 9 0 20 > $OUT/s$i.log 2>&1 || exit $?
  timeout -k 10 60 python tools/gemm_one.py $spec 3 -1 20 >> $OUT/s$i.log 2>&1 || exit $?
done
find $OUT -name "*.db" -delete
for f in $OUT/s*/run_kernel_stats.csv; do echo "== $f"; cut -d, -f1-4 $f | head -4; done > $OUT/summary.txt
cat $OUT/s*.log >> $OUT/summary.txt
