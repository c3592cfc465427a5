# Timing-only diagnostic builds of gemm_w4 (no barrier / no operand staging): where the time goes
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=gpurun_out/w4diag; mkdir -p $O
for spec in "8064 768 3072 0 0" "8064 768 3072 0 1" "8064 768 768 0 0"; do
  for v in libgvl libgvl_diag1 libgvl_diag2; do
    GVL_LIB=$R/gpt2-vision-language_amd/gvl/$v.so timeout -k 10 60 python tools/gemm_one.py $spec 3 -1 50 2>/dev/null | sed "s/^/$v /" >> $O/shapes.txt || exit $?
  done
done
