# A/B of compile-time variants built as gvl/libgvl_<v>.so (GVL_LIB): caption N=768 GEMM shapes
# and the Q-Former bench, alternated.  args: TAG variant...  ("base" = gvl/libgvl.so)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=$1; shift
O=gpurun_out/ablib_$TAG; mkdir -p $O
lib() { if [ "$1" = base ]; then echo "$R/gpt2-vision-language_amd/gvl/libgvl.so"; else echo "$R/gpt2-vision-language_amd/gvl/libgvl_$1.so"; fi; }
for spec in "8064 768 3072 0 0" "8064 768 3072 0 1" "8064 768 2304 0 1" "8064 768 768 0 0"; do
  for v in "$@"; do
    GVL_LIB=$(lib $v) timeout -k 10 60 python tools/gemm_one.py $spec 3 -1 50 2>/dev/null | sed "s/^/$v /" >> $O/shapes.txt || exit $?
  done
done
[ "${WIDE:-0}" = 1 ] && for spec in "8064 3072 768 0 0" "8064 3072 768 0 1" "8064 2304 768 0 0" "4096 768 768 0 0" "4224 1536 768 0 0"; do
  for v in "$@"; do
    for cfg in -1 10; do
      GVL_LIB=$(lib $v) timeout -k 10 60 python tools/gemm_one.py $spec 3 $cfg 50 2>/dev/null | sed "s/^/$v /" >> $O/shapes.txt || exit $?
    done
  done
done
for rep in 1 2; do
  for v in "$@"; do
    GVL_LIB=$(lib $v) timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_$v.json 2>> $O/qf.err || exit $?
    tail -1 $O/qf_$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['value'], d['ms_per_step'])" >> $O/shapes.txt
  done
done
