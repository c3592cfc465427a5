# Ring-depth A/B: default libgvl.so (NS 4/4/4) vs libgvl_ns.so (NS 5 for 256-row tiles, 6 for 128x192).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-n}
O=gpurun_out/ns_$TAG; mkdir -p $O
V=$R/gpt2-vision-language_amd/gvl/libgvl_ns.so
GVL_LIB=$V timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider \
  -k "gemm_persistent or tile192 or tile128 or gelu_derivative or wgrad" > $O/tests.log 2>&1 || exit $?
for spec in "8064 768 3072 0 0" "8064 768 768 0 0" "8064 768 2304 0 1" "8064 2304 768 0 0" "8064 3072 768 0 0" "16384 768 3072 0 0" "16384 2304 768 0 0" "16384 3072 768 0 0" "8192 8192 8192 0 0"; do
  for lib in libgvl libgvl_ns; do
    GVL_LIB=$R/gpt2-vision-language_amd/gvl/$lib.so timeout -k 10 60 python tools/gemm_one.py $spec 3 -1 30 2>/dev/null | sed "s/^/$lib /" >> $O/shapes.txt || exit $?
  done
done
for lib in libgvl_ns libgvl libgvl_ns libgvl; do
  GVL_LIB=$R/gpt2-vision-language_amd/gvl/$lib.so timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_$lib.json 2>> $O/qf.err || exit $?
  tail -1 $O/qf_$lib.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('qf $lib', d['value'], d['ms_per_step'])" >> $O/shapes.txt
done
for lib in libgvl_ns libgvl; do
  GVL_LIB=$R/gpt2-vision-language_amd/gvl/$lib.so timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-secondary > $O/lm_$lib.json 2>> $O/lm.err || exit $?
  tail -1 $O/lm_$lib.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('lm $lib', d['value'], d['ms_per_step'])" >> $O/shapes.txt
done
