#!/bin/bash
# attention dropout case (Tq 40, Tk 130) that failed once: 3 repeats each with the current
# library and with the previous attention source (libgvl_attprev)
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-attbug}; O=gpurun_out/$TAG; mkdir -p $O
for v in cur prev; do
  L=gpt2-vision-language_amd/gvl/libgvl.so; [ $v = prev ] && L=gpt2-vision-language_amd/gvl/libgvl_attprev.so
  GVL_LIB=$L timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
    tests/test_gpu_kernels.py -k "attention" > $O/$v.log 2>&1 || true
  for i in 1 2 3; do
    GVL_LIB=$L timeout -k 10 120 python -u -m pytest -q --timeout 120 --timeout-method thread -p no:cacheprovider \
      "tests/test_gpu_kernels.py::test_attention_dropout_exact_mask" > $O/${v}_$i.log 2>&1
    echo "$v run $i: $(tail -1 $O/${v}_$i.log) $(grep -o 'd[qkv] rel err [0-9.e-]*' $O/${v}_$i.log | head -2 | tr '\n' ' ')"
  done
done
