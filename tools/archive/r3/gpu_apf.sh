#!/bin/bash
# w4d epilogue operand fetched one step ahead (GVL_W4D_AUXPF=1, default) vs inside the epilogue
# (libgvl_apf0): GEMM tests, then the Q-Former caption step alternated.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-apf}; O=gpurun_out/$TAG; mkdir -p $O
fatal() { case $1 in 124|134|137|139) echo "fatal rc $1 at $2"; exit $1;; esac; }
timeout -k 10 400 python -u -m pytest -q -x --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_kernels.py -k "gemm" > $O/tests.log 2>&1; rc=$?
echo "gemm tests rc=$rc: $(tail -1 $O/tests.log)"; [ $rc -ne 0 ] && { grep -E "FAIL|Error|assert" $O/tests.log | head -20; exit $rc; }
for v in base apf0 base apf0; do
  L=gpt2-vision-language_amd/gvl/libgvl.so; [ $v = apf0 ] && L=gpt2-vision-language_amd/gvl/libgvl_apf0.so
  GVL_LIB=$L timeout -k 10 300 python bench.py --workload qformer --steps 20 --warmup 5 --no-cpu-baseline > $O/qf_$v.json 2> $O/qf_$v.err; fatal $? qf
  python -c "
import json
d=json.loads(open('$O/qf_$v.json').read().strip().splitlines()[-1]); print('qf $v', d['value'], d['ms_per_step'], [(g['kernel'], g['avg_us']) for g in d['roofline']['top_gemms'][:2]])"
done
