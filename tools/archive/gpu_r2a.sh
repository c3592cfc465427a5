set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity_full.py tests/test_gpu_boundary.py -v -s --timeout 300 --timeout-method thread > gpurun_out/r2a_new.log 2>&1
rc=$?
echo "new tests rc=$rc"
if [ $rc -eq 0 ] || [ $rc -eq 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > gpurun_out/r2a_all.log 2>&1
  echo "all rc=$?"
fi
