#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration on known-byte kernels (no AMD_SERIALIZE_KERNEL), then one
# FETCH_SIZE pass over the eager LM bench step without AMD_SERIALIZE_KERNEL (the round-1 abort).
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"
OUT=gpurun_out/pmc_calib; mkdir -p $OUT
timeout -k 10 120 python tools/pmc_calib.py > $OUT/expect.log 2>&1 || exit $?
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/$c -o run -- \
    python tools/pmc_calib.py > $OUT/$c.log 2>&1 || exit $?
done
python tools/pmc_calib_report.py $OUT > $OUT/calibration.json || exit $?
cat $OUT/calibration.json
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/lm_noserial -o run -- \
  python bench.py --steps 1 --warmup 0 --no-secondary --no-cpu-baseline --no-graph --no-kernel-pass > $OUT/lm_noserial.log 2>&1
echo "lm eager FETCH_SIZE pass without AMD_SERIALIZE_KERNEL: exit $?"
tail -5 $OUT/lm_noserial.log
