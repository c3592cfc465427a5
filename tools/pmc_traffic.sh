#!/bin/bash
# HBM traffic of the bench's kernels from PMC counters (calibration: profiles/r2/pmc_calibration.md): one
# rocprofv3 pass per counter (FETCH_SIZE and WRITE_SIZE do not fit one TCC pass), kernel-trace
# only, eager step (graph replays are not attributed per dispatch), each pass time-limited.
# Then tools/pmc_traffic.py turns them into per-launch bytes -> gpurun_out/pmc_traffic_$TAG.json.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; TAG=${1:-x}; WLS=${2:-"lm qf"}
OUT=gpurun_out/pmc_traffic_$TAG; mkdir -p $OUT
# Round 1 ran these passes with AMD_SERIALIZE_KERNEL=3 after one HSA_STATUS_ERROR_INVALID_PACKET_FORMAT
# abort; the same eager LM pass without it completed in round 2 (tools/pmc_calib.sh,
# profiles/r2/pmc_calibration.md), so the passes run unserialised.
# Third pass: MFMA busy cycles + achieved clock (SQ 2 + GRBM 1 counters: one pass).
# Workloads (round 6): lm, qf (Q-Former), cross, linear — every bench line gets its traffic.
for c in FETCH_SIZE WRITE_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  d=${c%% *}
  for wl in $WLS; do
    if [ $wl = lm ]; then a="--steps 1 --warmup 0 --no-secondary"
    else a="--workload $([ $wl = qf ] && echo qformer || echo $wl) --steps 2 --warmup 0"; fi
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $OUT/${wl}_$d -o run -- \
      python bench.py $a --no-cpu-baseline --no-graph > $OUT/${wl}_$d.log 2>&1 || exit $?
  done
done
python tools/pmc_traffic.py $OUT > gpurun_out/pmc_traffic_$TAG.json
