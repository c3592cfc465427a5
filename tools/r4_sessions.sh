#!/bin/bash
# Round-4 GPU sessions (run on the GPU box through gpurun): bash tools/r4_sessions.sh <name>.
# Every GPU step has its own time limit; a session stops at the first failing step.
export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; S=${1:?session}; O=gpurun_out/$S; mkdir -p $O
LIBDIR=gpt2-vision-language_amd/gvl
fatal() { [ "$1" -eq 0 ] || { echo "fatal rc $1 at $2"; exit $1; }; }
suite() {  # GPU suite (margins recorded) + smoke
  GVL_MARGINS_DIR=$O/parity_margins timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf \
    --timeout 300 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
  rc=$?; echo "suite rc=$rc"; tail -3 $O/suite.log; fatal $rc suite
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; echo "smoke rc=$rc $(tail -1 $O/smoke.log)"; fatal $rc smoke
}
diag() {  # diag <lib-suffix|base> <M> <set> <cols>
  local L=$LIBDIR/libgvl_$1.so; [ "$1" = base ] && L=$LIBDIR/libgvl.so
  GVL_LIB=$L GVL_DIAG_COLS=$4 timeout -k 10 240 python -u tools/gemm_diag.py $2 $3 > $O/diag_$1_$2_$3.log 2>&1
  rc=$?; echo "== $1 M=$2 $3"; cat $O/diag_$1_$2_$3.log | grep "N=" ; fatal $rc diag
}
case $S in
r4a)  # HEAD check + epilogue share of the short-K wide GEMMs (timing-only pp3 builds)
  suite
  diag base 8064 all all
  diag base 16384 wide all
  for v in pp3d1 pp3d2 base; do diag $v 8064 wide epi; diag $v 16384 wide epi; done
  ;;
r4c)  # counted epilogue: GEMM kernel tests, then A/B (GVL_PP3_CNT=1 default / 0) on shapes and steps
  timeout -k 10 900 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "gemm or batched" --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/kt.log 2>&1; rc=$?; tail -3 $O/kt.log; fatal $rc kernel_tests
  for c in 1 0; do GVL_PP3_CNT=$c diag base 8064 all epi; mv $O/diag_base_8064_all.log $O/diag_c${c}_8064.log
    GVL_PP3_CNT=$c diag base 16384 wide epi; mv $O/diag_base_16384_wide.log $O/diag_c${c}_16384.log; done
  for w in qformer lm; do for c in 1 0; do
    a="--workload qformer --steps 10 --warmup 3"; [ $w = lm ] && a="--steps 2 --warmup 1 --no-secondary"
    GVL_PP3_CNT=$c timeout -k 10 300 python bench.py $a --no-cpu-baseline > $O/${w}_c$c.json 2> $O/${w}_c$c.err
    fatal $? bench_$w
    echo "$w cnt=$c $(python -c "import json;d=json.load(open('$O/${w}_c$c.json'));print(d['value'],d.get('step_mfma_frac'))")"
  done; done
  ;;
r4d)  # early-clobber fix + fused D re-landed: GPU suite once, smoke, the driver's default bench
  suite
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; fatal $? bench
  python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac'],[(k,v.get('value')) for k,v in d.get('secondary',{}).items()] if isinstance(d.get('secondary'),dict) else '')"
  ;;
r4e)  # rocprof kernel stats of both steps at this head; Q-Former DP overlap traces (world-1 RCCL)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_qf -o qf -- \
    python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_qf.json 2> $O/prof_qf.err; fatal $? prof_qf
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lm -o lm -- \
    python bench.py --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > $O/prof_lm.json 2> $O/prof_lm.err; fatal $? prof_lm
  for w in qf lm; do f=$(find $O/prof_$w -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 40 > $O/${w}_table.txt; head -25 $O/${w}_table.txt; done
  for mb in 32 8; do for mode in qf_eager qf_graph; do
    GVL_BUCKET_MB=$mb GVL_TRACE_BUCKETS=1 timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --output-format csv \
      -d $O/dp_${mode}_$mb -o dp -- python tools/dp_overlap_trace.py $mode > $O/dp_${mode}_$mb.log 2>&1; fatal $? dp_$mode
    python tools/dp_overlap_report.py $O/dp_${mode}_$mb > $O/dp_overlap_${mode}_$mb.txt 2>&1; echo "== $mode $mb MB"; head -12 $O/dp_overlap_${mode}_$mb.txt
  done; done
  ;;
r4f)  # batched weight gradients vs the hipBLASLt yardstick; N = 768 shapes on the persistent kernel
  timeout -k 10 300 python -u tools/wgrad_diag.py > $O/wgrad.log 2>&1; rc=$?; cat $O/wgrad.log; fatal $rc wgrad
  diag base 8064 narrow all; mv $O/diag_base_8064_narrow.log $O/diag_def_8064n.log
  GVL_GEMM_CFG=3 diag base 8064 narrow all; mv $O/diag_base_8064_narrow.log $O/diag_pp3_8064n.log
  GVL_GEMM_CFG=3 diag base 16384 narrow all; mv $O/diag_base_16384_narrow.log $O/diag_pp3_16384n.log
  diag base 16384 narrow all
  ;;
r4g)  # attention forward: LDS-DMA ring vs register staging (GVL_ATTN_FWD_DMA), alternated
  for r in 1 2; do for f in 1 0; do
    GVL_ATTN_FWD_DMA=$f timeout -k 10 200 python -u tools/attn_one.py 20 > $O/attn_f${f}_$r.log 2>&1; fatal $? attn
    echo "fwd_dma=$f round $r"; head -3 $O/attn_f${f}_$r.log
  done; done
  for f in 1 0; do
    GVL_ATTN_FWD_DMA=$f timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_f$f.json 2> $O/lm_f$f.err
    fatal $? bench_lm; echo "lm fwd_dma=$f $(python -c "import json;d=json.load(open('$O/lm_f$f.json'));print(d['value'])")"
  done
  ;;
r4h|r4w3)  # PMC passes of both bench steps (HBM bytes, MFMA busy, achieved clock per kernel)
  bash tools/pmc_traffic.sh $S; rc=$?; fatal $rc pmc
  python -c "import json;d=json.load(open('gpurun_out/pmc_traffic_$S.json'));[print(w,k,v) for w in d['workloads'] for k,v in sorted(d['workloads'][w].items(),key=lambda kv:-kv[1].get('launches',0))[:6]]"
  ;;
r4i)  # which hipBLASLt kernels (macro tile, MFMA, depth) beat the persistent / direct-A GEMMs on N = 768
  for M in 16384 8064; do
    GVL_DIAG_COLS=all timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_diag_$M -o diag -- \
      python tools/gemm_diag.py $M narrow > $O/diag_$M.log 2>&1; fatal $? prof_diag
    f=$(find $O/prof_diag_$M -name "*kernel_stats.csv" | head -1)
    python -c "import csv,sys;rows=sorted(csv.DictReader(open(sys.argv[1])),key=lambda r:-float(r['TotalDurationNs']));[print(r['Calls'],round(float(r['AverageNs'])/1e3,2),r['Name'][:400]) for r in rows[:30]]" $f > $O/diag_table_$M.txt
    cat $O/diag_table_$M.txt
  done
  ;;
r4j)  # plain N = 768 GEMMs on hipBLASLt (gemm_lib.cpp): the route tests alone first, full suite, then A/B
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "library_route" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $O/route.log 2>&1; rc=$?; tail -3 $O/route.log; fatal $rc route_tests
  suite
  for c in 1 0; do GVL_GEMM_LIB=$c diag base 16384 narrow all; mv $O/diag_base_16384_narrow.log $O/diag_lib${c}_16384.log
    GVL_GEMM_LIB=$c diag base 8064 all all; mv $O/diag_base_8064_all.log $O/diag_lib${c}_8064.log; done
  for w in qformer lm; do for c in 1 0 1 0; do
    a="--workload qformer --steps 10 --warmup 3"; [ $w = lm ] && a="--steps 2 --warmup 1 --no-secondary"
    GVL_GEMM_LIB=$c timeout -k 10 300 python bench.py $a --no-cpu-baseline > $O/${w}_l$c.json 2> $O/${w}_l$c.err
    fatal $? bench_$w
    echo "$w lib=$c $(python -c "import json;d=json.load(open('$O/${w}_l$c.json'));print(d['value'],d.get('step_mfma_frac'))")"
  done; done
  ;;
r4k)  # PMC anatomy of the persistent GEMM vs hipBLASLt: wave waits, MFMA busy, LDS, L2 (tools/pmc_gemm.sh)
  GVL_GEMM_LIB=0 bash tools/pmc_gemm.sh $S "16384 3072 768 0 0 3 -1 5 act" "16384 768 3072 0 1 3 -1 5 plain" \
    "16384 768 3072 0 1 9 -1 5 plain" "16384 50304 768 0 0 3 3 5 plain" "16384 50304 768 0 0 9 -1 5 plain"; fatal $? pmc_gemm
  for pn in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
            "GRBM_GUI_ACTIVE GRBM_COUNT TCC_HIT_sum TCC_MISS_sum"; do
    d=gpurun_out/pmc_$S/wgrad_${pn%% *}
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $pn --output-format csv -d $d -o run -- python tools/wgrad_diag.py > $d.log 2>&1; fatal $? pmc_wgrad
  done
  python tools/pmc_summary.py gpurun_out/pmc_$S > $O/pmc_summary.txt; cat $O/pmc_summary.txt; cat gpurun_out/pmc_$S/times.log | grep -v amdgpu.ids
  ;;
r4l)  # persistent GEMM ring depth: NS = 5 (three K-steps in flight) vs 4, alternated; the
      # direct-A four-wave kernel forced onto the wide (K = 768) shapes (GVL_W4=2)
  for v in ns5 base ns5 base; do diag $v 16384 wide all; diag $v 8064 wide all; done
  GVL_W4=2 diag base 16384 wide all; mv $O/diag_base_16384_wide.log $O/diag_w4_16384_wide.log
  GVL_W4=2 diag base 8064 wide all; mv $O/diag_base_8064_wide.log $O/diag_w4_8064_wide.log
  GVL_LIB=$LIBDIR/libgvl_ns5.so timeout -k 10 300 python -u tools/wgrad_diag.py > $O/wgrad_ns5.log 2>&1; fatal $? wgrad; grep x12 $O/wgrad_ns5.log
  timeout -k 10 300 python -u tools/wgrad_diag.py > $O/wgrad_base.log 2>&1; fatal $? wgrad; grep x12 $O/wgrad_base.log
  for w in lm qformer; do for v in ns5 base ns5 base; do
    L=$LIBDIR/libgvl_$v.so; [ $v = base ] && L=$LIBDIR/libgvl.so
    a="--workload qformer --steps 10 --warmup 3"; [ $w = lm ] && a="--steps 2 --warmup 1 --no-secondary"
    GVL_LIB=$L timeout -k 10 300 python bench.py $a --no-cpu-baseline > $O/${w}_$v.json 2> $O/${w}_$v.err; fatal $? bench_$w
    echo "$w $v $(python -c "import json;d=json.load(open('$O/${w}_$v.json'));print(d['value'],d.get('step_mfma_frac'))")"
  done; done
  ;;
r4m)  # re-entry check of HEAD (hipBLASLt route on): route tests alone, GPU suite + smoke; persistent
      # GEMM start stagger A/B (GVL_PP3_STAGGER, wide shapes + lm_head); step A/B of the route
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "library_route" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $O/route.log 2>&1; rc=$?; tail -3 $O/route.log; fatal $rc route_tests
  suite
  for st in 0 6 12 0 6 12; do GVL_PP3_STAGGER=$st diag base 16384 wide epi; mv $O/diag_base_16384_wide.log $O/diag_st${st}_16384.log
    GVL_PP3_STAGGER=$st diag base 8064 wide epi; mv $O/diag_base_8064_wide.log $O/diag_st${st}_8064.log; done
  for w in qformer lm; do for c in 1 0 1 0; do
    [ $w = lm ] && [ $c = 1 ] && [ -f $O/lm_l0.json ] && break
    a="--workload qformer --steps 10 --warmup 3"; [ $w = lm ] && a="--steps 2 --warmup 1 --no-secondary"
    GVL_GEMM_LIB=$c timeout -k 10 300 python bench.py $a --no-cpu-baseline > $O/${w}_l$c.json 2> $O/${w}_l$c.err
    fatal $? bench_$w
    echo "$w lib=$c $(python -c "import json;d=json.load(open('$O/${w}_l$c.json'));print(d['value'],d.get('step_mfma_frac'))")"
  done; done
  ;;
r4n)  # cache policy of the persistent GEMM's counted-epilogue stores (GVL_PP3_ST_AUX builds), alternated
  for r in 1 2; do for v in base stnt stsc1 stsc1nt; do
    diag $v 16384 wide epi; mv $O/diag_${v}_16384_wide.log $O/diag_${v}_16384_$r.log
    diag $v 8064 wide epi; mv $O/diag_${v}_8064_wide.log $O/diag_${v}_8064_$r.log
  done; done
  ;;
r4o)  # AGPR four-wave GEMM (gemm_w4x.hip): parity tests first, then shapes vs the defaults and hipBLASLt
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "test_gemm_w4x" --timeout 120 \
    --timeout-method thread -p no:cacheprovider > $O/w4x_tests.log 2>&1; rc=$?; tail -3 $O/w4x_tests.log; fatal $rc w4x_tests
  for r in 1 2; do
    diag base 16384 narrow all; mv $O/diag_base_16384_narrow.log $O/diag_def_16384n_$r.log
    GVL_GEMM_CFG=12 diag base 16384 narrow all; mv $O/diag_base_16384_narrow.log $O/diag_w4x_16384n_$r.log
  done
  ;;
r4p)  # LM step with the AGPR four-wave kernel on its N = 768 shapes (GVL_W4X=1) vs off, alternated
  for x in 1 0 1 0; do
    GVL_W4X=$x timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_x$x.json 2> $O/lm_x$x.err
    fatal $? bench_lm
    echo "lm w4x=$x $(python -c "import json;d=json.load(open('$O/lm_x$x.json'));r=d['roofline'];print(d['value'],d.get('step_mfma_frac'),[(g['kernel'][:40],g['ms_per_step'],g['avg_us']) for g in r['top_gemms'][:8]])")"
  done
  ;;
r4q)  # head check with the AGPR four-wave kernel on by default + refined hipBLASLt route: GPU suite,
      # smoke, the driver's default bench
  suite
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; fatal $? bench
  python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernel'],d['caption_qformer']['value'])"
  ;;
r4r)  # AGPR four-wave kernel: 128-row tiles on the caption decoder's N = 768 shapes (GVL_W4X_128) and
      # the batched weight gradients (GVL_W4X_DW): parity tests, shapes, step A/B
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "test_gemm_w4x or library_route or batched_wgrad" \
    --timeout 120 --timeout-method thread -p no:cacheprovider > $O/w4x_tests.log 2>&1; rc=$?; tail -3 $O/w4x_tests.log; fatal $rc w4x_tests
  for r in 1 2; do
    diag base 8064 narrow all; mv $O/diag_base_8064_narrow.log $O/diag_def_8064n_$r.log
    GVL_W4X_128=1 diag base 8064 narrow all; mv $O/diag_base_8064_narrow.log $O/diag_x128_8064n_$r.log
  done
  for x in 1 0 1 0; do
    GVL_W4X_DW=$x timeout -k 10 300 python -u tools/wgrad_diag.py > $O/wgrad_dw$x.log 2>&1; fatal $? wgrad; echo "dw=$x"; grep x12 $O/wgrad_dw$x.log
  done
  for x in 1 0 1 0; do
    GVL_W4X_128=$x timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_x$x.json 2> $O/qf_x$x.err
    fatal $? bench_qf
    echo "qformer w4x128=$x $(python -c "import json;d=json.load(open('$O/qf_x$x.json'));print(d['value'],d.get('step_mfma_frac'))")"
  done
  for x in 1 0 1 0; do
    GVL_W4X_DW=$x timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_dw$x.json 2> $O/lm_dw$x.err
    fatal $? bench_lm
    echo "lm w4x_dw=$x $(python -c "import json;d=json.load(open('$O/lm_dw$x.json'));r=d['roofline'];print(d['value'],d.get('step_mfma_frac'),[(g['kernel'][:44],g['ms_per_step'],g['avg_us']) for g in r['top_gemms'][:4]])")"
  done
  ;;
r4s)  # streaming stores for outputs past the MALL (GVL_PP3_NT) + w4x batched dW on full-round batches:
      # kernel tests, then LM step A/B of each
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "test_gemm_w4x or batched_wgrad or counted_epilogue or library_route" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > $O/kt.log 2>&1; rc=$?; tail -3 $O/kt.log; fatal $rc kernel_tests
  for v in "1 1" "0 1" "1 0" "1 1" "0 1" "1 0"; do set -- $v
    GVL_PP3_NT=$1 GVL_W4X_DW=$2 timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$1$2.json 2> $O/lm_$1$2.err
    fatal $? bench_lm
    echo "lm nt=$1 dw=$2 $(python -c "import json;d=json.load(open('$O/lm_$1$2.json'));r=d['roofline'];print(d['value'],d.get('step_mfma_frac'),[(g['kernel'][:44],g['ms_per_step'],g['avg_us']) for g in r['top_gemms'][:6]])")"
  done
  for v in 1 0 1 0; do
    GVL_PP3_NT=$v timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_nt$v.json 2> $O/qf_nt$v.err
    fatal $? bench_qf
    echo "qformer nt=$v $(python -c "import json;d=json.load(open('$O/qf_nt$v.json'));print(d['value'],d.get('step_mfma_frac'))")"
  done
  ;;
r4t)  # 256 x 256 AGPR tiles for the weight gradients (batched c_fc / mlp.c_proj, lm_head dW): tests, wgrad A/B, LM A/B
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "test_gemm_w4x or batched_wgrad" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > $O/kt.log 2>&1; rc=$?; tail -3 $O/kt.log; fatal $rc kernel_tests
  for x in 1 0; do
    GVL_W4X_DW=$x timeout -k 10 300 python -u tools/wgrad_diag.py > $O/wgrad_dw$x.log 2>&1; fatal $? wgrad; echo "dw=$x"; grep x12 $O/wgrad_dw$x.log | cut -c1-200
  done
  for x in 1 0 1 0; do
    GVL_W4X_DW=$x timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_dw$x.json 2> $O/lm_dw$x.err
    fatal $? bench_lm
    echo "lm w4x_dw=$x $(python -c "import json;d=json.load(open('$O/lm_dw$x.json'));r=d['roofline'];print(d['value'],d.get('step_mfma_frac'),[(g['kernel'][:48],g['ms_per_step'],g['avg_us']) for g in r['top_gemms'][:6]])")"
  done
  ;;
r4u)  # persistent AGPR four-wave kernel (gemm_w4p.hip) on the wide short-K shapes: parity tests, shapes, steps
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "test_gemm_w4p" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > $O/kt.log 2>&1; rc=$?; tail -3 $O/kt.log; fatal $rc kernel_tests
  for r in 1 2; do for M in 16384 8064; do
    diag base $M wide all; mv $O/diag_base_${M}_wide.log $O/diag_def_${M}_$r.log
    GVL_GEMM_CFG=13 diag base $M wide epi; mv $O/diag_base_${M}_wide.log $O/diag_w4p_${M}_$r.log
  done; done
  for x in 1 0 1 0; do
    GVL_W4P=$x timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_p$x.json 2> $O/lm_p$x.err
    fatal $? bench_lm
    echo "lm w4p=$x $(python -c "import json;d=json.load(open('$O/lm_p$x.json'));r=d['roofline'];print(d['value'],d.get('step_mfma_frac'),[(g['kernel'][:40],g['ms_per_step'],g['avg_us']) for g in r['top_gemms'][:8]])")"
  done
  for x in 1 0 1 0; do
    GVL_W4P=$x timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_p$x.json 2> $O/qf_p$x.err
    fatal $? bench_qf
    echo "qformer w4p=$x $(python -c "import json;d=json.load(open('$O/qf_p$x.json'));print(d['value'],d.get('step_mfma_frac'))")"
  done
  ;;
r4v|r4fin|r4fin2|r4fin3)  # head check: GPU suite + smoke, the driver's default bench, rocprofv3 kernel stats of both steps
  suite
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; fatal $? bench
  python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernel'],d['caption_qformer']['value'])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_qf -o qf -- \
    python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_qf.json 2> $O/prof_qf.err; fatal $? prof_qf
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lm -o lm -- \
    python bench.py --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > $O/prof_lm.json 2> $O/prof_lm.err; fatal $? prof_lm
  for w in qf lm; do f=$(find $O/prof_$w -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 40 > $O/${w}_table.txt; head -25 $O/${w}_table.txt; done
  ;;
r4x)  # bridge weight gradients deferred and flushed as ONE grouped AGPR launch (gvl_gemm_grouped):
      # grouped kernel test, GPU suite + smoke, then the Q-Former step A/B (GVL_DEFER_BRIDGE)
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "grouped or batched_wgrad" --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $O/kt.log 2>&1; rc=$?; tail -3 $O/kt.log; fatal $rc kernel_tests
  suite
  for x in 1 0 1 0; do
    GVL_DEFER_BRIDGE=$x timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_b$x.json 2> $O/qf_b$x.err
    fatal $? bench_qf
    echo "qformer defer_bridge=$x $(python -c "import json;d=json.load(open('$O/qf_b$x.json'));r=d['roofline'];print(d['value'],d.get('step_mfma_frac'),[(g['kernel'][:44],g['ms_per_step'],g['avg_us']) for g in r['top_gemms'][:6]])")"
  done
  ;;
r4y)  # the MHA in_proj row slices deferred into the grouped launch too (GVL_DEFER_INPROJ): grouped tests,
      # GPU suite + smoke, Q-Former step A/B (in_proj deferred / bridge deferred without in_proj / nothing)
  timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "grouped" --timeout 200 \
    --timeout-method thread -p no:cacheprovider > $O/kt.log 2>&1; rc=$?; tail -3 $O/kt.log; fatal $rc kernel_tests
  suite
  for v in "1 1" "1 0" "0 0" "1 1" "1 0" "0 0"; do set -- $v
    GVL_DEFER_BRIDGE=$1 GVL_DEFER_INPROJ=$2 timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf_$1$2.json 2> $O/qf_$1$2.err
    fatal $? bench_qf
    echo "qformer bridge=$1 inproj=$2 $(python -c "import json;d=json.load(open('$O/qf_$1$2.json'));print(d['value'],d.get('step_mfma_frac'))")"
  done
  ;;
r4z)  # rocprofv3 kernel stats of the Q-Former step at this head
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_qf -o qf -- \
    python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_qf.json 2> $O/prof_qf.err; fatal $? prof_qf
  f=$(find $O/prof_qf -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 45 > $O/qf_table.txt; cat $O/qf_table.txt
  ;;
r4db)  # fused bias sums of the batched AGPR dW without per-step branch joins: kernel tests, wgrad
       # (gvl vs gvl + dbias per shape), LM step twice
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "test_gemm_w4x or batched_wgrad or grouped" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > $O/kt.log 2>&1; rc=$?; tail -3 $O/kt.log; fatal $rc kernel_tests
  timeout -k 10 300 python -u tools/wgrad_diag.py > $O/wgrad.log 2>&1; fatal $? wgrad; grep x12 $O/wgrad.log | cut -c1-220
  for r in 1 2; do
    timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$r.json 2> $O/lm_$r.err
    fatal $? bench_lm
    echo "lm $(python -c "import json;d=json.load(open('$O/lm_$r.json'));r=d['roofline'];print(d['value'],d.get('step_mfma_frac'),[(g['kernel'][:48],g['ms_per_step'],g['avg_us']) for g in r['top_gemms'][:6]])")"
  done
  timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/qf.json 2> $O/qf.err; fatal $? bench_qf
  echo "qformer $(python -c "import json;d=json.load(open('$O/qf.json'));print(d['value'],d.get('step_mfma_frac'))")"
  ;;
r4g48)  # every LM weight gradient of a flush as ONE grouped launch (GVL_GROUPED_WGRAD=2, 48 problems):
        # grouped kernel tests, wgrad (grouped vs the four batches), LM / caption step A/B, GPU suite
  timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "grouped or batched_wgrad or test_gemm_w4x" \
    --timeout 200 --timeout-method thread -p no:cacheprovider > $O/kt.log 2>&1; rc=$?; tail -3 $O/kt.log; fatal $rc kernel_tests
  timeout -k 10 300 python -u tools/wgrad_diag.py > $O/wgrad.log 2>&1; fatal $? wgrad; cut -c1-200 $O/wgrad.log
  for g in 2 1 2 1; do
    GVL_GROUPED_WGRAD=$g timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_g$g.json 2> $O/lm_g$g.err
    fatal $? bench_lm
    echo "lm grouped=$g $(python -c "import json;d=json.load(open('$O/lm_g$g.json'));r=d['roofline'];print(d['value'],d.get('step_mfma_frac'),[(g['kernel'][:48],g['ms_per_step'],g['avg_us']) for g in r['top_gemms'][:4]])")"
  done
  for w in qformer cross; do for g in 2 1; do
    GVL_GROUPED_WGRAD=$g timeout -k 10 300 python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/${w}_g$g.json 2> $O/${w}_g$g.err
    fatal $? bench_$w
    echo "$w grouped=$g $(python -c "import json;d=json.load(open('$O/${w}_g$g.json'));print(d['value'],d.get('step_mfma_frac'))")"
  done; done
  suite
  ;;
r4dbs)  # bias sums spread over the column blocks (libgvl_dbs1.so: GVL_W4X_DBSPREAD) vs the shipped
        # build (all in column block 0): dbias kernel tests on the variant, wgrad per family, LM A/B
  GVL_LIB=$LIBDIR/libgvl_dbs1.so timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -q -x \
    -k "grouped or batched_wgrad or test_gemm_w4x" --timeout 200 --timeout-method thread -p no:cacheprovider > $O/kt.log 2>&1
  rc=$?; tail -3 $O/kt.log; fatal $rc kernel_tests
  for v in dbs1 base dbs1 base; do
    L=$LIBDIR/libgvl_$v.so; [ $v = base ] && L=$LIBDIR/libgvl.so
    GVL_LIB=$L timeout -k 10 300 python -u tools/wgrad_diag.py > $O/wgrad_$v.log 2>&1; fatal $? wgrad
    echo "== $v"; grep x12 $O/wgrad_$v.log | cut -c1-112
  done
  for v in dbs1 base dbs1 base; do
    L=$LIBDIR/libgvl_$v.so; [ $v = base ] && L=$LIBDIR/libgvl.so
    GVL_LIB=$L timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline > $O/lm_$v.json 2> $O/lm_$v.err
    fatal $? bench_lm
    echo "lm $v $(python -c "import json;d=json.load(open('$O/lm_$v.json'));r=d['roofline'];print(d['value'],d.get('step_mfma_frac'),[(g['kernel'][:48],g['ms_per_step'],g['avg_us']) for g in r['top_gemms'][:3]])")"
  done
  ;;
r4ln)  # LayerNorm forward with 2 / 4 rows per half-wave in flight (GVL_LN_RPH builds): LN tests on each,
       # launch times at the bench shapes, alternated
  for v in ln2 ln4; do
    GVL_LIB=$LIBDIR/libgvl_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "layernorm" \
      --timeout 120 --timeout-method thread -p no:cacheprovider > $O/kt_$v.log 2>&1; rc=$?; tail -1 $O/kt_$v.log; fatal $rc ln_tests
  done
  for v in base ln2 ln4 base ln2 ln4; do
    L=$LIBDIR/libgvl_$v.so; [ $v = base ] && L=$LIBDIR/libgvl.so
    GVL_LIB=$L timeout -k 10 200 python -u tools/ln_one.py > $O/ln_$v.log 2>&1; fatal $? ln_one
    echo "== $v"; grep ln_ $O/ln_$v.log
  done
  ;;
r4lnb|r4lnb2)  # LayerNorm backward block count (GVL_LN_BWD_MAXB builds vs 1024): LN tests, launch times
  V1="lnb512 lnb2048"; V2="base lnb512 lnb2048 base lnb512 lnb2048"
  [ $S = r4lnb2 ] && V1="lnb256 lnb384" && V2="base lnb512 lnb256 lnb384 base lnb512 lnb256 lnb384"
  for v in $V1; do
    GVL_LIB=$LIBDIR/libgvl_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -q -x -k "layernorm" \
      --timeout 120 --timeout-method thread -p no:cacheprovider > $O/kt_$v.log 2>&1; rc=$?; tail -1 $O/kt_$v.log; fatal $rc ln_tests
  done
  for v in $V2; do
    L=$LIBDIR/libgvl_$v.so; [ $v = base ] && L=$LIBDIR/libgvl.so
    GVL_LIB=$L timeout -k 10 200 python -u tools/ln_one.py > $O/ln_$v.log 2>&1; fatal $? ln_one
    echo "== $v"; grep ln_bwd $O/ln_$v.log
  done
  ;;
r4lnc)  # LayerNorm backward 512 (shipped) vs 1024 blocks (libgvl_lnb1024.so) inside the steps, same box, alternated
  for w in qformer lm; do for v in base lnb1024 base lnb1024; do
    L=$LIBDIR/libgvl_$v.so; [ $v = base ] && L=$LIBDIR/libgvl.so
    a="--workload qformer --steps 10 --warmup 3"; [ $w = lm ] && a="--steps 2 --warmup 1 --no-secondary"
    GVL_LIB=$L timeout -k 10 300 python bench.py $a --no-cpu-baseline > $O/${w}_$v.json 2> $O/${w}_$v.err; fatal $? bench_$w
    echo "$w $v $(python -c "import json;d=json.load(open('$O/${w}_$v.json'));print(d['value'],d.get('step_mfma_frac'))")"
  done; done
  ;;
*) echo "unknown session $S"; exit 2;;
esac
