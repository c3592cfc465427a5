#!/bin/bash
# Round-5 GPU sessions (run on the GPU box through gpurun): bash tools/r5_sessions.sh <name>.
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
ktests() {  # ktests <log> <pytest -k expression> [file]
  timeout -k 10 600 python -u -m pytest ${3:-tests/test_gpu_kernels.py} -q -x -k "$2" --timeout 300 \
    --timeout-method thread -p no:cacheprovider > $O/$1.log 2>&1; rc=$?; echo "$1: $(tail -1 $O/$1.log)"; fatal $rc $1
}
diag() {  # diag <tag> <M> <set> <cols>   (env passes through)
  GVL_DIAG_COLS=$4 timeout -k 10 240 python -u tools/gemm_diag.py $2 $3 > $O/diag_$1_$2_$3.log 2>&1
  rc=$?; echo "== $1 M=$2 $3"; grep "N=" $O/diag_$1_$2_$3.log; fatal $rc diag
}
bench() {  # bench <tag> <workload> [steps]   (env passes through)
  local a="--workload $2 --steps ${3:-10} --warmup 3"; [ $2 = lm ] && a="--steps ${3:-2} --warmup 1 --no-secondary"
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $O/$1.json 2> $O/$1.err; fatal $? bench_$1
  echo "$1 $(python -c "import json;d=json.load(open('$O/$1.json'));print(d['value'],d.get('step_mfma_frac'))")"
}
case $S in
r5a)  # gated four-wave epilogue (cross-att xattn.c_proj), grouped single problem, hipBLASLt-off A/B
  [ -n "$SKIP_KT" ] || ktests kt "w4_gated or grouped_wgrad or gemm_dropout_gate or test_gemm_w4x"
  ktests dp "two_ranks" tests/test_gpu_dp.py
  for r in 1 2; do for g in 1 0; do GVL_W4_GATE=$g bench cross_g${g}_$r cross; done; done
  for r in 1 2; do
    bench qf_lib1_$r qformer
    GVL_GEMM_LIB=0 bench qf_lib0_$r qformer
    GVL_GEMM_LIB=0 GVL_W4X_128=1 bench qf_lib0x128_$r qformer
  done
  for M in 8064 4096; do
    diag lib1 $M narrow all
    GVL_GEMM_LIB=0 diag lib0 $M narrow epi
    GVL_GEMM_LIB=0 GVL_W4X_128=1 diag lib0x128 $M narrow epi
  done
  ;;
r5b)  # hipBLASLt gone (ABI v10), AGPR kernel's in-launch K split for the N = 768 products
  ktests kt "w4x_split or w4_gated or caption_dx or strided_output or test_gemm_w4x or tile128x192 or splitk_combined or grouped_wgrad or test_gemm_w4 or bias_dropout_residual"
  for r in 1 2; do for v in 1 0; do GVL_W4X_SPLIT=$v bench qf_s${v}_$r qformer; done; done
  for v in 1 0; do GVL_W4X_SPLIT=$v bench lin_s${v} linear; GVL_W4X_SPLIT=$v bench cross_s${v} cross; done
  for M in 8064 4096; do for v in 1 0; do GVL_W4X_SPLIT=$v diag s$v $M narrow epi; done; done
  ;;
r5c)  # two-slice split (GVL_W4X_SPLIT=1) A/B; attention row max by lane swaps A/B; Q-Former grad scale
  ktests kt "w4x_split or caption_dx or test_gemm_w4x or tile128x192 or attention"
  for v in 1 0 1 0; do GVL_W4X_SPLIT=$v diag s$v 8064 narrow epi; done
  for r in 1 2; do for v in 1 0; do GVL_W4X_SPLIT=$v bench qf_s${v}_$r qformer; done; done
  for r in 1 2; do for L in base shfl; do
    LIB=$LIBDIR/libgvl.so; [ $L = shfl ] && LIB=$LIBDIR/libgvl_shfl.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/attn_one.py 20 > $O/attn_${L}_$r.log 2>&1; fatal $? attn
    echo "attn $L $r"; head -3 $O/attn_${L}_$r.log
  done; done
  GVL_MARGINS_DIR=$O/parity_margins ktests bench_parity "qformer" tests/test_gpu_parity_bench.py
  ;;
r5d)  # attention row max by lane swaps vs ds_bpermute (libgvl_shfl.so) A/B; Q-Former grad scale
  ktests kt "attention or attn or caption_dx or test_gemm_w4x or tile128x192"
  for r in 1 2; do for L in base shfl; do
    LIB=$LIBDIR/libgvl.so; [ $L = shfl ] && LIB=$LIBDIR/libgvl_shfl.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/attn_one.py 20 > $O/attn_${L}_$r.log 2>&1; fatal $? attn
    echo "attn $L $r"; grep "B=" $O/attn_${L}_$r.log | head -3
  done; done
  for r in 1 2; do for L in base shfl; do
    LIB=$LIBDIR/libgvl.so; [ $L = shfl ] && LIB=$LIBDIR/libgvl_shfl.so
    GVL_LIB=$LIB bench lm_${L}_$r lm
  done; done
  GVL_MARGINS_DIR=$O/parity_margins ktests bench_parity "qformer" tests/test_gpu_parity_bench.py
  bash tools/pmc_attn.sh $S; fatal $? pmc_attn
  ;;
r5e)  # attention LDS reads software-pipelined (fwd V, dQ K^T, dK/dV lse/D) vs r5d's (libgvl_att0.so)
  ktests kt "attention or attn" tests/test_gpu_kernels.py
  for r in 1 2 3; do for L in base att0; do
    LIB=$LIBDIR/libgvl.so; [ $L = att0 ] && LIB=$LIBDIR/libgvl_att0.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_${L}_$r.log 2>&1; fatal $? attn
    echo "attn $L $r"; grep "B=" $O/attn_${L}_$r.log | head -2
  done; done
  GVL_MARGINS_DIR=$O/parity_margins ktests bench_parity "linear or cross or lm" tests/test_gpu_parity_bench.py
  ;;
r5f)  # Q-Former gradient probes vs the reference
  GVL_MARGINS_DIR=$O/parity_margins ktests probe "grad_probe" tests/test_gpu_parity_bench.py
  python -c "import json;print(json.dumps(json.load(open('$O/parity_margins/qformer_grad_probe.json')),indent=1))"
  ;;
r5g|r5fin|r5fin2|r5fin3|r5fin4|r5fin5|r5fin6)  # head check: GPU suite + smoke, the driver's default bench, rocprofv3 kernel stats of all four steps
  suite
  timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err; fatal $? bench
  python -c "import json;d=json.load(open('$O/bench.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernel'],[(k,d[k]['value']) for k in d if k.startswith('caption')])"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_qf -o qf -- \
    python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_qf.json 2> $O/prof_qf.err; fatal $? prof_qf
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lm -o lm -- \
    python bench.py --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > $O/prof_lm.json 2> $O/prof_lm.err; fatal $? prof_lm
  for w in cross linear; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$w -o $w -- \
      python bench.py --workload $w --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_$w.json 2> $O/prof_$w.err; fatal $? prof_$w
  done
  for w in qf lm cross linear; do f=$(find $O/prof_$w -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 40 > $O/${w}_table.txt; head -12 $O/${w}_table.txt; done
  ;;
r5h)  # linear decoder's 8192-row N = 768 GEMMs on 128-row AGPR tiles (GVL_W4X_128=2 default) vs 0
  ktests kt "linear_decoder_rows or test_gemm_w4x or tile128x192 or caption_dx"
  GVL_MARGINS_DIR=$O/parity_margins ktests bench_parity "bench_shape" tests/test_gpu_parity_bench.py
  for r in 1 2; do for v in 2 0; do GVL_W4X_128=$v bench lin_x${v}_$r linear; done; done
  for v in 2 0; do GVL_W4X_128=$v bench qf_x${v} qformer; done
  for v in 2 0; do GVL_W4X_128=$v diag x$v 8192 narrow epi; done
  ;;
r5i)  # N = 768 shapes at the cross decoder's 3968 rows and the Q-Former bridge's 4096: default vs 128-row direct-A
  for M in 3968 4096; do for v in 1 2; do GVL_W4D=$v diag w4d$v $M narrow epi; done; done
  ;;
r5j)  # wide K = 768 GEMMs: row sweep (fixed vs per-tile cost), shipped / d1 (plain stores) / d2 (no stores); attention G A/B
  for L in base d1 d2; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB timeout -k 10 240 python -u tools/pp3_sweep.py > $O/sweep_$L.log 2>&1; fatal $? sweep_$L
    echo "== $L"; cat $O/sweep_$L.log
  done
  for r in 1 2; do for G in 0 1; do
    if [ $G = 1 ]; then export GVL_ATTN_G=1; else unset GVL_ATTN_G; fi
    timeout -k 10 200 python -u tools/attn_one.py 20 > $O/attn_g${G}_$r.log 2>&1; fatal $? attn
    echo "attn G=$G $r"; grep "B=" $O/attn_g${G}_$r.log | head -2
  done; done
  unset GVL_ATTN_G
  ;;
r5k)  # LM weight gradients: c_attn / c_fc / mlp.c_proj batches + the lm_head dW as ONE grouped launch (whole rounds)
  GVL_WGRAD_LM=1 timeout -k 10 400 python -u tools/wgrad_diag.py > $O/wgrad_lm.log 2>&1; rc=$?; cat $O/wgrad_lm.log | grep -v amdgpu.ids; fatal $rc wgrad
  ;;
r5l)  # the tied lm_head's dW deferred and grouped with the blocks' (ABI v11 device scale per problem)
  ktests kt "grouped or w4x or wgrad"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "lm" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "lm" tests/test_gpu_parity_full.py
  ktests dp "lm or overlap" tests/test_gpu_dp.py
  ktests bnd "" tests/test_gpu_boundary.py
  for r in 1 2; do for v in 1 0; do GVL_DEFER_LMHEAD=$v bench lm_d${v}_$r lm; done; done
  ;;
r5m)  # wide K = 768 plain products on the AGPR four-wave kernel (GVL_W4X=2) vs the persistent kernel
  for v in 1 2 1 2; do GVL_W4X=$v timeout -k 10 240 python -u tools/pp3_sweep.py > $O/sweep_w4x$v.log 2>&1; fatal $? sweep; echo "== GVL_W4X=$v"; grep -v amdgpu.ids $O/sweep_w4x$v.log; done
  ;;
r5o)  # kernel trace (sequence) of the LM step
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace_lm -o lm -- \
    python bench.py --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > $O/trace_lm.json 2> $O/trace_lm.err; fatal $? trace_lm
  ;;
r5n)  # kernel traces (sequence) of one graphed Q-Former / cross / linear step
  for w in qformer cross; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$w -o $w -- \
      python bench.py --workload $w --steps 2 --warmup 2 --no-cpu-baseline > $O/trace_$w.json 2> $O/trace_$w.err; fatal $? trace_$w
  done
  ;;
r5p)  # LayerNorm weight grads deferred, one batched finalize per flush (ABI v12); LM trace
  ktests kt "layernorm or grouped"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "bench_shape" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "full_size or accumulation" tests/test_gpu_parity_full.py
  ktests dp "" tests/test_gpu_dp.py
  ktests bnd "" tests/test_gpu_boundary.py
  for r in 1 2; do for v in 1 0; do GVL_DEFER_LN=$v bench lm_ln${v}_$r lm; GVL_DEFER_LN=$v bench qf_ln${v}_$r qformer; done; done
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace_lm -o lm -- \
    python bench.py --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > $O/trace_lm.json 2> $O/trace_lm.err; fatal $? trace_lm
  ;;
r5q)  # LM N = 768 shapes at 16384 rows: model epilogue vs plain (w4x), both B layouts
  for r in 1 2; do diag r$r 16384 narrow all; done
  ;;
r5r)  # residual folded into the AGPR accumulators at tile start (w4x bias + residual) vs libgvl_nofold.so
  ktests kt "w4x or residual or tile128x192 or caption_dx"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "bench_shape" tests/test_gpu_parity_bench.py
  for r in 1 2; do for L in base nofold; do
    LIB=$LIBDIR/libgvl.so; [ $L = nofold ] && LIB=$LIBDIR/libgvl_nofold.so
    GVL_LIB=$LIB diag ${L}_$r 16384 narrow epi
  done; done
  for r in 1 2; do for L in base nofold; do
    LIB=$LIBDIR/libgvl.so; [ $L = nofold ] && LIB=$LIBDIR/libgvl_nofold.so
    GVL_LIB=$LIB bench lm_${L}_$r lm
  done; done
  ;;
r5s)  # cross-entropy cache policy: nontemporal dlogits stores / logit loads (variant builds)
  for r in 1 2; do for L in base cest celd ceboth; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/ce_one.py > $O/ce_${L}_$r.log 2>&1; fatal $? ce
    echo "$L $r: $(grep rows= $O/ce_${L}_$r.log | tr '\n' ' ')"
  done; done
  ;;
r5t)  # cross-entropy nontemporal loads + stores (libgvl_ceboth.so) in the steps
  for r in 1 2 3; do for L in base ceboth; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB bench qf_${L}_$r qformer
    GVL_LIB=$LIB bench lm_${L}_$r lm
  done; done
  ;;
r5u)  # short-sequence attention backward: all global loads issued before the first wait (vs libgvl_old.so)
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "qformer or linear or cross" tests/test_gpu_parity_bench.py
  for r in 1 2 3; do for L in base old; do
    LIB=$LIBDIR/libgvl.so; [ $L = old ] && LIB=$LIBDIR/libgvl_old.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_${L}_$r.log 2>&1; fatal $? attn
    echo "attn $L $r"; grep "B=128" $O/attn_${L}_$r.log
  done; done
  for r in 1 2; do for L in base old; do
    LIB=$LIBDIR/libgvl.so; [ $L = old ] && LIB=$LIBDIR/libgvl_old.so
    GVL_LIB=$LIB bench qf_${L}_$r qformer; GVL_LIB=$LIB bench cross_${L}_$r cross
  done; done
  ;;
r5v)  # 8-wide dropout-apply / gate-backward, pooling window loads unrolled (vs libgvl_old.so)
  ktests kt "colsum_dropout_gate or pool_clip or attention_short or gated"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "qformer or cross or linear" tests/test_gpu_parity_bench.py
  for r in 1 2 3; do for L in base old; do
    LIB=$LIBDIR/libgvl.so; [ $L = old ] && LIB=$LIBDIR/libgvl_old.so
    GVL_LIB=$LIB bench qf_${L}_$r qformer; GVL_LIB=$LIB bench cross_${L}_$r cross
  done; done
  ;;
r5w)  # cross-att gate gradient accumulated into its bf16 grad by the gate kernel (ABI v13) vs GVL_GATE_SINK=0
  ktests kt "colsum_dropout_gate or gated"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "cross" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "cross" tests/test_gpu_parity_full.py
  ktests capi "" tests/test_capi.py
  for r in 1 2 3; do for v in 1 0; do GVL_GATE_SINK=$v bench cross_g${v}_$r cross; done; done
  ;;
r5x)  # cross-att kv_proj stacked in the optimizer arena (view instead of torch.cat per step)
  ktests models "cross" tests/test_gpu_models.py
  ktests dp "" tests/test_gpu_dp.py
  ktests bnd "" tests/test_gpu_boundary.py
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "cross" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "cross" tests/test_gpu_parity_full.py
  for r in 1 2 3; do bench cross_$r cross; done
  ;;
r5y)  # CE finalize loads unrolled; kernel traces (sequence) of all four steps at head
  ktests kt "cross_entropy or lm_head"
  for w in qformer cross linear; do
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_$w -o $w -- \
      python bench.py --workload $w --steps 2 --warmup 2 --no-cpu-baseline > $O/trace_$w.json 2> $O/trace_$w.err; fatal $? trace_$w
  done
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace_lm -o lm -- \
    python bench.py --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > $O/trace_lm.json 2> $O/trace_lm.err; fatal $? trace_lm
  ;;
r5z)  # software-pipelined attention forward (S(kt+1) || exp(kt)) vs attn_fwd_dma_kernel (GVL_ATTN_FWD_PIPE=0); CE finalize
  ktests kt "attention or attn or cross_entropy"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "lm" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "lm" tests/test_gpu_parity_full.py
  for r in 1 2; do for v in 1 0; do
    GVL_ATTN_FWD_PIPE=$v timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_p${v}_$r.log 2>&1; fatal $? attn
    echo "attn pipe=$v $r"; grep "B=16" $O/attn_p${v}_$r.log
  done; done
  for r in 1 2; do for v in 1 0; do GVL_ATTN_FWD_PIPE=$v bench lm_p${v}_$r lm; done; done
  ;;
r5z2)  # pipelined forward: 3-slot ring (default build) vs 4-slot (libgvl_p4.so), picked G vs G = 1
  ktests kt "attention or attn"
  GVL_ATTN_FWD_PIPE=2 ktests kt2 "attention or attn"
  GVL_LIB=$LIBDIR/libgvl_p4.so GVL_ATTN_FWD_PIPE=2 ktests kt3 "attention or attn"
  for r in 1 2; do for L in base p4; do for v in 0 1 2; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB GVL_ATTN_FWD_PIPE=$v timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_${L}_${v}_$r.log 2>&1; fatal $? attn
    echo "attn $L pipe=$v $r: $(grep B=16 $O/attn_${L}_${v}_$r.log)"
  done; done; done
  ;;
r5y2)  # CE finalize: branch-free row loads, mask presence as a template argument
  ktests kt "cross_entropy or lm_head"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "lm or cross or linear" tests/test_gpu_parity_bench.py
  ktests models "forward_loss or masked" tests/test_gpu_models.py
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lm -o lm -- \
    python bench.py --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > $O/prof_lm.json 2> $O/prof_lm.err; fatal $? prof_lm
  f=$(find $O/prof_lm -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 40 > $O/lm_table.txt; grep -E "ce_|emb_" $O/lm_table.txt
  ;;
r5ln)  # persistent LayerNorm forward (next row's loads before this row's stores) vs the one-shot grid
  for L in p512 p1024 p2048; do GVL_LIB=$LIBDIR/libgvl_$L.so ktests kt_$L "layernorm"; done
  for r in 1 2; do for L in base p512 p1024 p2048; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/ln_one.py > $O/ln_${L}_$r.log 2>&1; fatal $? ln
    echo "$L $r"; grep ln_fwd $O/ln_${L}_$r.log
  done; done
  ;;
r5e2)  # persistent LayerNorm forward (default), embedding backward run-head loads overlapped: tests + LM / Q-Former steps + LM kernel table
  ktests kt "layernorm or embedding or embed"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "lm or accumulation" tests/test_gpu_parity_full.py
  for r in 1 2; do bench lm_$r lm; bench qf_$r qformer; done
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lm -o lm -- \
    python bench.py --steps 1 --warmup 1 --no-secondary --no-cpu-baseline > $O/prof_lm.json 2> $O/prof_lm.err; fatal $? prof_lm
  f=$(find $O/prof_lm -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 40 > $O/lm_table.txt; grep -E "ln_|emb_" $O/lm_table.txt
  ;;
r5aq)  # attention prologues: fragment loads + first DMAs in one round trip, branch-free dQ prologue (vs libgvl_old.so)
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "" tests/test_gpu_parity_full.py
  for r in 1 2 3; do for L in base old; do
    LIB=$LIBDIR/libgvl.so; [ $L = old ] && LIB=$LIBDIR/libgvl_old.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_${L}_$r.log 2>&1; fatal $? attn
    echo "attn $L $r: $(grep 'B=16 ' $O/attn_${L}_$r.log)"; grep "B=128 H=12 Tq=32 Tk=257" $O/attn_${L}_$r.log
  done; done
  for r in 1 2; do for L in base old; do
    LIB=$LIBDIR/libgvl.so; [ $L = old ] && LIB=$LIBDIR/libgvl_old.so
    GVL_LIB=$LIB bench lm_${L}_$r lm; GVL_LIB=$LIB bench qf_${L}_$r qformer
  done; done
  ;;
r5pl)  # 16-B CLIP pooling (pool4_kernel), coalesced LayerNorm finalize (64 columns x 16 groups) vs libgvl_old.so
  ktests kt "layernorm or pool"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "" tests/test_gpu_parity_full.py
  for r in 1 2; do for L in base old; do
    LIB=$LIBDIR/libgvl.so; [ $L = old ] && LIB=$LIBDIR/libgvl_old.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/ln_one.py > $O/ln_${L}_$r.log 2>&1; fatal $? ln
    echo "$L $r"; grep ln_bwd $O/ln_${L}_$r.log
  done; done
  for r in 1 2; do for L in base old; do
    LIB=$LIBDIR/libgvl.so; [ $L = old ] && LIB=$LIBDIR/libgvl_old.so
    GVL_LIB=$LIB bench qf_${L}_$r qformer; GVL_LIB=$LIB bench cross_${L}_$r cross; GVL_LIB=$LIB bench lm_${L}_$r lm
  done; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_qf -o qf -- \
    python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_qf.json 2> $O/prof_qf.err; fatal $? prof_qf
  f=$(find $O/prof_qf -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 40 > $O/qf_table.txt; grep -E "pool|ln_" $O/qf_table.txt
  ;;
r5pl2)  # 16-B CLIP pooling for 12-patch windows too (side 14: the linear bridge's features)
  ktests kt "pool"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "linear or qformer" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests edge "edge" tests/test_gpu_parity_full.py
  for r in 1 2; do bench lin_$r linear; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lin -o lin -- \
    python bench.py --workload linear --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_lin.json 2> $O/prof_lin.err; fatal $? prof_lin
  f=$(find $O/prof_lin -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 40 > $O/lin_table.txt; grep -E "pool" $O/lin_table.txt
  ;;
r5dpp)  # LayerNorm / CE row reductions by DPP + lane swaps (no ds_bpermute) vs libgvl_nodpp.so; 16-B pooling at side 14
  ktests kt "layernorm or pool or cross_entropy or lm_head"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "" tests/test_gpu_parity_full.py
  for r in 1 2; do for L in base nodpp; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/ln_one.py > $O/ln_${L}_$r.log 2>&1; fatal $? ln
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/ce_one.py > $O/ce_${L}_$r.log 2>&1; fatal $? ce
    echo "$L $r"; cat $O/ln_${L}_$r.log | grep -v amdgpu.ids; grep rows= $O/ce_${L}_$r.log
  done; done
  for r in 1 2; do for L in base nodpp; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB bench qf_${L}_$r qformer; GVL_LIB=$LIB bench cross_${L}_$r cross; GVL_LIB=$LIB bench lin_${L}_$r linear; GVL_LIB=$LIB bench lm_${L}_$r lm
  done; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_lin -o lin -- \
    python bench.py --workload linear --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_lin.json 2> $O/prof_lin.err; fatal $? prof_lin
  f=$(find $O/prof_lin -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 40 > $O/lin_table.txt; grep -E "pool|ln_" $O/lin_table.txt
  ;;
r5sw)  # attention D / row-sum lane reductions by VALU swaps (bit-identical) vs libgvl_old.so
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "" tests/test_gpu_parity_bench.py
  for r in 1 2 3; do for L in base old; do
    LIB=$LIBDIR/libgvl.so; [ $L = old ] && LIB=$LIBDIR/libgvl_old.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_${L}_$r.log 2>&1; fatal $? attn
    echo "attn $L $r"; grep -v amdgpu.ids $O/attn_${L}_$r.log
  done; done
  for r in 1 2; do for L in base old; do
    LIB=$LIBDIR/libgvl.so; [ $L = old ] && LIB=$LIBDIR/libgvl_old.so
    GVL_LIB=$LIB bench qf_${L}_$r qformer; GVL_LIB=$LIB bench cross_${L}_$r cross
  done; done
  ;;
r5l32)  # short-sequence attention backward in 32 KiB of LDS (P / dS over V / K): 5 blocks per CU vs 3 (libgvl_l48.so)
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "" tests/test_gpu_parity_full.py
  for r in 1 2 3; do for L in base l48; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_${L}_$r.log 2>&1; fatal $? attn
    echo "attn $L $r"; grep "B=128" $O/attn_${L}_$r.log
  done; done
  for r in 1 2; do for L in base l48; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB bench qf_${L}_$r qformer; GVL_LIB=$LIB bench cross_${L}_$r cross; GVL_LIB=$LIB bench lin_${L}_$r linear
  done; done
  ;;
r5pf)  # LayerNorm backward two rows in flight ahead (GVL_LN_BWD_PF=2) vs one (libgvl_pf1.so)
  ktests kt "layernorm"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "" tests/test_gpu_parity_bench.py
  for r in 1 2; do for L in base pf1; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/ln_one.py > $O/ln_${L}_$r.log 2>&1; fatal $? ln
    echo "$L $r"; grep ln_bwd $O/ln_${L}_$r.log
  done; done
  for r in 1 2; do for L in base pf1; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB bench qf_${L}_$r qformer; GVL_LIB=$LIB bench cross_${L}_$r cross; GVL_LIB=$LIB bench lm_${L}_$r lm
  done; done
  ;;
r5one)  # single-tile short forward (16 KiB, 6 waves/SIMD; libgvl_w5.so: 5) vs the two-stage kernel (GVL_ATTN_FWD_ONE=0)
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "" tests/test_gpu_parity_full.py
  for r in 1 2 3; do for v in base w5 off; do
    LIB=$LIBDIR/libgvl.so; [ $v = w5 ] && LIB=$LIBDIR/libgvl_w5.so; ONE=1; [ $v = off ] && ONE=0
    GVL_LIB=$LIB GVL_ATTN_FWD_ONE=$ONE timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_${v}_$r.log 2>&1; fatal $? attn
    echo "attn $v $r"; grep -E "Tq=63|Tq=31" $O/attn_${v}_$r.log
  done; done
  for r in 1 2; do for v in base off; do
    ONE=1; [ $v = off ] && ONE=0
    GVL_ATTN_FWD_ONE=$ONE bench qf_${v}_$r qformer; GVL_ATTN_FWD_ONE=$ONE bench cross_${v}_$r cross; GVL_ATTN_FWD_ONE=$ONE bench lin_${v}_$r linear
  done; done
  ;;
*) echo "unknown session $S"; exit 2 ;;
esac
