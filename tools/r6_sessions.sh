#!/bin/bash
# Round-6 GPU sessions (run on the GPU box through gpurun): bash tools/r6_sessions.sh <name>.
# Every GPU step has its own time limit; a session stops at the first failing step.
# Each session names the bound it tests (only levers with a committed
# predicted gain >= 3 % of a step get GPU minutes).
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
bench() {  # bench <tag> <workload> [steps]   (env passes through)
  local a="--workload $2 --steps ${3:-10} --warmup 3"; [ $2 = lm ] && a="--steps ${3:-2} --warmup 1 --no-secondary"
  timeout -k 10 300 python bench.py $a --no-cpu-baseline > $O/$1.json 2> $O/$1.err; fatal $? bench_$1
  echo "$1 $(python -c "import json;d=json.load(open('$O/$1.json'));print(d['value'],d.get('step_mfma_frac'),d.get('peak_hbm_gib'))")"
}
case $S in
r6pp)  # PMC of the wide K = 768 class at the Q-Former shape (8064 x 3072 x 768): c_fc + GELU with its
       # gelu' side output (act) vs the plain product — where the un-overlapped stores' time goes
       # (evidence for the next round's plan; no code change)
  EPI=act timeout -k 10 600 bash tools/pmc_gemm.sh pp3act_r6pp "8064 3072 768 0 0 3 -1"; fatal $? pmc_act
  EPI=plain timeout -k 10 600 bash tools/pmc_gemm.sh pp3plain_r6pp "8064 3072 768 0 0 3 -1"; fatal $? pmc_plain
  for t in pp3act_r6pp pp3plain_r6pp; do for pn in 1 2 3; do echo "== $t pass $pn"; python tools/pmc_summary.py gpurun_out/pmc_$t/c1_p$pn; done; grep -v amdgpu.ids gpurun_out/pmc_$t/times.log; done > $O/pmc_summary.txt 2>&1
  cat $O/pmc_summary.txt
  ;;
r6z)  # residual folded into the direct-A kernel's accumulators (GVL_W4D_FOLD, as the LM's w4x): the
      # caption decoders' bias + residual forward N = 768 GEMMs (22.0 / 56.1 us at K = 768 / 3072 vs
      # the plain product's 17.9 / 49.0). Bound: w4d<false, 2> is 11.7 % of the Q-Former step; half
      # the gap back = ~0.8 %. A/B against libgvl_nofold.so.
  ktests kt "w4 or gated or dropout_residual or linear_decoder or caption"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "qformer or linear" tests/test_gpu_parity_bench.py
  ktests full "qformer" tests/test_gpu_parity_full.py
  for r in 1 2; do for v in nofold new; do for K in 768 3072; do
    L=$LIBDIR/libgvl.so; [ $v = nofold ] && L=$LIBDIR/libgvl_nofold.so
    GVL_LIB=$L timeout -k 10 120 python tools/gemm_one.py 8064 768 $K 0 0 3 -1 20 bias_res > $O/g_${v}_${K}_$r.log 2>&1; fatal $? g
    echo "$v K=$K $r $(grep -v amdgpu.ids $O/g_${v}_${K}_$r.log | tail -1)"
  done; done; done
  for r in 1 2 3; do for v in nofold new; do
    L=$LIBDIR/libgvl.so; [ $v = nofold ] && L=$LIBDIR/libgvl_nofold.so
    GVL_LIB=$L bench qf_${v}_$r qformer
  done; done
  ;;
r6y)  # rehearsal of the driver's N = 2 bench path on the one-GPU box (GVL_BENCH_ONE_DEVICE=1: both ranks
      # on cuda:0, collectives over gloo; never a bench line): the DP buckets, the max-over-ranks
      # timing and the library-owned teardown (gvl.dist.destroy_process_group) end to end
  for w in qformer lm; do
    a="--workload $w --steps 2 --warmup 1"; [ $w = lm ] && a="--steps 1 --warmup 1 --no-secondary"
    GVL_BENCH_ONE_DEVICE=1 timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
      --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 2 $a --no-cpu-baseline > $O/n2_$w.json 2> $O/n2_$w.err
    rc=$?; echo "n2 $w rc=$rc $(tail -c 400 $O/n2_$w.json)"; fatal $rc n2_$w
  done
  ;;
r6x)  # s_setprio(1) around the T > 64 attention kernels' MFMA clusters (libgvl_prio.so, GVL_ATTN_PRIO=1):
      # the guide's T5 (null to +6 % where hipcc moves MFMAs across barriers). Bound: attention is
      # 14 % of the LM step -> a few % of it = ~0.3-0.8 %. attn_one + LM alternated.
  for r in 1 2; do for v in base prio; do
    L=$LIBDIR/libgvl.so; [ $v = prio ] && L=$LIBDIR/libgvl_prio.so
    GVL_LIB=$L timeout -k 10 200 python -u tools/attn_one.py 20 > $O/attn_${v}_$r.log 2>&1; fatal $? attn_$v
    echo "== attn $v $r"; grep -v amdgpu.ids $O/attn_${v}_$r.log | head -1
  done; done
  for r in 1 2; do for v in base prio; do
    L=$LIBDIR/libgvl.so; [ $v = prio ] && L=$LIBDIR/libgvl_prio.so
    GVL_LIB=$L bench lm_${v}_$r lm
  done; done
  ;;
r6w)  # direct-A N = 768 dX on 128-row tiles with two workgroups per CU (gemm_w4d2_kernel, 254 VGPRs;
      # GVL_W4D_2WG=1, plain epilogue only). Bound (r6v PMC): one wave per SIMD, 38-41 % of wave
      # cycles in s_waitcnt, MFMA busy 0.15-0.28; the dX class is 16 % of the Q-Former step -> if a
      # second wave per SIMD lifts MFMA busy by half, ~4-5 % of the step.
  GVL_W4D_2WG=1 ktests kt "w4 or caption or linear_decoder or strided"
  for r in 1 2; do for v in 0 1; do for K in 768 2304 3072; do
    GVL_W4D_2WG=$v timeout -k 10 120 python tools/gemm_one.py 8064 768 $K 0 1 3 -1 20 > $O/g_${v}_${K}_$r.log 2>&1; fatal $? g
    echo "2wg=$v K=$K $r $(grep -v amdgpu.ids $O/g_${v}_${K}_$r.log | tail -1)"
  done; done; done
  GVL_W4D_2WG=1 GVL_MARGINS_DIR=$O/parity_margins ktests parity "qformer or linear" tests/test_gpu_parity_bench.py
  for r in 1 2; do for v in 0 1; do GVL_W4D_2WG=$v bench qf_w${v}_$r qformer; done; done
  ;;
r6v)  # PMC of the direct-A N = 768 dX launches at K = 768 and 3072 (8064 rows): where the ~0.5 us per
      # 32-deep K-step (3.2x its MFMA time) goes — evidence for the next round's plan, no code change
  timeout -k 10 600 bash tools/pmc_gemm.sh w4d_r6v "8064 768 768 0 1 3 -1" "8064 768 3072 0 1 3 -1"; fatal $? pmc
  for c in 1 2; do for pn in 1 2 3; do echo "== case $c pass $pn"; python tools/pmc_summary.py gpurun_out/pmc_w4d_r6v/c${c}_p$pn; done; done > $O/pmc_summary.txt 2>&1
  cat $O/pmc_summary.txt
  cat gpurun_out/pmc_w4d_r6v/times.log | grep -v amdgpu.ids
  ;;
r6u)  # gate backward with its final sum in the same launch (last block by ticket): the cross-att step's 12
      # gate_finish dispatches (~4.5 us each for 1 KiB of work) gone. Bound: 54 us of the 6.2 ms step
      # = ~0.9 %. A/B by GVL_GATE_FUSED=0.
  ktests kt "gate or colsum or dropout"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "cross" tests/test_gpu_parity_bench.py
  ktests full "cross" tests/test_gpu_parity_full.py
  for r in 1 2 3; do for v in 0 1; do GVL_GATE_FUSED=$v bench cross_g${v}_$r cross; done; done
  ;;
r6t)  # 32-query tiles over a 64-key tile (attn_fwd_kernel<1, *, true, 32, 64>, attn_bwd_short_kernel<*, 32, 64>)
      # for Tq <= 32 < Tk <= 64: the cross-att decoder's 31 x 33 cross-attention (12 fwd + 12 bwd per
      # step) and the Q-Former bridge's 32 x 33. Bound: the 64-row kernels at half padding, ~16.7 us bwd
      # + ~9 us fwd x 12 in cross -> ~25 % off = ~1 % of cross, ~0.3 % of the Q-Former step.
      # A/B by GVL_ATTN_SHORT3264=0 (kernel stats + steps).
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "qformer or cross" tests/test_gpu_parity_bench.py
  ktests full "qformer or cross" tests/test_gpu_parity_full.py
  for v in 0 1; do
    GVL_ATTN_SHORT3264=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s$v -o s$v -- \
      python tools/attn_one.py 50 > $O/prof_s$v.log 2>&1; fatal $? prof_s$v
    f=$(find $O/prof_s$v -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 14 > $O/table_s$v.txt
    echo "== SHORT3264=$v"; grep -E "short|fwd_kernel" $O/table_s$v.txt
  done
  for r in 1 2 3; do for v in 0 1; do
    GVL_ATTN_SHORT3264=$v bench cross_s${v}_$r cross; GVL_ATTN_SHORT3264=$v bench qf_s${v}_$r qformer
  done; done
  ;;
r6s)  # 16 KiB short attention backward (attn_bwd_short16_kernel: never more than two 64-row tiles in LDS,
      # 76 VGPRs) for 32 < T <= 64: 6 blocks per CU instead of 5, the 1536 (b, h) blocks of the
      # Q-Former / linear decoders in one round. Bound: attn_bwd_short<false, 64> is 3.4 % of the
      # Q-Former step (22.3 us x 12); 1.2 rounds -> 1 at ~equal block time -> up to ~15 % off = ~0.5 %.
      # A/B by GVL_ATTN_SHORT16=0 (kernel stats + steps).
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "qformer or linear or cross" tests/test_gpu_parity_bench.py
  ktests full "qformer or linear or cross" tests/test_gpu_parity_full.py
  for v in 0 1; do
    GVL_ATTN_SHORT16=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s$v -o s$v -- \
      python tools/attn_one.py 50 > $O/prof_s$v.log 2>&1; fatal $? prof_s$v
    f=$(find $O/prof_s$v -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 12 > $O/table_s$v.txt
    echo "== SHORT16=$v"; grep -E "short" $O/table_s$v.txt
  done
  for r in 1 2 3; do for v in 0 1; do
    GVL_ATTN_SHORT16=$v bench qf_s${v}_$r qformer; GVL_ATTN_SHORT16=$v bench lin_s${v}_$r linear
  done; done
  ;;
r6r)  # 32-row one-tile forward (attn_fwd_kernel<1, *, true, 32>: 2 waves, 8 KiB LDS) with the r6q backward
      # under the same switch (GVL_ATTN_SHORT32). Bound: the T = 31 forward is ~9 us x 12 per cross step
      # with half its waves idle -> ~3 us each = ~0.6 % of cross. Kernel stats (rocprofv3) + steps.
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "qformer or cross" tests/test_gpu_parity_bench.py
  ktests full "qformer or cross" tests/test_gpu_parity_full.py
  for v in 0 1; do
    GVL_ATTN_SHORT32=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s$v -o s$v -- \
      python tools/attn_one.py 50 > $O/prof_s$v.log 2>&1; fatal $? prof_s$v
    f=$(find $O/prof_s$v -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 12 > $O/table_s$v.txt
    echo "== SHORT32=$v"; grep -E "short|attn_fwd_kernel" $O/table_s$v.txt
  done
  for r in 1 2 3; do for v in 0 1; do
    GVL_ATTN_SHORT32=$v bench cross_s${v}_$r cross; GVL_ATTN_SHORT32=$v bench qf_s${v}_$r qformer
  done; done
  ;;
r6q2)  # r6q's A/B was within noise at the step level: kernel durations by rocprofv3 (attn_one 50
       # iterations each) and three more alternated cross / Q-Former pairs
  for v in 0 1; do
    GVL_ATTN_SHORT32=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_s$v -o s$v -- \
      python tools/attn_one.py 50 > $O/prof_s$v.log 2>&1; fatal $? prof_s$v
    f=$(find $O/prof_s$v -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 12 > $O/table_s$v.txt
    echo "== SHORT32=$v"; grep -E "short|attn_fwd_kernel" $O/table_s$v.txt
  done
  for r in 1 2 3; do for v in 0 1; do
    GVL_ATTN_SHORT32=$v bench cross_s${v}_$r cross; GVL_ATTN_SHORT32=$v bench qf_s${v}_$r qformer
  done; done
  ;;
r6q)  # 32-row short attention backward (attn_bwd_short_kernel<*, 32>: 2 waves, 16 KiB LDS, 56 VGPRs) for
      # Tq, Tk <= 32: the cross-att decoder's 31-token self-attention (12 per step) and the Q-Former
      # bridge's 32-query self-attention. Bound: attn_bwd_short is 6.2 % of the cross step, half of it
      # T = 31; 64-row blocks were half padding at 5 per CU -> ~40 % off those = ~1.2 % of cross,
      # ~0.4 % of the Q-Former step. A/B by GVL_ATTN_SHORT32=0.
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "qformer or cross" tests/test_gpu_parity_bench.py
  ktests full "qformer or cross" tests/test_gpu_parity_full.py
  for r in 1 2; do for v in 0 1; do
    GVL_ATTN_SHORT32=$v timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_s${v}_$r.log 2>&1; fatal $? attn_$v
    echo "== attn SHORT32=$v $r"; grep -v amdgpu.ids $O/attn_s${v}_$r.log | sed -n 3,4p
  done; done
  for r in 1 2; do for v in 0 1; do
    GVL_ATTN_SHORT32=$v bench cross_s${v}_$r cross; GVL_ATTN_SHORT32=$v bench qf_s${v}_$r qformer
  done; done
  ;;
r6p)  # T > 64 dQ kernel (G = 2, no dropout) compiled for 3 blocks per CU (168 VGPRs, 48 B of spill
      # outside the unmasked loop) instead of 2 (192 VGPRs). Bound: dQ is 4.9 % of the LM step at
      # 2 waves per SIMD with ~38 % of wave cycles waiting; a third more waves -> 10-15 % off dQ =
      # 0.5-0.7 % of the LM step. A/B against libgvl_dq2.so (GVL_ATTN_DQ_BPC=2).
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "lm" tests/test_gpu_parity_bench.py
  for r in 1 2; do for v in dq2 new; do
    L=$LIBDIR/libgvl.so; [ $v = dq2 ] && L=$LIBDIR/libgvl_dq2.so
    GVL_LIB=$L timeout -k 10 200 python -u tools/attn_one.py 20 > $O/attn_${v}_$r.log 2>&1; fatal $? attn_$v
    echo "== attn $v $r"; grep -v amdgpu.ids $O/attn_${v}_$r.log | head -1
  done; done
  for r in 1 2; do for v in dq2 new; do
    L=$LIBDIR/libgvl.so; [ $v = dq2 ] && L=$LIBDIR/libgvl_dq2.so
    GVL_LIB=$L bench lm_${v}_$r lm
  done; done
  ;;
r6o)  # split-K slabs of 256 x 192 tiles for the caption lm_head dX (M = 3968, N = 768, K = 50304: 64 x 4
      # = 256 items, one full round, instead of 48 x 4 = 192 of 256 x 256). Bound: the launch is
      # 4.4 % of the Q-Former step, 7.5 % of cross; a quarter off -> ~1.1 % / ~1.9 %.
      # A/B by GVL_PP3_SPLIT192=0.
  ktests kt "splitk or wgrad or gemm_lmhead or caption"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "qformer or cross or linear" tests/test_gpu_parity_bench.py
  for r in 1 2; do for v in 0 1; do
    GVL_PP3_SPLIT192=$v timeout -k 10 120 python tools/gemm_one.py 3968 768 50304 0 1 3 -1 20 > $O/g_s${v}_$r.log 2>&1; fatal $? g_$v
    echo "split192=$v $r $(grep -v amdgpu.ids $O/g_s${v}_$r.log | tail -1)"
  done; done
  for r in 1 2; do for v in 0 1; do
    GVL_PP3_SPLIT192=$v bench cross_s${v}_$r cross; GVL_PP3_SPLIT192=$v bench qf_s${v}_$r qformer
  done; done
  ;;
r6n)  # one-tile short attention forward (attn_fwd_kernel<1, *, true>: single 16 KiB LDS stage, 63 / 72
      # VGPRs, up to 8 blocks per CU): T = 63 decoder forward 1536 blocks in one round instead of 1.5.
      # Bound: attn_fwd_kernel<1, *> is 3.9 % of the cross step, 2.8 % of the Q-Former step; a third
      # off -> cross ~1.3 %, Q-Former ~0.9 %. A/B by GVL_ATTN_FWD_ONE=0.
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "qformer or cross or linear" tests/test_gpu_parity_bench.py
  ktests full "qformer or cross or linear" tests/test_gpu_parity_full.py
  for r in 1 2; do for v in 0 1; do
    GVL_ATTN_FWD_ONE=$v timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_one${v}_$r.log 2>&1; fatal $? attn_$v
    echo "== attn ONE=$v $r"; grep -v amdgpu.ids $O/attn_one${v}_$r.log | sed -n 2,5p
  done; done
  for r in 1 2; do for v in 0 1; do
    GVL_ATTN_FWD_ONE=$v bench cross_o${v}_$r cross; GVL_ATTN_FWD_ONE=$v bench qf_o${v}_$r qformer
  done; done
  ;;
r6m)  # attention address registers (tr_lane / frag_tr_imm: one VGPR per column block, the k-half
      # and row group as ds offsets; dK/dV slot offset opaque). Bound: ISA count per dK/dV query
      # tile 64 -> 12 v_add_u32 (of ~250 vector issues), forward / dQ key tile 29 -> 13; attention
      # is 14.2 % of the LM step, dK/dV 7.8 % -> if issue-bound ~15-20 % off dK/dV, ~5 % off fwd / dQ:
      # LM +1.5-2 %. Base = the same tree with HEAD's attention.hip (libgvl_base.so).
  ktests kt "attention or attn"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "lm" tests/test_gpu_parity_bench.py
  ktests full "lm or accumulation" tests/test_gpu_parity_full.py
  for r in 1 2; do for v in base new; do
    L=$LIBDIR/libgvl.so; [ $v = base ] && L=$LIBDIR/libgvl_base.so
    GVL_LIB=$L timeout -k 10 200 python -u tools/attn_one.py 20 > $O/attn_${v}_$r.log 2>&1; fatal $? attn_$v
    echo "== attn $v $r"; grep -v amdgpu.ids $O/attn_${v}_$r.log | head -8
  done; done
  for r in 1 2; do for v in base new; do
    L=$LIBDIR/libgvl.so; [ $v = base ] && L=$LIBDIR/libgvl_base.so
    GVL_LIB=$L bench lm_${v}_$r lm
  done; done
  ;;
r6a)  # teardown (GraphedStep.close, gvl.dist.destroy_process_group) tests; two-stream overlap probe
      # (bound for the Q-Former two-branch lever: up to the 20 % non-GEMM share if half-batch chains
      # overlap); DEFER_LMHEAD peak memory
  ktests dp "" tests/test_gpu_dp.py
  ktests graph "" tests/test_gpu_graph.py
  for v in 1 0; do
    GVL_W4_BM128=$v timeout -k 10 200 python -u tools/concurrency_probe.py 20 > $O/probe_bm128_$v.log 2>&1; fatal $? probe
    echo "== probe GVL_W4_BM128=$v"; grep -v amdgpu.ids $O/probe_bm128_$v.log
  done
  for v in 1 0; do GVL_DEFER_LMHEAD=$v bench lm_d$v lm; done
  ;;
r6b)  # LM grouped dW launch: one workgroup per tile (GVL_W4X_NP=1) so the three tiles sharing a
      # dY slab start together every round. Bound: the launch is 20.7 % of the LM step at 1.81 GHz
      # and 2.16x its operand bytes; back at the dX kernels' 2.45 GHz it would be ~26 % shorter
      # (5 % of the step); predicted gain >= 3 % only if traffic drops toward 1.4x and the clock
      # follows. Kernel tests + bench-shape LM parity with NP=1, LM A/B alternated, PMC of the launch.
  GVL_W4X_NP=1 ktests kt "grouped or w4x or wgrad or batched"
  GVL_W4X_NP=1 GVL_MARGINS_DIR=$O/parity_margins ktests parity "lm" tests/test_gpu_parity_bench.py
  for r in 1 2; do for v in 0 1; do GVL_W4X_NP=$v bench lm_np${v}_$r lm; done; done
  GVL_W4X_NP=1 GVL_W4X_DW_GROUP=1 bench lm_np1g1 lm
  for v in 0 1; do for c in FETCH_SIZE "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
    d=${c%% *}
    GVL_W4X_NP=$v timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $c --output-format csv -d $O/pmc_np$v/lm_$d -o run -- \
      python bench.py --steps 1 --warmup 0 --no-secondary --no-cpu-baseline --no-graph > $O/pmc_np${v}_$d.log 2>&1; fatal $? pmc
  done; done
  ;;
r6c)  # 128 x 96 four-wave tiles (gemm_w4n_kernel) for the 3968 / 4096-row N = 768 GEMMs. Bound: the
      # cross step's w4m classes are 29.4 % at 186 tiles (one round, paced by the per-CU operand
      # stream); 248 tiles streaming 224 instead of 256 rows each -> ~12 % off those kernels =
      # ~3.7 % of the cross step, ~0.7 % of the Q-Former step (bridge rows)
  ktests kt "test_gemm_w4 or gated or dropout_residual or grouped"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "cross or qformer" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "cross or qformer" tests/test_gpu_parity_full.py
  for M in 3968 4096; do for v in 1 0; do
    GVL_W4_BN96=$v GVL_DIAG_COLS=epi timeout -k 10 240 python -u tools/gemm_diag.py $M narrow > $O/diag_bn96_${v}_$M.log 2>&1; fatal $? diag
    echo "== M=$M BN96=$v"; grep "N=" $O/diag_bn96_${v}_$M.log
  done; done
  for r in 1 2; do for v in 1 0; do GVL_W4_BN96=$v bench cross_b${v}_$r cross; GVL_W4_BN96=$v bench qf_b${v}_$r qformer; done; done
  ;;
r6d)  # short attention backward: two (b, h) per block with the second's loads issued before the
      # first's math (GVL_ATTN_SHORT_PAIR=1) vs one per block. Bound: attn_bwd_short is 5.1 % of the
      # Q-Former step, 4.9 % of linear, 6.4 % of cross at ~3.5 TB/s of its 99 MB; at 5.5 TB/s -> ~35 %
      # off it = 1.7-2.2 % of those steps. Also: 128 x 96 tiles on K-contiguous B only (default now).
  ktests kt "attention or attn or test_gemm_w4 or gated or dropout_residual"
  GVL_W4_BN96=2 ktests kt96 "test_gemm_w4 and not w4x"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "" tests/test_gpu_parity_full.py
  for r in 1 2; do for v in 1 0; do
    GVL_ATTN_SHORT_PAIR=$v timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_p${v}_$r.log 2>&1; fatal $? attn
    echo "attn pair=$v $r"; grep -E "Tq=63|Tq=31|Tq=32" $O/attn_p${v}_$r.log
  done; done
  for r in 1 2; do for v in 1 0; do
    GVL_ATTN_SHORT_PAIR=$v bench qf_p${v}_$r qformer; GVL_ATTN_SHORT_PAIR=$v bench cross_p${v}_$r cross; GVL_ATTN_SHORT_PAIR=$v bench lin_p${v}_$r linear
  done; done
  ;;
r6e)  # Q-Former floor budget inputs: every GEMM instance of the step with its
      # FLOP (bench --gemm-table) and the rocprofv3 kernel table at this head; same for the LM
  timeout -k 10 300 python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline --gemm-table > $O/qf_gemms.json 2> $O/qf_gemms.err; fatal $? qf_gemms
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-secondary --no-cpu-baseline --gemm-table > $O/lm_gemms.json 2> $O/lm_gemms.err; fatal $? lm_gemms
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_qf -o qf -- \
    python bench.py --workload qformer --steps 10 --warmup 3 --no-cpu-baseline > $O/prof_qf.json 2> $O/prof_qf.err; fatal $? prof_qf
  f=$(find $O/prof_qf -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 45 > $O/qf_table.txt; head -30 $O/qf_table.txt
  ;;
r6fin|r6fin2|r6fin3|r6fin4)  # head check: GPU suite + smoke, the driver's default bench, rocprofv3 kernel stats of all four steps
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
  for w in qf lm cross linear; do f=$(find $O/prof_$w -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 40 > $O/${w}_table.txt; head -8 $O/${w}_table.txt; done
  ;;
r6pmc|r6pmc2)  # PMC passes (FETCH / WRITE / MFMA busy + clock) of all four bench workloads at the head
  timeout -k 10 1100 bash tools/pmc_traffic.sh $S "lm qf cross linear"; fatal $? pmc
  python -c "import json;d=json.load(open('gpurun_out/pmc_traffic_$S.json'));[print(w, k, v['hbm_bytes'], v.get('mfma_busy'), v.get('clock_ghz')) for w in d['workloads'] for k, v in list(d['workloads'][w].items())[:2]]"
  ;;
r6f)  # short attention backward: memory floor of its access pattern (timing-only libgvl_sdiag.so:
      # the loads, then the stores of the same bytes) vs the shipped kernel. Bound: if the floor is
      # near the kernel's 23 us, the kernel is paced by its 99 MB at ~4 TB/s and only the access
      # pattern can move it (2-4 % of the caption steps)
  for r in 1 2; do for L in base sdiag; do
    LIB=$LIBDIR/libgvl.so; [ $L != base ] && LIB=$LIBDIR/libgvl_$L.so
    GVL_LIB=$LIB timeout -k 10 200 python -u tools/attn_one.py 30 > $O/attn_${L}_$r.log 2>&1; fatal $? attn
    echo "attn $L $r"; grep -E "Tq=63|Tq=31|Tq=32 Tk=32" $O/attn_${L}_$r.log
  done; done
  ;;
r6g)  # frozen CLIP ViT-L/14 stage (configs[3] pixel input; stock PyTorch-ROCm): where its ~38 ms per
      # B = 128 go. Bound: it is ~85 % of the caption_linear_pixels step at ~0.22 of the bf16 peak
  timeout -k 10 300 python -u tools/clip_prof.py 128 10 eager > $O/clip_eager.log 2>&1; fatal $? clip; cat $O/clip_eager.log | grep CLIP
  timeout -k 10 300 python -u tools/clip_prof.py 128 10 graph > $O/clip_graph.log 2>&1; fatal $? clip_graph; cat $O/clip_graph.log | grep CLIP
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_clip -o clip -- \
    python tools/clip_prof.py 128 5 eager > $O/prof_clip.log 2>&1; fatal $? prof_clip
  f=$(find $O/prof_clip -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 30 > $O/clip_table.txt; cat $O/clip_table.txt
  ;;
r6h)  # gvl-native CLIP encoder (configs[3] pixel input) + the quick-GELU epilogue (ABI v14). Bound: the
      # stock tower's 38.5 ms per B = 128 spends ~12 ms in elementwise / LayerNorm passes and 4.6 ms in
      # SDPA around 21.7 ms of GEMMs at ~0.38: fused epilogues + gvl attention/LN -> ~22-25 ms
  ktests kt "gemm or quick_gelu"
  ktests capi "" tests/test_capi.py
  GVL_MARGINS_DIR=$O/parity_margins ktests clip "clip" tests/test_gpu_decode.py
  for m in eager native native_graph; do
    timeout -k 10 300 python -u tools/clip_prof.py 128 10 $m > $O/clip_$m.log 2>&1; fatal $? clip_$m; grep CLIP $O/clip_$m.log
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_clipn -o clipn -- \
    python tools/clip_prof.py 128 5 native > $O/prof_clipn.log 2>&1; fatal $? prof_clipn
  f=$(find $O/prof_clipn -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 25 > $O/clipn_table.txt; cat $O/clipn_table.txt
  timeout -k 10 600 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err; fatal $? bench
  python -c "import json;d=json.load(open('$O/bench.json'));p=d['caption_linear_pixels'];print('pixels stock',p['value'],p['clip_ms_per_batch'],'native',p['native_clip'])"
  ;;
r6i)  # native CLIP GEMMs split at 256 x floor(M / 256) rows (whole CU rounds). Bound: out_proj / fc2 run
      # 3 rounds for 2.02 rounds of tiles (12.7 ms of the 29 ms forward) -> ~4 ms off
  GVL_MARGINS_DIR=$O/parity_margins ktests clip "clip" tests/test_gpu_decode.py
  cat $O/parity_margins/clip_native_vs_stock.json
  for m in native eager native; do
    timeout -k 10 300 python -u tools/clip_prof.py 128 10 $m > $O/clip_$m.log 2>&1; fatal $? clip_$m; grep CLIP $O/clip_$m.log
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_clipn -o clipn -- \
    python tools/clip_prof.py 128 5 native > $O/prof_clipn.log 2>&1; fatal $? prof_clipn
  f=$(find $O/prof_clipn -name "*kernel_stats.csv" | head -1); python tools/prof_table.py $f 25 > $O/clipn_table.txt; head -14 $O/clipn_table.txt
  ;;
r6j)  # native CLIP attention at T = 257 with 64-row query blocks (GVL_ATTN_G=1) vs 128-row (default G = 2:
      # 257 = 2 x 128 + 1, the third block of every (b, h) holds one query row). Bound: 2.7 ms of 24.8
  for r in 1 2; do for g in 0 1; do
    if [ $g = 1 ]; then export GVL_ATTN_G=1; else unset GVL_ATTN_G; fi
    timeout -k 10 300 python -u tools/clip_prof.py 128 10 native > $O/clip_g${g}_$r.log 2>&1; fatal $? clip; echo "G1=$g $(grep CLIP $O/clip_g${g}_$r.log)"
  done; done
  unset GVL_ATTN_G
  ;;
r6k)  # 96 x 128 dX tiles (gemm_w4r_kernel) for the cross-att decoder's 3968-row N = 768 dX products.
      # Bound: gemm_w4m_kernel<3, true, 0> is 18.9 % of the cross step at 186 tiles, one round;
      # 252 tiles streaming 224 instead of 256 rows each -> ~12 % off = ~2.3 % of the step
  ktests kt "test_gemm_w4 or gated or caption_dx or tile128x192"
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "cross" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "cross" tests/test_gpu_parity_full.py
  for v in 1 0; do
    GVL_W4_BM96=$v GVL_DIAG_COLS=epi timeout -k 10 240 python -u tools/gemm_diag.py 3968 narrow > $O/diag_bm96_${v}.log 2>&1; fatal $? diag
    echo "== 3968 BM96=$v"; grep "N=" $O/diag_bm96_${v}.log
  done
  for r in 1 2; do for v in 1 0; do GVL_W4_BM96=$v bench cross_r${v}_$r cross; done; done
  ;;
r6l)  # c_attn forward split into q (N = 768, four-wave kernels) + k|v (N = 1536, 256 tiles) at the caption
      # decoders' 8064 / 8192 rows (GVL_QKV_SPLIT=1) vs one 384-tile GEMM (1.5 rounds). Bound: pp3 1 is
      # 8.0 % of the Q-Former and 8.8 % of the linear step; one round each -> ~20 % off = ~1.6-2 %
  GVL_MARGINS_DIR=$O/parity_margins ktests parity "qformer or linear or lm" tests/test_gpu_parity_bench.py
  GVL_MARGINS_DIR=$O/parity_margins ktests full "" tests/test_gpu_parity_full.py
  ktests models "" tests/test_gpu_models.py
  for r in 1 2; do for v in 1 0; do GVL_QKV_SPLIT=$v bench qf_s${v}_$r qformer; GVL_QKV_SPLIT=$v bench lin_s${v}_$r linear; done; done
  ;;
*) echo "unknown session $S"; exit 2 ;;
esac
