"""Floor budget of the Q-Former caption step: per kernel class the current
time, the MFMA floor (algorithmic FLOP at the 2516.6 TFLOP/s dense bf16 peak), the HBM floor
(algorithmic bytes at 8 TB/s), and the best-measured ceiling of this design, summed into an
achievable step and its fraction of the bf16 roofline.

python tools/qformer_budget.py BENCH_JSON KERNEL_TABLE
  BENCH_JSON   bench.py --workload qformer --gemm-table line (exact GEMM FLOP per instance)
  KERNEL_TABLE tools/prof_table.py output of the same step (rocprofv3 --kernel-trace --stats,
               steps 10 + warmup 3 + 1 capture = 14 per-step launches per kernel)

Shapes (B = 128 images, the bench's caption_batch): decoder rows M = 128 x 63 = 8064
(32 query + 31 text tokens, gpt2_q_former/model.py:213-249), 3968 text rows for the loss,
bridge query rows 4096 (32 per image), image rows 4224 (33 pooled tokens per image).
Algorithmic bytes count each operand read once and each output written once (bf16)."""
import json
import re
import sys

PEAK_TF = 2516.6
HBM_TBS = 8.0
STEPS_IN_TABLE = 14
MB = 1e6
C, V = 768, 50304
M, MT, MQ, MI = 8064, 3968, 4096, 4224


def mbytes(*elems):
    return sum(elems) * 2 / MB


# algorithmic bytes per step, per class (decoder layers x 12)
DEC = 12
BYTES = {
    "N=768 direct-A (decoder)": DEC * (
        mbytes(M * 4 * C, 4 * C * C, M * C)                                         # c_fc.dX
        + mbytes(M * C, C * C, M * C)                                               # attn.c_proj.dX
        + mbytes(M * 3 * C, 3 * C * C, M * C)                                       # c_attn.dX
        + mbytes(M * C, C * C, M * C, M * C)                                        # attn.c_proj fwd + res
        + mbytes(M * 4 * C, 4 * C * C, M * C, M * C)),                              # mlp.c_proj fwd + res
    "wide K=768 (c_attn / c_fc fwd, mlp.c_proj dX)": DEC * (
        mbytes(M * C, 4 * C * C, 2 * M * 4 * C)                                     # c_fc + gelu, gelu'
        + mbytes(M * C, 4 * C * C, 2 * M * 4 * C)                                   # c_proj.dX x gelu'
        + mbytes(M * C, 3 * C * C, M * 3 * C))                                      # c_attn + bias
    + 2 * mbytes(MQ * C, 4 * C * C, 2 * MQ * 4 * C)                                 # bridge MLP fc
    + 2 * mbytes(MQ * C, 3 * C * C, MQ * 3 * C)                                     # bridge in_proj
    + 2 * mbytes(MQ * C, 4 * C * C, 2 * MQ * 4 * C),                                # bridge MLP dX
    "lm_head fwd + dX": mbytes(M * C, V * C, M * V) + mbytes(MT * V, V * C, MT * C),
    "bridge GEMMs (w4m / w4n / grouped dW / ring)": 2 * (
        mbytes(MQ * C, C * C, MQ * C) * 4 + mbytes(MI * C, 2 * C * C, MI * 2 * C))
    + mbytes(MI * 1024, 1024 * C, MI * C) + 2 * 15 * mbytes(C * C * 2),
    "attention (decoder T=63, bridge T=32/33)": DEC * (mbytes(M * 3 * C, M * C) + mbytes(M * 5 * C, M * 3 * C))
    + 2 * (mbytes(MQ * 3 * C, MQ * C) + mbytes(MQ * 5 * C, MQ * 3 * C))
    + 2 * (mbytes(MQ * C, MI * 2 * C, MQ * C) + mbytes(MQ * 3 * C, MI * 2 * C, MQ * C, MI * 2 * C)),
    "LayerNorm fwd + bwd": 25 * (mbytes(2 * M * C) + mbytes(4 * M * C)) + 8 * (mbytes(2 * MQ * C) + mbytes(4 * MQ * C)),
    "cross-entropy": mbytes(2 * MT * V),
    "optimizer (grad norm + AdamW, fp32 masters)": 19.6e6 * 30 / MB + 19.6e6 * 2 / MB,
}

# class -> (kernel-name patterns, best-measured ceiling: fraction of peak for GEMMs or TB/s
# for memory-bound classes, and its source)
CLASSES = [
    ("N=768 direct-A (decoder)", [r"^gemm_w4d_kernel"], ("frac", 0.36,
     "timing-only build without in-loop A loads and hipBLASLt both ~0.36 on c_fc.dX "
     "(profiles/r3/w4d_diag_r3s2.txt): one 192x128 tile per CU, per-CU operand stream")),
    ("wide K=768 (c_attn / c_fc fwd, mlp.c_proj dX)", [r"^gemm_pp3_kernel<4, false, \w+, (1|9|10|11), 192"],
     ("frac+stores", 0.53, "K-loop alone 0.53 (no-store build, profiles/r5/pp3_row_sweep_r5j_r5m.txt) "
      "plus the outputs' HBM write at 5.9 TB/s, un-overlapped (vmcnt is in order)")),
    ("lm_head fwd + dX", [r"^gemm_pp3_kernel<4, false, \w+, 0, 256, 256>"],
     ("frac+stores", 0.53, "same K-loop ceiling + the 811 MB logits write")),
    ("bridge GEMMs (w4m / w4n / grouped dW / ring)", [r"^gemm_w4m_kernel", r"^gemm_w4n_kernel",
                                                       r"^gemm_w4x_kernel", r"^gemm_ring_kernel",
                                                       r"^gemm_splitk_reduce"],
     ("frac", 0.36, "as the decoder's N=768 class (4096-row shapes, one round)")),
    ("attention (decoder T=63, bridge T=32/33)", [r"^attn_"], ("tbs", 5.5,
     "gathered 128-B rows: 5.5-5.8 TB/s (MI355X_MICROARCH.md)")),
    ("LayerNorm fwd + bwd", [r"^ln_"], ("tbs", 5.5, "streaming rows, measured 5.3-5.5 TB/s here")),
    ("cross-entropy", [r"^ce_"], ("tbs", 5.5, "the LM's CE at 5.2 TB/s")),
    ("optimizer (grad norm + AdamW, fp32 masters)", [r"^adamw", r"^sumsq", r"^norm_finish"],
     ("tbs", 5.5, "streaming")),
]
STORE_BYTES = {  # outputs written by the wide / lm_head classes (MB per step)
    "wide K=768 (c_attn / c_fc fwd, mlp.c_proj dX)":
        DEC * (mbytes(2 * M * 4 * C) + mbytes(M * 4 * C) + mbytes(M * 3 * C))
        + 2 * mbytes(2 * MQ * 4 * C) + 2 * mbytes(MQ * 3 * C) + 2 * mbytes(MQ * 4 * C),
    "lm_head fwd + dX": mbytes(M * V) + mbytes(MT * C),
}


def main(bench_json, table):
    d = json.load(open(bench_json))
    gemms = d["roofline"]["all_gemms"]
    step_us = d["ms_per_step"] * 1e3
    images = d["config"].get("global_batch", 128) if isinstance(d.get("config"), dict) else 128
    rows = []
    for line in open(table):
        m = re.match(r"\s*[\d.]+%\s+(\d+)\s+([\d.]+)us\s+(.*)", line)
        if m:
            rows.append((m.group(3).strip(), int(m.group(1)) / STEPS_IN_TABLE, float(m.group(2))))
    table_us = sum(n * us for _, n, us in rows)
    scale = step_us / table_us  # table (eager + graph mix) -> this step's time
    used = set()
    out = []
    for cls, pats, (kind, ceil, src) in CLASSES:
        t = 0.0
        for name, n, us in rows:
            if any(re.search(p, name) for p in pats) and name not in used:
                used.add(name)
                t += n * us * scale
        flop = sum(g["launches_per_step"] * g["gflop_per_launch"] for g in gemms
                   if any(re.search(p, g["kernel"]) for p in pats))
        byt = BYTES[cls]
        mf = flop / PEAK_TF * 1e3  # us
        hb = byt / HBM_TBS  # MB / (TB/s) = us
        if kind == "frac":
            best = flop / (ceil * PEAK_TF) * 1e3
        elif kind == "frac+stores":
            best = flop / (ceil * PEAK_TF) * 1e3 + STORE_BYTES[cls] / 5.9
        else:
            best = byt / ceil
        out.append((cls, t, flop, byt, mf, hb, best, src))
    rest = step_us - sum(o[1] for o in out)
    total_flop = 35.16 * images  # GFLOP per step, SURVEY §8(d)
    print(f"Q-Former caption step, B={images}: {step_us:.0f} us measured ({d['value']:.0f} images/s, "
          f"{total_flop / step_us * 1e3 / PEAK_TF:.3f} of the bf16 peak); target 0.40 = "
          f"{total_flop / (0.40 * PEAK_TF) * 1e3:.0f} us")
    print(f"{'class':48s} {'now us':>7s} {'GFLOP':>7s} {'MB':>7s} {'MFMA fl':>8s} {'HBM fl':>7s} "
          f"{'best-meas':>9s}  ceiling source")
    for cls, t, flop, byt, mf, hb, best, src in out:
        print(f"{cls:48s} {t:7.0f} {flop:7.0f} {byt:7.0f} {mf:8.0f} {hb:7.0f} {best:9.0f}  {src}")
    print(f"{'other (dropout, pool, copies, embedding, colsum)':48s} {rest:7.0f} {'':>7s} {'':>7s} "
          f"{'':>8s} {'':>7s} {rest * 0.6:9.0f}  assumed 40 % off")
    floor = sum(max(o[4], o[5]) for o in out)
    best = sum(o[6] for o in out) + rest * 0.6
    print(f"sum of hard floors (max(MFMA, HBM) per class): {floor:.0f} us -> "
          f"{total_flop / floor * 1e3 / PEAK_TF:.3f}")
    print(f"sum of best-measured ceilings: {best:.0f} us -> {total_flop / best * 1e3 / PEAK_TF:.3f} "
          f"({images / best * 1e6:.0f} images/s)")
    # what 0.40 needs: GEMM classes at a common fraction f with stores hidden, memory classes at 5.5
    mem = sum(o[3] / 5.5 for o in out[4:]) + rest * 0.6
    gflop = sum(o[2] for o in out[:4])
    need = total_flop / (0.40 * PEAK_TF) * 1e3
    f = gflop / ((need - mem) * 1e-3) / PEAK_TF if need > mem else float("inf")
    print(f"0.40 needs: memory-bound classes at 5.5 TB/s ({mem:.0f} us) and every GEMM class at "
          f"{f:.2f} of peak with its stores hidden ({gflop:.0f} GFLOP in {need - mem:.0f} us)")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
