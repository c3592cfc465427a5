"""Per-kernel HBM bytes per launch from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

FETCH_SIZE and WRITE_SIZE are in KiB.  gfx950 correction, calibrated on known-byte kernels
(tools/pmc_calib.sh -> profiles/r2/pmc_calibration.json): FETCH_SIZE counts half the bytes of
16-B-per-lane streaming reads — expected/counter = 1.995 for the CE kernel's register loads and
1.90 for a GEMM whose A operand (512 MiB, read once) moves by buffer_load ... lds (the 5 % gap
is B re-fetched per XCD) — so it is doubled; WRITE_SIZE is exact for 16-B stores (0.998-1.000).
Kernels with narrower loads (LayerNorm backward's 8-B accesses) are not calibrated: their
traffic is an estimate.
usage: python tools/pmc_traffic.py DIR   (DIR holds {lm,qf}_{FETCH_SIZE,WRITE_SIZE}/**.csv)"""
import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    """'void (anonymous namespace)::gemm_ring_kernel<128, ...>(GemmP)' -> 'gemm_ring_kernel<128, ...>'
    (the names bench.py's kernel timer reports)."""
    s = name.replace("void ", "", 1).replace("(anonymous namespace)::", "")
    m = re.match(r"[\w:]+<[^<>()]*>", s)
    return m.group(0) if m else s.split("(")[0][:120]


def load(d, counter, with_time=False):
    """kernel -> [sum of the counter over dispatches, dispatches(, sum of durations in ns)]"""
    acc = defaultdict(lambda: [0.0, 0, 0.0])
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                k = short(row["Kernel_Name"])
                acc[k][0] += float(row["Counter_Value"])
                acc[k][1] += 1
                if row.get("End_Timestamp") and row.get("Start_Timestamp"):
                    acc[k][2] += float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    return acc


CUS, SIMDS = 256, 4


def mfma_clock(root, wl):
    """kernel -> (MFMA busy fraction, achieved clock in GHz).  SQ_VALU_MFMA_BUSY_CYCLES sums the
    matrix-pipe cycles over every SIMD (16 per 16x16x32 bf16 MFMA: 2^30 for an 8192^3 GEMM,
    profiles/r1/pmc), GRBM_GUI_ACTIVE the GPU-busy cycles over the 8 XCDs (MI355X_MICROARCH.md
    'DVFS give-back'), so busy = MFMA / (CUs x SIMDs x GRBM / 8) and clock = GRBM / 8 / duration.
    busy x clock / 2.4 GHz = the fraction of the 2.4 GHz bf16 peak the kernel reached."""
    d = os.path.join(root, f"{wl}_SQ_VALU_MFMA_BUSY_CYCLES")
    mf = load(d, "SQ_VALU_MFMA_BUSY_CYCLES")
    gr = load(d, "GRBM_GUI_ACTIVE")
    out = {}
    for k, (m, n, _) in mf.items():
        if k not in gr or not n or not gr[k][1] or gr[k][0] <= 0 or gr[k][2] <= 0:
            continue
        cyc = gr[k][0] / 8.0
        out[k] = (m / (CUS * SIMDS * cyc), cyc / gr[k][2])
    return out


def main(root):
    out = {"source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                     "eager bench steps; hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per launch; "
                     "mfma_busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE / 8), "
                     "clock_ghz = GRBM_GUI_ACTIVE / 8 / kernel duration (third pass; over-reads on launches "
                     "of <~100 us, whose GRBM window exceeds the dispatch), mfma_rate_frac = mfma_busy x "
                     "clock / 2.4 GHz = MFMA-pipe cycles per dispatch-duration cycle at the 2.4 GHz peak "
                     "clock (exact either way)",
           "workloads": {}}
    wls = sorted({os.path.basename(d).rsplit("_FETCH_SIZE", 1)[0]
                  for d in glob.glob(os.path.join(root, "*_FETCH_SIZE"))})
    for wl in wls:
        fe = load(os.path.join(root, f"{wl}_FETCH_SIZE"), "FETCH_SIZE")
        wr = load(os.path.join(root, f"{wl}_WRITE_SIZE"), "WRITE_SIZE")
        mc = mfma_clock(root, wl)
        ks = {}
        for k in fe:
            if k not in wr or not fe[k][1] or not wr[k][1]:
                continue
            f_kib, w_kib = fe[k][0] / fe[k][1], wr[k][0] / wr[k][1]
            ks[k] = dict(launches=fe[k][1], fetch_kib=round(f_kib, 1), write_kib=round(w_kib, 1),
                         hbm_bytes=round(2 * f_kib * 1024 + w_kib * 1024))
            if k in mc:
                ks[k]["mfma_busy"] = round(mc[k][0], 4)
                ks[k]["clock_ghz"] = round(mc[k][1], 3)
                # busy x clock = MFMA cycles / duration: exact, where the two factors are not for
                # short launches (GRBM_GUI_ACTIVE spans a few us more than the dispatch: clocks
                # above the 2.4 GHz peak on ~10-80 us kernels)
                ks[k]["mfma_rate_frac"] = round(mc[k][0] * mc[k][1] / 2.4, 4)
        out["workloads"][wl] = dict(sorted(ks.items(), key=lambda kv: -kv[1]["hbm_bytes"] * kv[1]["launches"]))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
