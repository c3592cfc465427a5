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


def load(d, counter):
    acc = defaultdict(lambda: [0.0, 0])
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] != counter:
                    continue
                k = short(row["Kernel_Name"])
                acc[k][0] += float(row["Counter_Value"])
                acc[k][1] += 1
    return acc


def main(root):
    out = {"source": "rocprofv3 --kernel-trace --pmc FETCH_SIZE / WRITE_SIZE (separate passes), "
                     "eager bench steps; hbm_bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024 per launch",
           "workloads": {}}
    for wl in ("lm", "qf"):
        fe = load(os.path.join(root, f"{wl}_FETCH_SIZE"), "FETCH_SIZE")
        wr = load(os.path.join(root, f"{wl}_WRITE_SIZE"), "WRITE_SIZE")
        ks = {}
        for k in fe:
            if k not in wr or not fe[k][1] or not wr[k][1]:
                continue
            f_kib, w_kib = fe[k][0] / fe[k][1], wr[k][0] / wr[k][1]
            ks[k] = dict(launches=fe[k][1], fetch_kib=round(f_kib, 1), write_kib=round(w_kib, 1),
                         hbm_bytes=round(2 * f_kib * 1024 + w_kib * 1024))
        out["workloads"][wl] = dict(sorted(ks.items(), key=lambda kv: -kv[1]["hbm_bytes"] * kv[1]["launches"]))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
