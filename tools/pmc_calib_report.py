"""Pair tools/pmc_calib.py's expected bytes with the FETCH_SIZE / WRITE_SIZE passes.
usage: python tools/pmc_calib_report.py DIR  (DIR/{FETCH_SIZE,WRITE_SIZE}/**.csv, DIR/expect.log)"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def counters(d, name):
    out = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == name:
                    out[row["Kernel_Name"]].append(float(row["Counter_Value"]) * 1024)
    return out


def classify(k):
    if "ce_row_kernel" in k:
        return "ce_row_kernel"
    if "gemm_pp3_kernel" in k or "gemm_ring_kernel" in k:
        return "gemm"
    if "copy" in k.lower() or "elementwise" in k:
        return "copy"
    return None


def main(root):
    exp = None
    for line in open(os.path.join(root, "expect.log")):
        if line.startswith("EXPECT "):
            exp = json.loads(line[7:])
    res = {}
    for cname, key in (("FETCH_SIZE", "read"), ("WRITE_SIZE", "write")):
        for k, vals in counters(os.path.join(root, cname), cname).items():
            c = classify(k)
            if c is None or c not in exp:
                continue
            v = sorted(vals)[len(vals) // 2]  # median launch
            r = res.setdefault(c, {"kernel": k.split("(")[0][:90]})
            r[f"{cname}_bytes"] = v
            r[f"expected_{key}_bytes"] = exp[c][key]
            r[f"{key}_ratio_expected_over_counter"] = round(exp[c][key] / v, 4) if v else None
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
