"""Average rocprofv3 --pmc counter values per kernel name over a directory of passes."""
import csv
import glob
import os
import sys
from collections import defaultdict


def main(root):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "").replace("(anonymous namespace)::", "")
                name = name.replace("void ", "").split("(")[0][:70]
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    for name, ctrs in sorted(acc.items()):
        if "gemm" not in name and not name.startswith("Cijk"):
            continue
        print(name)
        for c, v in sorted(ctrs.items()):
            # several rows per dispatch are possible (per-dimension); sum per dispatch ~ mean*rows
            print(f"   {c:32s} {sum(v) / len(v):16.4g}  (n={len(v)})")


if __name__ == "__main__":
    main(sys.argv[1])
