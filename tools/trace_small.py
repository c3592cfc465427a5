"""List the framework-side (torch / runtime copy) kernels of a rocprofv3 kernel trace with their
gvl neighbours, so each can be traced back to the Python line that launches it.

usage: python tools/trace_small.py <kernel_trace.csv> [last_n]
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 400
    rows = rows[-n:]
    short = lambda r: r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "")[:80]
    dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000
    tot = 0.0
    for i, r in enumerate(rows):
        k = r["Kernel_Name"]
        if "at::native" in k or "rocclr" in k:
            tot += dur(r)
            prev = short(rows[i - 1]) if i else "-"
            nxt = short(rows[i + 1]) if i + 1 < len(rows) else "-"
            print(f"{i:5d} {dur(r):7.2f}  {short(r)}\n        after {prev}\n        before {nxt}")
    print(f"framework kernels: {tot:.1f} us over the last {len(rows)} kernels")


if __name__ == "__main__":
    main()
