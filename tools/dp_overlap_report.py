"""From a rocprofv3 run with --kernel-trace --marker-trace of tools/dp_overlap_trace.py
(GVL_TRACE_BUCKETS=1): for the last optimizer step, when each gradient bucket's all-reduce was
issued (roctx marker) relative to the backward's GEMM / attention kernels — how many backward
kernels still ran after the first and after each bucket issue.  (At world size 1 RCCL runs no
kernel for an in-place AVG, so the issue points are the evidence; at N > 1 the all-reduce
runs on RCCL's stream from that point while those kernels run.)
python tools/dp_overlap_report.py <out_dir>"""
import csv
import glob
import sys

d = sys.argv[1]
kt = glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)
mt = glob.glob(f"{d}/**/*marker_api_trace.csv", recursive=True)
ker = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
             for r in csv.DictReader(open(kt[0])))
marks = []
if mt:
    for r in csv.DictReader(open(mt[0])):
        name = r.get("Function") or r.get("Message") or r.get("Marker_Name") or ""
        if "gvl.bucket" in name:
            marks.append((int(r.get("Start_Timestamp") or r.get("Timestamp")), name))
marks.sort()
print(f"{len(ker)} kernels, {len(marks)} bucket markers")
if not marks:
    sys.exit(0)
# the last optimizer step: its issues are the last len(distinct buckets) markers
nb = len({n for _, n in marks})
last = marks[-nb:]
work = [k for k in ker if ("gemm" in k[2] or "attn" in k[2]) and k[0] >= last[0][0] - 50_000_000]
end_bwd = max((k[1] for k in work), default=0)
print(f"last step: {len(last)} buckets issued")
for ts, name in last:
    after = [k for k in work if k[0] >= ts]
    print(f"{name:14s} issued with {len(after):4d} GEMM/attention kernels still to start "
          f"({(end_bwd - ts) / 1e3:8.1f} us of backward/optimizer work after it)")
