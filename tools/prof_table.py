"""Summarise a rocprofv3 --stats kernel CSV: share of GPU time, calls, average duration,
and (for the bench's GEMM instances) the check against a bench JSON's dispatch-timed table.
python tools/prof_table.py <run_kernel_stats.csv> [bench.json [caption_key]] [top]"""
import csv
import json
import sys


def load(path):
    rows = list(csv.DictReader(open(path)))
    out = {}
    for r in rows:
        name = r["Name"]
        short = name.replace("void (anonymous namespace)::", "").replace("(anonymous namespace)::", "")
        short = short.split("(GemmP)")[0].split("((anonymous")[0].split("(unsigned")[0]
        out[short] = (int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]))
    return out


def main():
    stats = load(sys.argv[1])
    tot = sum(v[1] for v in stats.values())
    top = int(sys.argv[-1]) if sys.argv[-1].isdigit() else 15
    for k, (n, t, a) in sorted(stats.items(), key=lambda kv: -kv[1][1])[:top]:
        print(f"{t / tot * 100:5.1f}% {n:6d} {a / 1e3:9.2f}us  {k[:100]}")
    print(f"total GPU ms {tot / 1e6:.2f}")
    if len(sys.argv) > 2 and sys.argv[2].endswith(".json"):
        b = json.load(open(sys.argv[2]))
        key = sys.argv[3] if len(sys.argv) > 3 and not sys.argv[3].isdigit() else None
        roof = (b[key] if key else b)["roofline"]
        for row in roof["top_gemms"]:
            k = row["kernel"]
            if k in stats:
                r = stats[k][2] / 1e3
                print(f"{k[:60]:60s} bench {row['avg_us']:8.2f}us rocprof {r:8.2f}us "
                      f"ratio {row['avg_us'] / r:.3f}")


if __name__ == "__main__":
    main()
