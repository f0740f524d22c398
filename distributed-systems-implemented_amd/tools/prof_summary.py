"""Summarize a rocprofv3 --kernel-trace --stats SQLite db into a CSV (per kernel:
calls, total/avg/min/max duration in us, share).  Kernel names are shortened.

usage: python tools/prof_summary.py gpurun_out/prof3/bench_results.db profiles/rocprof_r01_bench.csv
"""
import csv
import re
import sqlite3
import sys


def short(name: str) -> str:
    if "rocprim" in name:
        m = re.search(r"wrapped_(\w+?)_config", name)
        return "rocprim::" + (m.group(1) if m else "kernel")
    return name.split("(")[0]


def main(db_path, out_path):
    db = sqlite3.connect(db_path)
    rows = db.execute("select name, duration from kernels").fetchall()
    agg = {}
    for name, dur in rows:
        k = short(name)
        # wc_map_kernel / wc_agg_kernel run on the dictionary samples (a few MB)
        # and on the whole split: report the split's launches on their own row so
        # their average is the one bench.py's roofline uses (> 1 ms at C2 sizes)
        if "wc_map_kernel" in k:
            k += " [split]" if dur > 1_000_000 else " [dictionary sample]"
        elif "wc_agg_kernel" in k:  # round 0 of a split vs samples and later (carried-miss) rounds
            k += " [split round 0]" if dur > 1_000_000 else " [sample / later round]"
        a = agg.setdefault(k, [0, 0.0, float("inf"), 0.0])
        a[0] += 1
        a[1] += dur
        a[2] = min(a[2], dur)
        a[3] = max(a[3], dur)
    total = sum(a[1] for a in agg.values())
    with open(out_path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "min_us", "max_us", "pct"])
        for k, a in sorted(agg.items(), key=lambda kv: -kv[1][1]):
            w.writerow([k, a[0], round(a[1] / 1e3, 1), round(a[1] / a[0] / 1e3, 2), round(a[2] / 1e3, 2),
                        round(a[3] / 1e3, 2), round(100 * a[1] / total, 2)])
    print(open(out_path).read())


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
