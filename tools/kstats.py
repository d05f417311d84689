"""Per-kernel duration statistics from a rocprofv3 --kernel-trace CSV, with the
first W dispatches of each kernel (the bench's warm-up steps, a cold first call)
left out, so the average describes the timed steps only.

  python tools/kstats.py <dir with *_kernel_trace.csv> [--skip W] [--out file.csv]

Writes the rocprofv3 --stats columns (Name, Calls, TotalDurationNs, AverageNs,
Percentage, MinNs, MaxNs, StdDev) over the kept dispatches."""
import argparse
import collections
import csv
import glob
import math
import os
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--skip", type=int, default=1, help="dispatches of each kernel left out (warm-up)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    files = glob.glob(os.path.join(a.root, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        sys.exit(f"no *kernel_trace.csv under {a.root}")
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), r["Kernel_Name"], int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    rows.sort()
    seen = collections.Counter()
    dur = collections.defaultdict(list)
    for _, name, d in rows:
        seen[name] += 1
        if seen[name] > a.skip:
            dur[name].append(d)
    total = sum(sum(v) for v in dur.values()) or 1
    out = [("Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev", "SkippedWarmup")]
    for name, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        m = sum(v) / len(v)
        sd = math.sqrt(sum((x - m) ** 2 for x in v) / len(v))
        out.append((name, len(v), sum(v), round(m, 3), round(100.0 * sum(v) / total, 2), min(v), max(v), round(sd, 3),
                    min(a.skip, seen[name])))
    w = csv.writer(open(a.out, "w", newline="") if a.out else sys.stdout, quoting=csv.QUOTE_NONNUMERIC)
    for r in out:
        w.writerow(r)


if __name__ == "__main__":
    main()
