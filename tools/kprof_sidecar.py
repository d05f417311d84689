"""Sidecar of a committed rocprofv3 kernel profile, read by bench.py (``kernel_avg_ms_rocprof``).

The profile must come from the bench command itself (same workload, same sizes, same
steps/warm-up): this tool takes the bench's own JSON line from that profiled run and the
tools/kstats.py summary of its kernel trace (warm-up dispatches skipped), picks the dominant
kernel, and refuses to write a sidecar whose average launch exceeds the run's ms_per_step
(a profile of another tree or other sizes cannot be the one the line quotes).  It records the
sha256 of the library the profiled run loaded (--lib): bench.py quotes the sidecar only for a
run of that same binary (a stale profile of an older, faster build is never quoted).

  python tools/kprof_sidecar.py <bench log or json> <kstats.csv> --kernel <name prefix> \
      --cmd "<the profiled command>" --out profiles/kernel_profile_<workload>.json"""
import argparse
import csv
import hashlib
import json
import re
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("bench")
    ap.add_argument("kstats")
    ap.add_argument("--kernel", required=True, help="prefix of the kernel's demangled name after 'fognet::'")
    ap.add_argument("--cmd", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--tree", default=None, help="the commit the profiled tree was built from")
    ap.add_argument("--lib", default="fognetsimpp_amd/libfognet_hip.so", help="the library the profiled run loaded")
    a = ap.parse_args()
    line = [ln for ln in open(a.bench) if ln.startswith("{")][-1]
    b = json.loads(line)
    pat = re.compile(r"(^|[ :])" + re.escape(a.kernel) + r"\b")
    rows = [r for r in csv.DictReader(open(a.kstats)) if pat.search(r["Name"])]
    if not rows:
        sys.exit(f"no kernel matching {a.kernel!r} in {a.kstats}")
    r = max(rows, key=lambda r: float(r["TotalDurationNs"]))
    avg_ms = float(r["AverageNs"]) / 1e6
    if avg_ms > b["ms_per_step"]:
        sys.exit(f"refused: rocprof average {avg_ms:.3f} ms > the run's {b['ms_per_step']:.3f} ms/step")
    side = {"command": a.cmd, "kernel": r["Name"], "calls": int(r["Calls"]), "avg_ms": avg_ms,
            "min_ms": float(r["MinNs"]) / 1e6, "max_ms": float(r["MaxNs"]) / 1e6,
            "skipped_warmup": int(r.get("SkippedWarmup") or 0), "steps": b["steps"], "warmup": b["warmup"],
            "ms_per_step": b["ms_per_step"], "kernel_avg_ms_hip_events": b["roofline"].get("kernel_avg_ms"),
            "config": b["config"], "stats_csv": a.kstats, "tree": a.tree,
            "lib_sha256": hashlib.sha256(open(a.lib, "rb").read()).hexdigest()}
    json.dump(side, open(a.out, "w"), indent=1)
    print(json.dumps({k: side[k] for k in ("kernel", "calls", "avg_ms", "ms_per_step", "kernel_avg_ms_hip_events")}))


if __name__ == "__main__":
    main()
