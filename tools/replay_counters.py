"""Loop counters of replay_kernel on the C3 sweep (profile build, GPU only).

`make prof` builds build/prof/libfognet_hip.so with FOGNET_REPLAY_PROFILE: the
kernel then writes its loop counters into the stats record instead of the
statistics (replay stage only).  This prints them per decision, per sweep class.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fognetsimpp_amd import _abi  # noqa: E402

MODE = "time" if ("--mode=time" in sys.argv or " ".join(sys.argv).find("--mode time") >= 0) else "count"
_abi.LIB_PATH = os.environ.get("FOGNET_LIB", os.path.join(ROOT, "build", "prof2" if MODE == "time" else "prof", "libfognet_hip.so"))
import fognetsimpp_amd as fa  # noqa: E402

FIELDS = [("n_queued", "iterations"), ("n_started", "advert_loop_iters"), ("last_tick", "adverts"),
          ("queue_min_raw", "scan_loads_lane"), ("queue_max_raw", "run_end_node_k"),
          ("resp_min_ticks", "horizon_slots"), ("resp_max_ticks", "refills"), ("queue_sum_lo", "nh_reads_young"),
          ("queue_sum_hi", "nh_reads"), ("queue_sq_lo", "chunks"), ("queue_sq_hi", "run_end_horizon"),
          ("resp_sum_lo", "runs_pend0"), ("resp_sum_hi", "run_end_chunk"),
          ("resp_sq_lo", "resumed_runs"), ("busy_s", "fresh_same_k"), ("resp_sq_hi", "horizon_end_then_same_k")]
TIME_FIELDS = [("n_queued", "cyc_chunk"), ("n_started", "cyc_adverts"), ("last_tick", "cyc_argmin"),
               ("queue_min_raw", "cyc_horizon"), ("queue_max_raw", "cyc_run_scan"),
               ("resp_min_ticks", "cyc_stores"), ("resp_max_ticks", "cyc_node_update"),
               ("queue_sum_lo", "cyc_chunk_flush_stats"), ("queue_sum_hi", "cyc_total"), ("queue_sq_lo", "cyc_advert_nh_wait"),
               ("queue_sq_hi", "cyc_horizon_nh_wait")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=576)
    ap.add_argument("--T", type=int, default=100_000)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--ring", type=int, default=1024)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--mode", choices=("count", "time"), default="count")
    a = ap.parse_args()
    ctx = fa.Context(0)
    mg, sc = fa.sweep_params(np.arange(a.R), a.N)
    trace = fa.generate_trace(ctx, a.seed, a.R, a.T, a.N, mg, sc)
    out = fa.allocate_outputs(a.R, a.T, torch.device("cuda", 0))
    fa.run_batch(ctx, trace, out, ring_capacity=a.ring, stage="replay")
    torch.cuda.synchronize()
    st = out.stats.cpu().numpy().view(_abi.REP_STATS_DTYPE)
    assert (st["status"] == 0).all(), np.unique(st["status"])
    res = {}
    cls = np.arange(a.R) % 9
    for c in range(-1, 9):
        m = np.ones(a.R, bool) if c < 0 else cls == c
        dec = st["n_tasks"][m].sum()
        fields = TIME_FIELDS if MODE == "time" else FIELDS
        row = {name: float(st[f][m].astype(np.float64).sum() / dec) for f, name in fields}
        if MODE == "count":
            row["decisions_per_iteration"] = float(dec / st["n_queued"][m].sum())
        key = "all" if c < 0 else f"rho={(0.5, 0.8, 0.95)[c % 3]} lat_x{(1, 10, 100)[c // 3]}"
        res[key] = row
    if MODE == "time":  # per-replication wall cycles: the spread that sets the launch's tail
        tot = st["queue_sum_hi"].astype(np.float64)
        res["per_rep_total_cycles"] = {
            "min": float(tot.min()), "p50": float(np.median(tot)), "p90": float(np.percentile(tot, 90)),
            "max": float(tot.max()), "mean": float(tot.mean()),
            "by_class_mean": [float(tot[cls == c].mean()) for c in range(9)],
            "by_class_max": [float(tot[cls == c].max()) for c in range(9)]}
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
