"""Loop segments of replay_wide_kernel at C5 (profile build `make prof`,
build/prof2; GPU only): s_memtime cycles per segment and loop event counts,
per decision.  Usage: python tools/wide_counters.py [--policy REF_V3|EXT_HIER] [--R 1024]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fognetsimpp_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.path.join(ROOT, "build", "prof2", "libfognet_hip.so")
import fognetsimpp_amd as fa  # noqa: E402

SEG = [("n_queued", "chunk"), ("n_started", "adverts"), ("last_tick", "decision"), ("queue_min_raw", "record"),
       ("queue_max_raw", "horizon"), ("resp_min_ticks", "run_fifo"), ("resp_max_ticks", "stores_stats"),
       ("queue_sum_lo", "node_update"), ("queue_sum_hi", "total")]
CNT = [("queue_sq_lo", "iterations"), ("queue_sq_hi", "advert_loop_iters"), ("resp_sum_lo", "adverts"),
       ("resp_sum_hi", "record_switches")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--R", type=int, default=1024)
    ap.add_argument("--T", type=int, default=10_000)
    ap.add_argument("--N", type=int, default=10_000)
    ap.add_argument("--policy", default="REF_V3")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    ctx = fa.Context(0)
    dev = torch.device("cuda", 0)
    mg, sc = fa.c5_params(np.arange(a.R), a.N)
    tr = {k: v for k, v in fa.generate_trace(ctx, 0x5EED0005, a.R, a.T, a.N, mg, sc).items() if not k.startswith("_")}
    if a.policy == "EXT_HIER":
        tr["region"] = torch.from_numpy(fa.mobility_regions(tr["arrive"].cpu().numpy(), a.N)).to(dev)
    out = fa.run_batch(ctx, tr, policy=a.policy)
    torch.cuda.synchronize()
    st = out.rep_stats()
    assert (st["status"] == 0).all(), np.unique(st["status"])
    dec = float(st["n_tasks"].sum())
    res = {"cycles_per_decision": {n: float(st[f].astype(np.float64).sum() / dec) for f, n in SEG},
           "per_decision": {n: float(st[f].astype(np.float64).sum() / dec) for f, n in CNT}}
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt)


if __name__ == "__main__":
    main()
