"""v2 model replay (fognet_run_v2_dev) time per step at wider node sets (N = 300 and
1,024 run replay_v2_kernel<8> / <16>, whose per-node arrays spill to scratch).  C1's recipe (one
user, 50-ms publishes, 1-ms links, 1000 MIPS everywhere) with a shorter stop time: every node
fires its ADVERTISEMIPS timer every 10 ms, so the events per replication grow with N.
  python tools/v2_nodes_timing.py <R> <stop_s> <N> [<N> ...]"""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fognetsimpp_amd import _abi  # noqa: E402
if os.environ.get("FOGNET_LIB"):  # a variant build (tools/build_variant.sh)
    _abi.LIB_PATH = os.environ["FOGNET_LIB"]
import fognetsimpp_amd as fa  # noqa: E402
from fognetsimpp_amd import formats  # noqa: E402

R, stop_s = int(sys.argv[1]), float(sys.argv[2])
MS = 10**9
stop = int(stop_s * 10**12)
ctx = fa.Context(0)
dev = torch.device("cuda", 0)
gens = [formats.gen_trace_mqtt(r + 1, [0], [50 * MS], [MS], [-1], stop) for r in range(R)]
T = max(g["arrive"].size for g in gens)
arrive = np.full((R, T), stop, np.int64)
req = np.zeros((R, T), np.int32)
for r, g in enumerate(gens):
    arrive[r, :g["arrive"].size] = g["arrive"]
    req[r, :g["req"].size] = g["req"]
for n in (int(x) for x in sys.argv[3:]):
    tr = fa.as_device_trace(dict(arrive=arrive, req=req, mips=np.full(n, 1000, np.int32), dl=np.full(n, MS, np.int64),
                                 ul=np.full(n, MS, np.int64), first_adv=np.full(n, 20 * MS, np.int64)), dev)
    out = fa.run_v2(ctx, tr, 1000, stop, 0.01)  # warm-up
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = fa.run_v2(ctx, tr, 1000, stop, 0.01)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    ev = int(out.rep_stats()["events"].sum())
    print(f"N={n} R={R} T={T} stop={stop_s}s: {dt * 1e3:.1f} ms/step, {ev} FES events, "
          f"{ev / dt:.3g} events/s", flush=True)
