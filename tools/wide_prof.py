"""C5 loop counters of replay_wide_kernel (GPU; profile build:
EXTRA=-DFOGNET_WIDE_PROF tools/build_variant.sh wideprof, FOGNET_HIER_REGIONS=0 for the sequential EXT_HIER).  Per decision: publish
iterations, advert-loop iterations, adverts applied, adverts followed by a due
advert of the same node, adverts on the lane's cached node, group key rescans, runs."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fognetsimpp_amd import _abi
_abi.LIB_PATH = os.environ.get("FOGNET_LIB", "build/live/wideprof/libfognet_hip.so")
import fognetsimpp_amd as fa
R = int(sys.argv[1]) if len(sys.argv) > 1 else 256
T, N = 10_000, 10_000
dev = torch.device("cuda", 0)
ctx = fa.Context(0)
mg, sc = fa.c5_params(np.arange(R), N)
tr = fa.generate_trace(ctx, 0x5EED0005, R, T, N, mg, sc)
for pol in ("REF_V3", "EXT_HIER"):
    kw = {}
    if pol == "EXT_HIER":
        tr["region"] = fa.mobility_regions(tr["arrive"], N)
    out = fa.allocate_outputs(R, T, dev, N=N, energy=False, hist=True)
    fa.run_batch(ctx, tr, out, policy=pol)
    torch.cuda.synchronize()
    st = out.rep_stats()
    d = st["n_tasks"].astype(np.float64).sum()
    f = lambda k: st[k].astype(np.float64).sum() / d
    print(pol, "per decision: iterations %.3f advert-loop iterations %.3f adverts %.3f same-node-next %.3f cached %.3f "
          "group-key rescans %.3f runs %.3f" % (f("queue_sum_lo"), f("queue_sum_hi"), f("queue_sq_lo"), f("resp_sum_hi"),
                                               f("resp_sq_lo"), f("resp_sq_hi"), f("resp_sum_lo")), flush=True)
    seg = [("chunk_end", "queue_min_raw"), ("adverts", "queue_max_raw"), ("decision", "resp_min_ticks"),
           ("record", "resp_max_ticks"), ("run", "last_tick"), ("record_update", "queue_sq_top"), ("chunk_start", "busy_s")]
    tot = sum(st[k].astype(np.float64).sum() for _, k in seg)
    print(pol, "time split:", ", ".join("%s %.1f%%" % (n, 100 * st[k].astype(np.float64).sum() / tot) for n, k in seg),
          "| ticks per decision %.0f" % (tot / d))
