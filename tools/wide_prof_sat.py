"""Loop counters and segment times of the sequential EXT_HIER replay (replay_wide_kernel) on the
saturating C5 recipe (bench.py --workload c5 --c5-recipe saturate; GPU; profile build:
EXTRA=-DFOGNET_WIDE_PROF tools/build_variant.sh wideprof).  Diagnostics only."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fognetsimpp_amd import _abi
_abi.LIB_PATH = os.environ.get("FOGNET_LIB", "build/live/wideprof/libfognet_hip.so")
os.environ["FOGNET_HIER_REGIONS"] = os.environ.get("REGIONS", "0")  # 0: the sequential kernel from the start; 1: resumed at the first escalation
import fognetsimpp_amd as fa
R = int(sys.argv[1]) if len(sys.argv) > 1 else 128
T, N = 32_768, 10_000
dev = torch.device("cuda", 0)
ctx = fa.Context(0)
tr = fa.as_device_trace(fa.saturating_trace(0x5EED0005, R, T, N), dev)
out = fa.allocate_outputs(R, T, dev, N=N, energy=False, hist=True)
fa.run_batch(ctx, tr, out, policy="EXT_HIER", hier_threshold_s=int(os.environ.get("THR", "60")),
             hier_up_tick=int(os.environ.get("UP_MS", "20")) * 10**9)
torch.cuda.synchronize()
st = out.rep_stats()
d = st["n_tasks"].astype(np.float64).sum()
f = lambda k: st[k].astype(np.float64).sum() / d
print("per decision: iterations %.3f advert-loop iterations %.3f adverts %.3f same-node-next %.3f cached %.3f "
      "group-key rescans %.3f runs %.3f" % (f("queue_sum_lo"), f("queue_sum_hi"), f("queue_sq_lo"), f("resp_sum_hi"),
                                           f("resp_sq_lo"), f("resp_sq_hi"), f("resp_sum_lo")), flush=True)
seg = [("chunk_end", "queue_min_raw"), ("adverts", "queue_max_raw"), ("decision", "resp_min_ticks"),
       ("record", "resp_max_ticks"), ("run", "last_tick"), ("record_update", "queue_sq_top"), ("chunk_start", "busy_s")]
tot = sum(st[k].astype(np.float64).sum() for _, k in seg)
print("time split:", ", ".join("%s %.1f%%" % (n, 100 * st[k].astype(np.float64).sum() / tot) for n, k in seg),
      "| ticks per decision %.0f" % (tot / d))
w = st["n_started"].astype(np.uint64)
print("backward walks per decision %.4f, walk steps per decision %.3f" % ((w & np.uint64(0xFFFFFFFF)).astype(np.float64).sum() / d,
                                                                        (w >> np.uint64(32)).astype(np.float64).sum() / d))
