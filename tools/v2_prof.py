"""C1 loop profile (GPU; profile build: EXTRA=-DFOGNET_V2_PROF tools/build_variant.sh v2prof):
wave iterations, batch and generic steps per replication and per publish."""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fognetsimpp_amd import _abi
_abi.LIB_PATH = os.environ.get("FOGNET_LIB", "build/ab/v2prof/libfognet_hip.so")
import fognetsimpp_amd as fa
from fognetsimpp_amd import formats
MS = 10**9
stop = 1000 * 10**12
R = int(sys.argv[1]) if len(sys.argv) > 1 else 256
gens = [formats.gen_trace_mqtt(r + 1, [0], [50 * MS], [MS], [-1], stop) for r in range(R)]
T = max(g["arrive"].size for g in gens)
arrive = np.full((R, T), stop, np.int64); req = np.zeros((R, T), np.int32)
for r, g in enumerate(gens):
    arrive[r, :g["arrive"].size] = g["arrive"]; req[r, :g["req"].size] = g["req"]
dev = torch.device("cuda", 0)
ctx = fa.Context(0)
tr = fa.as_device_trace(dict(arrive=arrive, req=req, mips=np.full(5, 1000, np.int32), dl=np.full(5, MS, np.int64),
                             ul=np.full(5, MS, np.int64), first_adv=np.full(5, 20 * MS, np.int64)), dev)
out = fa.run_v2(ctx, tr, 1000, stop, 0.01)
torch.cuda.synchronize()
st = out.rep_stats()
pubs = st["n_tasks"].astype(np.float64)
print("per replication: wave iterations %.0f, batch steps %.0f, generic steps %.0f, batched firings %.0f, events %.0f" % (
    st["n_no_nodes"].mean(), st["n_dropped"].mean(), st["n_inflated"].mean(), st["n_rejected"].mean(), st["events"].mean()))
print("per publish: wave iterations %.2f, batch %.2f, generic %.2f, firings per batch %.2f, events %.2f" % (
    (st["n_no_nodes"] / pubs).mean(), (st["n_dropped"] / pubs).mean(), (st["n_inflated"] / pubs).mean(),
    (st["n_rejected"] / np.maximum(st["n_dropped"], 1)).mean(), (st["events"] / pubs).mean()))
seg = [("H minimum", "n_local"), ("K, M", "n_forwarded"), ("batch", "n_accepted"), ("generic step", "n_released_broker")]
tot = sum(st[k].astype(np.float64).sum() for _, k in seg)
print("time split:", ", ".join("%s %.1f%%" % (n, 100 * st[k].astype(np.float64).sum() / tot) for n, k in seg))
