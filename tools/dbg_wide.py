"""Debug: the wide kernel (forced) on the ring-overflow test trace against the oracle; first divergent task per replication."""
import os, sys
import numpy as np, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from fognetsimpp_amd import _abi
_abi.LIB_PATH = os.environ.get("FOGNET_LIB", _abi.LIB_PATH)
import fognetsimpp_amd as fa, tracegen as tg, oracle_lib as ol
ctx = fa.Context(0)
over = tg.make_batch(11, 3, 4, 2000, rho=3.0)
light = tg.make_batch(12, 5, 4, 2000, rho=0.3)
tr = {k: np.concatenate([light[k][:2], over[k], light[k][2:]]) for k in over}
dev = torch.device("cuda", 0)
os.environ["FOGNET_REPLAY_KERNEL"] = "wide"
d = fa.as_device_trace(tr, dev)
out = fa.run_batch(ctx, d, hist=True)
torch.cuda.synchronize()
st = out.rep_stats()
print("status", st["status"], "n_tasks", st["n_tasks"])
o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8, hist=True)
for r in range(8):
    for k_gpu, k_ref in (("node", "node"), ("status", "status"), ("start_tick", "start"), ("done_tick", "done")):
        g = getattr(out, k_gpu)[r].cpu().numpy(); x = o[k_ref][r]
        bad = np.nonzero(g != x)[0]
        if bad.size:
            i = bad[0]
            print(r, k_gpu, "first mismatch task", i, "gpu", g[max(0,i-2):i+3], "ref", x[max(0,i-2):i+3])
            break
