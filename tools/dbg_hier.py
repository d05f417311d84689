"""Debug: EXT_HIER / forced-wide REF_V3 on small traces against the oracle; status and first divergent task."""
import os, sys
import numpy as np, torch
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
from fognetsimpp_amd import _abi
_abi.LIB_PATH = os.environ.get("FOGNET_LIB", _abi.LIB_PATH)
import fognetsimpp_amd as fa, tracegen as tg, oracle_lib as ol
ctx = fa.Context(0)
dev = torch.device("cuda", 0)
thr, up = 5, 20 * 10**9
tr = tg.make_batch(19, 3, 2500, 3000, rho=0.8)
tr = dict(tr, region=fa.mobility_regions(tr["arrive"], tr["mips"].shape[-1], users=37))
for pol in ("REF_V3", "EXT_HIER"):
    os.environ["FOGNET_REPLAY_KERNEL"] = "wide"
    kw = dict(hier_threshold_s=thr, hier_up_tick=up) if pol == "EXT_HIER" else {}
    out = fa.run_batch(ctx, fa.as_device_trace(tr, dev), policy=pol, hist=True, **kw)
    torch.cuda.synchronize()
    st = out.rep_stats()
    print(pol, "status", st["status"], "n_tasks", st["n_tasks"], flush=True)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8, hist=True,
                     policy=ol.POLICY_EXT_HIER if pol == "EXT_HIER" else 1, region=tr["region"] if pol == "EXT_HIER" else None,
                     **({"hier_threshold_s": thr, "hier_up_tick": up} if pol == "EXT_HIER" else {}))
    for r in range(3):
        for k_gpu, k_ref in (("node", "node"), ("status", "status"), ("start_tick", "start"), ("done_tick", "done")):
            g = getattr(out, k_gpu)[r].cpu().numpy(); x = o[k_ref][r]
            bad = np.nonzero(g != x)[0]
            if bad.size:
                i = bad[0]
                print(pol, r, k_gpu, "first mismatch task", i, "gpu", g[max(0, i - 2):i + 3], "ref", x[max(0, i - 2):i + 3])
                break
