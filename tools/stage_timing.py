"""Replay-only vs replay+fused-statistics kernel time at C3 (GPU; diagnostics only)."""
import sys, os, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fognetsimpp_amd import _abi
if os.environ.get("FOGNET_LIB"):  # time a variant build (tools/build_variant.sh)
    _abi.LIB_PATH = os.environ["FOGNET_LIB"]
import fognetsimpp_amd as fa

C5 = os.environ.get("WORKLOAD") == "c5"
R = int(sys.argv[1]) if len(sys.argv) > 1 else (1024 if C5 else 4096)
T, N = (10_000, 10_000) if C5 else (100_000, 256)
dev = torch.device("cuda", 0)
ctx = fa.Context(0)
mg, sc = (fa.c5_params if C5 else fa.sweep_params)(np.arange(R), N)
tr = fa.generate_trace(ctx, 0x5EED0005 if C5 else 0x5EED0003, R, T, N, mg, sc)
POL = os.environ.get("POLICY", "REF_V3")
if POL == "EXT_HIER":
    tr["region"] = fa.mobility_regions(tr["arrive"], N)
if os.environ.get("POWER"):  # the a11 power model (energy per node and per replication), as the bench runs it
    pb, pi = fa.power_model(tr["mips"].cpu().numpy())
    tr["p_busy"], tr["p_idle"] = torch.as_tensor(pb, device=dev), torch.as_tensor(pi, device=dev)
out = fa.allocate_outputs(R, T, dev, N=N, energy=bool(os.environ.get("POWER")), hist=True)
torch.cuda.synchronize()
for stage in os.environ.get("FOGNET_STAGES", "all,replay,stats,all,replay").split(","):
    ts = []
    for i in range(4):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(); fa.run_batch(ctx, tr, out, ring_capacity=2048, stage=stage, policy=POL); b.record()
        torch.cuda.synchronize(); ts.append(a.elapsed_time(b))
    print(os.path.basename(os.path.dirname(_abi.LIB_PATH)), POL, stage, ["%.2f" % t for t in ts], "min %.2f" % min(ts), flush=True)
