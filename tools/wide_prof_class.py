"""Per load class (C5 recipe: rho = (0.002, 0.01, 0.05)[r % 3], latency x(1, 10, 100)[(r // 3) % 3])
cycle totals and segment split of the flat wide kernel (FOGNET_WIDE_PROF build, build/live/wideprof).
  python tools/wide_prof_class.py <R>"""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.getcwd())
from fognetsimpp_amd import _abi
_abi.LIB_PATH = "build/live/wideprof/libfognet_hip.so"
import fognetsimpp_amd as fa
R = int(sys.argv[1]); T, N = 10_000, 10_000
dev = torch.device("cuda", 0); ctx = fa.Context(0)
mg, sc = fa.c5_params(np.arange(R), N)
tr = fa.generate_trace(ctx, 0x5EED0005, R, T, N, mg, sc)
out = fa.allocate_outputs(R, T, dev, N=N, energy=False, hist=True)
fa.run_batch(ctx, tr, out, policy="REF_V3"); torch.cuda.synchronize()
st = out.rep_stats()
seg = ["queue_min_raw","queue_max_raw","resp_min_ticks","resp_max_ticks","last_tick","queue_sq_top","busy_s"]
tot = sum(st[k].astype(np.float64) for k in seg)
r = np.arange(R)
for a in range(3):
    for b in range(3):
        m = (r % 3 == a) & ((r // 3) % 3 == b)
        print(f"rho class {a} lat class {b}: ticks mean {tot[m].mean():.3g} max {tot[m].max():.3g} runs {st['resp_sum_lo'][m].mean():.0f} advit {st['queue_sum_hi'][m].mean():.0f}", flush=True)
print("max overall", tot.max(), "argmax r", int(tot.argmax()))
names = ["chunk_end", "adverts", "decision", "record", "run", "record_update", "chunk_start"]
for a in range(3):
    m = r % 3 == a
    print(f"rho class {a} split:", ", ".join(f"{n} {100 * st[k][m].astype(np.float64).sum() / tot[m].sum():.1f}%" for n, k in zip(names, seg)),
          f"| per run {tot[m].sum() / st['resp_sum_lo'][m].astype(np.float64).sum():.0f} ticks, adverts/run {st['queue_sq_lo'][m].astype(np.float64).sum() / st['resp_sum_lo'][m].astype(np.float64).sum():.2f}, gkey/run {st['resp_sq_hi'][m].astype(np.float64).sum() / st['resp_sum_lo'][m].astype(np.float64).sum():.2f}, hits/advert {st['resp_sq_lo'][m].astype(np.float64).sum() / max(1.0, st['queue_sq_lo'][m].astype(np.float64).sum()):.2f}", flush=True)
