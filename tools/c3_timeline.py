"""C3 timeline per replication (GPU; profile build FOGNET_REPLAY_PROFILE=3,
EXTRA=-DFOGNET_REPLAY_PROFILE=3 tools/build_variant.sh tl3): each wave's start, replay end and
epilogue end (s_memtime) written over its first outputs, summarised per load class
(rho = (0.5, 0.8, 0.95)[r % 3], fa.sweep_params) -- does the statistics epilogue of the
replications that finish early overlap the others' replay?   python tools/c3_timeline.py [R]"""
import os, sys
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fognetsimpp_amd import _abi
_abi.LIB_PATH = os.environ.get("FOGNET_LIB", "build/live/tl3/libfognet_hip.so")
import fognetsimpp_amd as fa
R = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
T, N = 100_000, 256
dev = torch.device("cuda", 0)
ctx = fa.Context(0)
mg, sc = fa.sweep_params(np.arange(R), N)
tr = fa.generate_trace(ctx, 0x5EED0003, R, T, N, mg, sc)
out = fa.allocate_outputs(R, T, dev, N=N, energy=False, hist=True)
for i in range(3):
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(); fa.run_batch(ctx, tr, out, ring_capacity=2048); b.record(); torch.cuda.synchronize()
    print("launch ms", round(a.elapsed_time(b), 3), flush=True)
d = out.done_tick[:, :4].cpu().numpy().astype(np.int64)
t0, t1, t2, slot = d[:, 0], d[:, 1], d[:, 2], d[:, 3]
# s_memtime counters are not synchronised across CUs: per-wave durations, and start/end
# offsets within each CU (slot >> 6: XCC | SE/SH/CU), where the counter is shared
rep = (t1 - t0).astype(np.float64)
epi = (t2 - t1).astype(np.float64)
cu = slot >> 6
off0 = np.zeros(R); end = np.zeros(R)
for c in np.unique(cu):
    m = cu == c
    off0[m] = t0[m] - t0[m].min()
    end[m] = t2[m] - t0[m].min()
r = np.arange(R)
print("per wave (ticks): replay min/median/max %.3g %.3g %.3g | epilogue min/median/max %.3g %.3g %.3g"
      % (rep.min(), np.median(rep), rep.max(), epi.min(), np.median(epi), epi.max()))
print("start offset within a CU: median %.3g max %.3g | end within a CU (from its first start): median %.3g max %.3g"
      % (np.median(off0), off0.max(), np.median(end), end.max()))
for c in range(3):
    m = r % 3 == c
    print("rho class %d: replay median %.3g max %.3g | epilogue median %.3g max %.3g | replay+epilogue max %.3g"
          % (c, np.median(rep[m]), rep[m].max(), np.median(epi[m]), epi[m].max(), (rep + epi)[m].max()))
# within each CU: does an early finisher's epilogue overlap a later replay?
ov = []
for c in np.unique(cu):
    m = np.where(cu == c)[0]
    le = (t1[m] - t0[m].min()).max()  # the CU's last replay end
    ov.append(((t2[m] - t0[m].min()) <= le).mean())
print("fraction of a CU's epilogues that end before the CU's last replay ends: median %.2f" % np.median(ov))
print("epilogue / (replay + epilogue) of the slowest wave per CU: median %.3f" % np.median(
    [epi[np.where(cu == c)[0]][np.argmax((t2 - t0)[cu == c])] / (t2 - t0)[cu == c].max() for c in np.unique(cu)]))
