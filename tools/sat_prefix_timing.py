"""Where the saturated C5 step's time goes along the trace: the sequential EXT_HIER replay
(replay_wide_kernel, FOGNET_HIER_REGIONS=0) of the saturating recipe (bench.py --workload c5
--c5-recipe saturate, R = 1,024) cut at several prefix lengths T' (the same publishes: the
T = 32,768 trace sliced), min of 3 launches each, and the region pass on the same prefixes
(FOGNET_HIER_REGIONS=only: a replication finishes there, status 0, only when its prefix has no
escalation, so the counts over the cuts bound each replication's first escalation).  GPU;
diagnostics only (what resuming instead of restarting would save)."""
import os, subprocess, sys, time, json
import numpy as np

HERE = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, HERE)


def child(mode, cuts, R):
    os.environ["FOGNET_HIER_REGIONS"] = mode
    import torch
    import fognetsimpp_amd as fa
    T, N = 32_768, 10_000
    dev = torch.device("cuda", 0)
    ctx = fa.Context(0)
    full = fa.saturating_trace(0x5EED0005, R, T, N)
    res = {}
    for c in cuts:
        tr = {k: (np.ascontiguousarray(v[:, :c]) if k in ("arrive", "req", "region") else v) for k, v in full.items()}
        tr = fa.as_device_trace(tr, dev)
        out = fa.allocate_outputs(R, c, dev, N=N, energy=False, hist=True)
        ts = []
        for _ in range(3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            fa.run_batch(ctx, tr, out, policy="EXT_HIER", hier_threshold_s=60, hier_up_tick=20 * 10**9)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
        st = out.rep_stats()
        res[c] = dict(ms=round(1e3 * min(ts), 3), status_ok=int((st["status"] == 0).sum()))
        print(mode, c, res[c], flush=True)
    print("RESULT", json.dumps({"mode": mode, "R": R, "res": {str(k): v for k, v in res.items()}}), flush=True)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "child":
        child(sys.argv[2], [int(x) for x in sys.argv[3].split(",")], int(sys.argv[4]))
        sys.exit(0)
    R = int(os.environ.get("R", "1024"))
    cuts = os.environ.get("CUTS", "4096,8192,12288,16384,20480,24576,28672,32768")
    for mode in ("0", "only"):
        rc = subprocess.call([sys.executable, __file__, "child", mode, cuts, str(R)])
        if rc != 0:
            sys.exit(rc)
