"""Benchmark: task-offload decisions/sec of the batched FogNetSim++ replay engine.

Workload (BASELINE.json configs[2], SURVEY.md §8(d) C3 "policy sweep"): per GPU
R = 4096 replications x T = 100,000 tasks x N = 256 fog nodes, rho x latency
sweep, synthetic traces generated on the device (Philox recipe, untimed).  One
step = one pass of the hot path over the batch: the replay kernel (decisions +
node queues + adverts), the per-replication statistics pass and the exact
job-level reduction (+ an all-gather of the job record when N > 1).
Replications are sharded over ranks (weak scaling; no data-path collective).

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import fognetsimpp_amd as fa  # noqa: E402
from fognetsimpp_amd import _abi  # noqa: E402

METRIC = "task-offload decisions/sec (node) at R×T×N; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def algorithmic_bytes_per_decision(T: int, N: int) -> float:
    """Trace in (arrive i64 + req i32) + results out (node i32 + status u8 +
    start i64 + done i64) + node parameters read once per replication
    (mips i32 + dl, ul, init i64) amortised over T tasks."""
    return 12.0 + 21.0 + N * 28.0 / T


def log(msg: str):
    print(msg, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--R", type=int, default=4096, help="replications per GPU")
    ap.add_argument("--T", type=int, default=100_000)
    ap.add_argument("--N", type=int, default=256)
    ap.add_argument("--ring", type=int, default=1024)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0003)
    ap.add_argument("--cpu-reps", type=int, default=1024, help="replications in the CPU-baseline sample")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-cpu", action="store_true")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    R, T, N = args.R, args.T, args.N
    r0 = rank * R  # contiguous shard of the global replication index space
    ctx = fa.Context(local)
    mg, sc = fa.sweep_params(np.arange(r0, r0 + R), N)
    t0 = time.time()
    trace = fa.generate_trace(ctx, args.seed, R, T, N, mg, sc, r0=r0)
    out = fa.allocate_outputs(R, T, dev)
    torch.cuda.synchronize()
    log(f"[rank {rank}] trace generated R={R} T={T} N={N} in {time.time() - t0:.2f}s")

    job_buf = None

    def step(ev_a=None, ev_b=None):
        nonlocal job_buf
        if ev_a is not None:
            ev_a.record()
        fa.run_batch(ctx, trace, out, ring_capacity=args.ring, stage="replay")
        if ev_b is not None:
            ev_b.record()
        fa.run_batch(ctx, trace, out, ring_capacity=args.ring, stage="stats")
        job_buf = torch.zeros(_abi.JOB_STATS_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        ctx.check(ctx._lib.fognet_reduce_stats_dev(ctx.handle, fa.engine._ptr(out.stats), R,
                                                   fa.engine._ptr(job_buf), fa.engine._stream_ptr(dev)), "reduce")
        if dist is not None:
            gathered = [torch.empty_like(job_buf) for _ in range(world)]
            dist.all_gather(gathered, job_buf)
            job_buf = torch.cat(gathered)

    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        log(f"[rank {rank}] warmup {i + 1}/{args.warmup} done")

    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(*evs[i])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    replay_ms = [a.elapsed_time(b) for a, b in evs]
    replay_avg_s = float(np.mean(replay_ms)) / 1e3

    # correctness of the timed work: every replication finished
    rep = out.rep_stats()
    failed = int((rep["status"] != 0).sum())
    jobs = job_buf.cpu().numpy().view(_abi.JOB_STATS_DTYPE)
    job = fa.merge_job_stats(list(jobs))
    summary = fa.summarize(job)

    decisions = world * R * T * args.steps
    value = decisions / elapsed
    bpd = algorithmic_bytes_per_decision(T, N)
    achieved_gbs = R * T * bpd / replay_avg_s / 1e9

    traffic = None
    prof = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(prof):
        try:
            pj = json.load(open(prof))
            if pj.get("config") == {"R": R, "T": T, "N": N, "ring": args.ring}:
                traffic = pj.get("replay_hbm_bytes_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(trace, args, R, T, N)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "decisions/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (device-generated Philox traces, C3 policy-sweep recipe)",
            "config": {"workload": "C3 policy sweep (BASELINE.json configs[2])", "R_per_gpu": R, "T": T, "N": N,
                       "R_total": R * world, "ring_capacity": args.ring, "policy": "REF_V3 (BrokerBaseApp3)",
                       "parallelism": f"replications sharded over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "replay_kernel", "kernel_avg_ms": replay_avg_s * 1e3,
                         "bytes_per_decision": bpd},
            "cpu_baseline": cpu,
            "failed_replications": failed,
            "stats": {"queueTime_ms_mean": summary["queueTime_ms"].get("mean"),
                      "response_ms_mean": summary["response_ms"].get("mean"),
                      "max_pending": summary["max_pending"], "decisions": summary["decisions"]},
        }
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def cpu_baseline(trace, args, R, T, N):
    """Oracle (tests/oracle_lib: the CPU restatement, kind "port") timed on this
    host on a bounded sample of the same workload."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    reps = min(args.cpu_reps, R)
    h = {k: trace[k][:reps].cpu().numpy() for k in ("arrive", "req", "mips", "dl", "ul", "init")}
    threads = max(1, min(args.cpu_threads, os.cpu_count() or 1))
    log(f"cpu baseline: {reps} replications on {threads} threads ...")
    t0 = time.perf_counter()
    o = oracle_lib.run_batch(h["arrive"], h["req"], h["mips"], h["dl"], h["ul"], h["init"], threads=threads,
                             outputs=True)
    dt = time.perf_counter() - t0
    ok = int((o["stats"]["status"] == 0).sum())
    # single-thread rate on 4 replications of the sample
    t1 = time.perf_counter()
    s4 = min(4, reps)
    oracle_lib.run_batch(h["arrive"][:s4], h["req"][:s4], h["mips"][:s4], h["dl"][:s4], h["ul"][:s4], h["init"][:s4],
                         threads=1)
    dt1 = time.perf_counter() - t1
    cpu_model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                cpu_model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": reps * T / dt, "unit": "decisions/s", "cores": threads, "kind": "port",
            "sample": f"{reps} replications x {T} tasks x {N} nodes (rank 0's first replications of the same "
                      f"trace), one replication per thread, {ok}/{reps} completed",
            "wall_s": dt, "single_thread_value": s4 * T / dt1, "host_cpu": cpu_model,
            "host_nproc": os.cpu_count()}


if __name__ == "__main__":
    main()
