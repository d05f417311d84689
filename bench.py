"""Benchmark: task-offload decisions/sec of the batched FogNetSim++ replay engine.

Default workload (BASELINE.json configs[2], SURVEY.md §8(d) C3 "policy sweep"):
per GPU R = 4096 replications x T = 100,000 tasks x N = 256 fog nodes, rho x
latency sweep, synthetic traces generated on the device (Philox recipe,
untimed).  One step = one pass of the hot path over the batch: the replay
kernel (decisions + node queues + adverts), the statistics pass (queueTime /
response moments, latency histograms, node energy) and the exact job-level
reduction; with N > 1 ranks also the all-gather of the job record and the
RCCL all-reduce of histograms + energy.  Replications are sharded over ranks
(weak scaling; no data-path collective).

``--workload c5`` runs config C5 (large topology, BASELINE.json configs[4]):
1024 replications in total x T = 10,000 x N = 10,000 fog nodes, sharded over
the ranks (strong scaling), with the builder-defined light-load recipe of
``fognetsimpp_amd.c5_params``: the default EXT_HIER policy (hierarchical
brokers + mobility handoff) on the region kernel (replay_region.hip: one
wavefront per regional broker while no region escalates, the sequential wide
kernel for a replication that does), ``--policy REF_V3`` on the wide replay
kernel (replay_wide.hip).

``--workload c1`` runs config C1 (the reference's example General run,
BASELINE.json configs[0]) with the modules its ini names (BrokerBaseApp2 +
ComputeBrokerApp2, the v2 model): per replication one user publishing every
50 ms for 1000 s (mqttApp2's timer chain, glibc rand() seeded with the global
replication index + 1), broker and 5 nodes at 1000 MIPS, 1-ms links;
replications sharded over the ranks (``--R-total``, default 4096, strong
scaling).  Traces are generated on the host before timing.

``--workload c4`` runs config C4 (Monte Carlo what-if, BASELINE.json
configs[3]): 1M replications x T = 10,000 x N = 256 in total, sharded over the
ranks (strong scaling), replayed in blocks of ``--block`` replications by
fognet_run_generated_dev: each 64-publish chunk of a trace is generated inside
the replay kernel (the whole trace would be ~120 GB) and only statistics are
kept (no trace and no per-task output in memory).

  python bench.py [--gpus N --steps K --warmup W] [--workload c1|c3|c4|c5]
  torchrun --nproc-per-node N bench.py --gpus N ...
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import fognetsimpp_amd as fa  # noqa: E402
import fognetsimpp_amd.dist  # noqa: E402,F401
from fognetsimpp_amd import _abi  # noqa: E402

METRIC = "task-offload decisions/sec (node) at R×T×N; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)


def algorithmic_bytes_per_decision(T: int, N: int) -> float:
    """trace in (arrive i64 + req i32 = 12 B) + results out
    (node i32 + status u8 padded to 4 + start i64 + done i64 = 24 B) + the node
    SoA loaded and stored once per replication (2 x N x 48 B) amortised over T
    tasks: 36.25 B at C3, 132 B at C5."""
    return 12.0 + 24.0 + 2.0 * N * 48.0 / T


def reference_prefix(stats_np, arrive=None):
    """The reference's abort point over a batch (fognet_hip.h "Reference signal
    values"): replications whose reference run ends at an overflowing queueTime
    emission, and the decisions the reference defines (publishes with
    arrive_tick <= abort_tick; every publish of a replication that completes).
    ``arrive``: the device trace [R, T] (None: statistics-only, no count)."""
    big = np.iinfo(np.int64).max
    ab = stats_np["abort_tick"]
    out = {"ref_aborted_replications": int((ab != big).sum()), "replications": int(len(ab))}
    if arrive is not None:
        abt = torch.from_numpy(np.ascontiguousarray(ab)).to(arrive.device)
        out["ref_defined_decisions"] = int((arrive <= abt[:, None]).sum().item())
    if (ab != big).any():
        out["first_abort_task_median"] = int(np.median(stats_np["abort_task"][ab != big]))
    return out


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
    ap.add_argument("--ring", type=int, default=2048)
    ap.add_argument("--seed", type=lambda s: int(s, 0), default=0x5EED0003)
    ap.add_argument("--cpu-reps", type=int, default=None,
                    help="replications in the CPU-baseline sample (default 1024; 256 for c5)")
    ap.add_argument("--cpu-threads", type=int, default=0, help="0: every CPU this job may use")
    ap.add_argument("--cpu-reps-1t", type=int, default=16, help="replications of the single-thread CPU sample")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--policy", default=None, choices=("REF_V3", "EXT_LAT", "EXT_HIER"),
                    help="default REF_V3; c5: EXT_HIER (hierarchical brokers + mobility handoff, BASELINE configs[4])")
    ap.add_argument("--hier-threshold-s", type=int, default=60)
    ap.add_argument("--hier-up-ms", type=int, default=20)
    ap.add_argument("--c5-recipe", default="light", choices=("light", "saturate"),
                    help="c5: 'light' = fa.c5_params (device-generated; no region escalates), 'saturate' = "
                         "fa.saturating_trace (host-built, T = 32,768: every region saturates and escalates)")
    ap.add_argument("--workload", default="c3", choices=("c1", "c3", "c4", "c5"))
    ap.add_argument("--v2-nodes", type=int, default=5, help="c1: compute brokers (the example has 5)")
    ap.add_argument("--R-total", type=int, default=None,
                    help="c4/c5: replications over all ranks (default 1,000,000 / 1024)")
    ap.add_argument("--block", type=int, default=0,
                    help="c4: replications per fognet_run_generated_dev call (0: the rank's whole shard in one "
                         "launch; its resident workgroups take replications from a work counter)")
    args = ap.parse_args()
    if args.policy is None:
        args.policy = "EXT_HIER" if args.workload == "c5" else "REF_V3"
    if args.workload in ("c4", "c5"):
        if args.T == 100_000:
            args.T = 32_768 if args.workload == "c5" and args.c5_recipe == "saturate" else 10_000
        if args.seed == 0x5EED0003:
            args.seed = 0x5EED0004 if args.workload == "c4" else 0x5EED0005
        if args.R_total is None:
            args.R_total = 1_000_000 if args.workload == "c4" else 1024
    if args.workload == "c1" and args.R_total is None:
        args.R_total = 4096
    if args.workload == "c5":
        if args.N == 256:
            args.N = 10_000
        if args.cpu_reps is None:
            args.cpu_reps = 256  # ~1 s on 16 threads (~17 CPU-seconds)
    if args.cpu_reps is None:
        args.cpu_reps = 1024

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    # one rank per GPU; FOGNET_BENCH_SHARE_GPU=1 lets ranks share devices (a
    # multi-rank rehearsal on a 1-GPU box, with FOGNET_BENCH_BACKEND=gloo)
    gpu = local % torch.cuda.device_count() if os.environ.get("FOGNET_BENCH_SHARE_GPU") == "1" else local
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    dist = None
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("FOGNET_BENCH_BACKEND", "nccl")  # nccl = RCCL over xGMI
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    ctx = fa.Context(gpu)
    if args.workload == "c4":
        return bench_c4(args, ctx, dev, dist, world, rank)
    if args.workload == "c1":
        return bench_c1(args, ctx, dev, dist, world, rank)
    T, N = args.T, args.N
    if args.workload == "c5":  # a fixed job split over the ranks
        from fognetsimpp_amd.dist import shard
        r0, R = shard(args.R_total, world, rank)
        mg, sc = fa.c5_params(np.arange(r0, r0 + R), N)
    else:  # C3: R replications per rank, contiguous blocks of the global index
        R = args.R
        r0 = rank * R
        mg, sc = fa.sweep_params(np.arange(r0, r0 + R), N)
    t0 = time.time()
    if args.workload == "c5" and args.c5_recipe == "saturate":
        trace = fa.as_device_trace(fa.saturating_trace(args.seed, R, T, N, r0=r0), dev)
    else:
        trace = fa.generate_trace(ctx, args.seed, R, T, N, mg, sc, r0=r0)
    pb, pi = fa.power_model(trace["mips"].cpu().numpy())
    trace["p_busy"] = torch.from_numpy(pb).to(dev)
    trace["p_idle"] = torch.from_numpy(pi).to(dev)
    if args.policy == "EXT_HIER" and "region" not in trace:  # each publish's regional broker (mobility model)
        trace["region"] = fa.mobility_regions(trace["arrive"], N)
    hier = dict(hier_threshold_s=args.hier_threshold_s, hier_up_tick=args.hier_up_ms * 10**9)
    out = fa.allocate_outputs(R, T, dev, N=N, energy=False, hist=True)
    torch.cuda.synchronize()
    log(f"[rank {rank}] trace generated R={R} T={T} N={N} in {time.time() - t0:.2f}s")

    job_buf = None
    energy = None

    def step(ev_a=None, ev_b=None):
        nonlocal job_buf, energy
        out.hist.zero_()
        if ev_a is not None:
            ev_a.record()
        # replay kernel with the statistics pass fused as its epilogue
        fa.run_batch(ctx, trace, out, ring_capacity=args.ring, stage="all", policy=args.policy, **hier)
        if ev_b is not None:
            ev_b.record()
        job_buf = torch.zeros(_abi.JOB_STATS_DTYPE.itemsize, dtype=torch.uint8, device=dev)
        ctx.check(ctx._lib.fognet_reduce_stats_dev(ctx.handle, fa.engine._ptr(out.stats), R,
                                                   fa.engine._ptr(job_buf), fa.engine._stream_ptr(dev)), "reduce")
        eo = _abi.JOB_STATS_DTYPE.fields["energy_j"][1]
        energy = job_buf[eo:eo + 8].view(torch.float64).clone()  # fognet_job_stats.energy_j
        if dist is not None:
            gathered = [torch.empty_like(job_buf) for _ in range(world)]
            dist.all_gather(gathered, job_buf)
            job_buf = torch.cat(gathered)
            fa.dist.allreduce_hist_energy(out.hist, energy)

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
    hist = out.hist.cpu().numpy()

    decisions = (args.R_total if args.workload == "c5" else world * R) * T * args.steps
    value = decisions / elapsed
    bpd = algorithmic_bytes_per_decision(T, N)
    achieved_gbs = R * T * bpd / replay_avg_s / 1e9

    traffic = None
    valu = None
    default_policy = "EXT_HIER" if args.workload == "c5" else "REF_V3"
    prof = os.path.join(ROOT, "profiles", ("pmc_traffic" if args.workload == "c3" else f"pmc_traffic_{args.workload}")
                        + ("" if args.policy == default_policy else f"_{args.policy}") + ".json")
    if os.path.exists(prof):
        try:
            pj = json.load(open(prof))
            if pj.get("config") == {"R": R, "T": T, "N": N, "ring": args.ring} and \
                    pj.get("policy", "REF_V3" if args.workload == "c3" else "EXT_HIER") == args.policy:
                traffic = pj.get("replay_hbm_bytes_per_launch") or pj.get("hbm_bytes_per_launch")
                if pj.get("valu_busy") is not None:
                    # the issue-side figure beside the byte-count roofline: VALU pipe occupancy on gfx950
                    # (SQ_INSTS_VALU x 2 cycles / SIMD / active cycles, tools/pmc_summary.py)
                    valu = {"busy": pj["valu_busy"], "peak": 1.0, "unit": "VALU pipe busy fraction",
                            "valu_per_decision": pj.get("SQ_INSTS_VALU_per_decision"),
                            "salu_per_decision": pj.get("SQ_INSTS_SALU_per_decision"),
                            "hbm_bytes_per_decision": (traffic / (R * T) if traffic else None),
                            "source": os.path.relpath(prof, ROOT)}
        except Exception:
            traffic = None
    ref = reference_prefix(rep, trace["arrive"])
    hier_esc = None
    if args.policy == "EXT_HIER" and N > _abi.HIER_REGION_NODES:
        # escalations of the last step: a publish escalated iff its node lies outside its regional broker's
        # region; a replication with any is handed back by the region pass to the sequential wide kernel
        esc = (out.node // _abi.HIER_REGION_NODES) != trace["region"]
        n_rep = torch.tensor([int(esc.any(dim=1).sum().item()), int(esc.sum().item())], dtype=torch.int64, device=dev)
        if dist is not None:
            dist.all_reduce(n_rep)
        hier_esc = {"escalating_replications": int(n_rep[0]), "escalating_fraction": int(n_rep[0]) / args.R_total,
                    "escalated_publishes": int(n_rep[1]), "threshold_s": args.hier_threshold_s}
        # the path each launch took (fognet_hier_path_stats, warm-up included): the region pass, or
        # straight to the sequential replay once a region pass handed most replications over
        hier_esc["region_launches"], hier_esc["sequential_launches"] = ctx.hier_path_stats()
    if dist is not None:  # job totals over the ranks' shards
        tot = torch.tensor([ref["ref_defined_decisions"], ref["ref_aborted_replications"], ref["replications"]],
                           dtype=torch.int64, device=dev)
        dist.all_reduce(tot)
        ref["ref_defined_decisions"], ref["ref_aborted_replications"], ref["replications"] = \
            (int(x) for x in tot.cpu().tolist())
    # the rate over the decisions the reference itself defines (the prefix up to each replication's abort
    # point): the same elapsed time, only the reference-defined decisions counted
    value_ref = ref["ref_defined_decisions"] * args.steps / elapsed
    ref["decisions_per_step"] = decisions // args.steps

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(trace, args, R, T, N, out=out)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "decisions/s",
            "value_ref_defined": value_ref,
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.workload == "c5" else "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": ("synthetic (host-built fa.saturating_trace: every region saturates, escalations to the parent)"
                     if args.workload == "c5" and args.c5_recipe == "saturate" else
                     "synthetic (device-generated Philox traces, "
                     + ("C5 light-load recipe)" if args.workload == "c5" else "C3 policy-sweep recipe)")),
            "config": {"workload": "C5 large topology (BASELINE.json configs[4])" if args.workload == "c5"
                       else "C3 policy sweep (BASELINE.json configs[2])", "R_per_gpu": R, "T": T, "N": N,
                       "R_total": args.R_total if args.workload == "c5" else R * world, "ring_capacity": args.ring,
                       "policy": {"REF_V3": "REF_V3 (BrokerBaseApp3)",
                                  "EXT_LAT": "EXT_LAT (north-star cost; not in the reference)",
                                  "EXT_HIER": f"EXT_HIER (regional brokers of 1024 nodes + parent, mobility handoff, "
                                              f"escalation above {args.hier_threshold_s} s, +{args.hier_up_ms} ms hop; "
                                              f"not in the reference)"}[args.policy],
                       "parallelism": f"replications sharded over {world} GPU(s)"},
            "roofline": {"bound": "hbm", "achieved": achieved_gbs, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved_gbs / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": (("replay_wide_kernel (sequential replay of every replication: the warm-up's "
                                     "region pass handed all of them over, so the automatic path choice skips it; "
                                     "fognet_hier_path_stats)" if hier_esc and hier_esc["sequential_launches"] >= args.steps
                                     else "replay_region_kernel (one wavefront per regional broker) + "
                                     "region_finish_kernel (statistics pass)" +
                                     (" + replay_region_kernel<2> and replay_wide_kernel (the escalated replications "
                                      "replayed again up to their first escalated publish, then continued "
                                      "sequentially from there)"
                                      if hier_esc and hier_esc["escalating_replications"] else ""))
                                    if args.policy == "EXT_HIER" and N > _abi.HIER_REGION_NODES
                                    else "replay_wide_kernel (statistics inline)" if N > 256
                                    else "replay_kernel (statistics pass fused)"), "kernel_avg_ms": replay_avg_s * 1e3,
                         "bytes_per_decision": bpd, "bytes_per_decision_source": "SURVEY.md §8(d)",
                         "valu_issue": valu},
            "cpu_baseline": cpu,
            "failed_replications": failed,
            "hier_escalation": hier_esc,
            # the reference run of a replication ends at its first overflowing queueTime emission
            # (ComputeBrokerApp3.cc:238, no handler): what it defines is the prefix up to that tick; the
            # decisions after it are the engine's extension (fognet_hip.h "Reference signal values")
            "reference_abort": ref,
            "stats": {"queueTime_ms_mean": summary["queueTime_ms"].get("mean"),
                      "queueTime_overflows": summary["queueTime_ms"].get("overflow"),
                      "response_ms_mean": summary["response_ms"].get("mean"),
                      "max_pending": summary["max_pending"], "decisions": summary["decisions"],
                      "energy_j": float(energy[0]), "busy_s": summary["busy_s"],
                      "hist_counts": [int(hist[0].sum()), int(hist[1].sum())]},
        }
        line["roofline"].update(rocprof_kernel_avg(args, line))
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def rocprof_kernel_avg(args, line):
    """The committed rocprofv3 average launch of the dominant kernel for this exact workload
    (profiles/kernel_profile_<workload>[_<policy>|_<recipe>].json, written by tools/kprof_sidecar.py from a
    kernel trace of the bench command itself).  Quoted only when the profiled run loaded the very library
    this run loaded (sha256 of the .so: a profile of another build is never quoted), its config
    equals this line's, and the average does not exceed the profiled run's own ms_per_step; both runs'
    ms_per_step are printed, so a box-to-box difference shows instead of rejecting the profile."""
    tag = args.workload + ("" if args.policy in (None, "EXT_HIER" if args.workload == "c5" else "REF_V3")
                           else f"_{args.policy}") + ("_saturate" if getattr(args, "c5_recipe", "light") == "saturate"
                                                     and args.workload == "c5" else "")
    path = os.path.join(ROOT, "profiles", f"kernel_profile_{tag}.json")
    if not os.path.exists(path) or line["n_gpus"] != 1:
        return {"kernel_avg_ms_rocprof": None}
    try:
        side = json.load(open(path))
    except ValueError:
        return {"kernel_avg_ms_rocprof": None}
    rel = os.path.relpath(path, ROOT)
    with open(_abi.LIB_PATH, "rb") as f:
        lib_sha = hashlib.sha256(f.read()).hexdigest()
    if side.get("lib_sha256") != lib_sha:
        return {"kernel_avg_ms_rocprof": None, "rocprof_profile_other_build": rel}
    if side.get("config") != line["config"] or side["avg_ms"] > side["ms_per_step"]:
        return {"kernel_avg_ms_rocprof": None, "rocprof_profile_rejected": rel}
    return {"kernel_avg_ms_rocprof": side["avg_ms"], "rocprof_profile": rel,
            "rocprof_ms_per_step": side["ms_per_step"], "ms_per_step_this_run": line["ms_per_step"],
            "rocprof_command": side["command"], "rocprof_lib_sha256": lib_sha[:16]}


def bench_c4(args, ctx, dev, dist, world, rank):
    """Config C4: R_total replications (sharded over ranks) x T x N, replayed
    in blocks of ``args.block`` replications by fognet_run_generated_dev: each
    64-publish chunk of a replication's trace is generated inside the replay
    kernel, no trace and no per-task output reaches
    memory; only the per-replication records (reduced to one job record per
    block), the histograms and the energy survive.  Generation is inside the
    timed region."""
    from fognetsimpp_amd.dist import shard
    T, N = args.T, args.N
    r0, n = shard(args.R_total, world, rank)
    B = args.block if args.block > 0 else n
    blocks = [(r0 + b, min(B, n - b)) for b in range(0, n, B)]
    mg_all, sc_all = fa.sweep_params(np.arange(r0, r0 + n), N)
    mg_d = torch.from_numpy(np.ascontiguousarray(mg_all)).to(dev)
    sc_d = torch.from_numpy(np.ascontiguousarray(sc_all)).to(dev)
    pb, pi = fa.power_model(1000 * (1 + np.arange(N) % 4))  # the generator's MIPS pattern, shared by all
    power = (torch.from_numpy(pb).to(dev), torch.from_numpy(pi).to(dev))
    out = fa.allocate_outputs(B, T, dev, N=N, energy=False, hist=True, per_task=False)
    jrec = torch.zeros((max(1, len(blocks)), _abi.JOB_STATS_DTYPE.itemsize), dtype=torch.uint8, device=dev)
    stream = fa.engine._stream_ptr(dev)
    log(f"[rank {rank}] c4: {n} replications in {len(blocks)} blocks of <= {B}, T={T} N={N} (generated in-kernel)")

    def step(evs=None):
        out.hist.zero_()
        for i, (b0, nb) in enumerate(blocks):
            o = fa.BatchResult(None, None, None, None, out.stats[: nb * _abi.REP_STATS_DTYPE.itemsize], None, out.hist)
            if evs is not None:
                evs[i][0].record()
            fa.run_generated(ctx, args.seed, nb, T, N, mg_d[b0 - r0: b0 - r0 + nb], sc_d[b0 - r0: b0 - r0 + nb],
                             r0=b0, out=o, ring_capacity=args.ring, policy=args.policy, power=power)
            if evs is not None:
                evs[i][1].record()
            ctx.check(ctx._lib.fognet_reduce_stats_dev(ctx.handle, fa.engine._ptr(o.stats), nb,
                                                       fa.engine._ptr(jrec[i]), stream), "reduce")
        job = fa.merge_job_stats(list(jrec.cpu().numpy().view(_abi.JOB_STATS_DTYPE).reshape(-1)[:len(blocks)]))
        if dist is not None:
            jb = fa.dist.job_record_tensor(job, dev)
            job = fa.dist.allgather_job_stats(jb)
            energy = torch.tensor([float(job["energy_j"])], dtype=torch.float64, device=dev)
            fa.dist.allreduce_hist_energy(out.hist, energy)
        return job

    for i in range(args.warmup):
        step()
        torch.cuda.synchronize()
        log(f"[rank {rank}] warmup {i + 1}/{args.warmup} done")
    evs = [[(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in blocks]
           for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        job = step(evs[i])
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    replay_ms = float(np.mean([sum(a.elapsed_time(b) for a, b in e) for e in evs]))
    summary = fa.summarize(job)
    hist = out.hist.cpu().numpy()
    decisions = args.R_total * T * args.steps
    # reference-defined decisions (publishes up to each replication's abort tick): the traces were generated
    # inside the replay kernel, so they are regenerated here (untimed) in blocks from the same recipe
    ref_defined = None
    if len(blocks) == 1:
        abt = torch.from_numpy(np.ascontiguousarray(out.rep_stats()["abort_tick"][:n])).to(dev)
        cnt, G = 0, 8192
        for g0 in range(0, n, G):
            ng = min(G, n - g0)
            tr = fa.generate_trace(ctx, args.seed, ng, T, N, mg_d[g0:g0 + ng], sc_d[g0:g0 + ng], r0=r0 + g0)
            cnt += int((tr["arrive"] <= abt[g0:g0 + ng, None]).sum().item())
            del tr
        tot = torch.tensor([cnt], dtype=torch.int64, device=dev)
        if dist is not None:
            dist.all_reduce(tot)
        ref_defined = int(tot.item())
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        # the CPU baseline replays the first block's first replications from the materialised trace; its
        # records must equal the generated replay's (parity)
        nb = min(args.cpu_reps, blocks[0][1])
        tr = fa.generate_trace(ctx, args.seed, nb, T, N, mg_d[:nb], sc_d[:nb], r0=r0)
        tr = {k: v for k, v in tr.items() if not k.startswith("_")}
        tr["p_busy"], tr["p_idle"] = (x.expand(nb, N) for x in power)
        o = fa.run_generated(ctx, args.seed, nb, T, N, mg_d[:nb], sc_d[:nb], r0=r0, ring_capacity=args.ring,
                             policy=args.policy, power=power, hist=False)
        torch.cuda.synchronize()
        cpu = cpu_baseline(tr, args, nb, T, N, out=o)
    # VALU utilisation (C4 has no per-task HBM traffic, so no HBM roofline) from the PMC pass
    # committed under profiles/ when it exists for this configuration
    valu = None
    prof = os.path.join(ROOT, "profiles", "pmc_valu_c4.json")
    if os.path.exists(prof):
        with open(prof) as f:
            pj = json.load(f)
        if pj.get("config") == {"T": T, "N": N, "block": args.block, "ring": args.ring, "policy": args.policy}:
            valu = pj.get("valu_busy")
    if rank == 0:
        line = {
            "metric": METRIC, "value": decisions / elapsed, "unit": "decisions/s",
            "value_ref_defined": (ref_defined * args.steps / elapsed) if ref_defined is not None else None,
            "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (Philox traces generated inside the replay kernel, C4 recipe)",
            "config": {"workload": "C4 Monte Carlo what-if (BASELINE.json configs[3])", "R_total": args.R_total,
                       "T": T, "N": N, "block": B, "ring_capacity": args.ring, "policy": args.policy,
                       "parallelism": f"replications sharded over {world} GPU(s); RCCL all-reduce of histograms"
                                      f" + energy, all-gather of the job record"},
            "roofline": {"bound": "valu", "achieved": valu, "peak": 1.0, "unit": "VALU busy fraction",
                         "frac": valu, "traffic": None,
                         "kernel": "replay_gen_kernel (trace generated per 64-publish chunk, statistics in "
                                   "registers, no per-task stores)",
                         "kernel_ms_per_step": replay_ms,
                         "note": "SURVEY.md §8(d): C4 has no per-task HBM traffic, so VALU pipe occupancy "
                                 "(PMC: SQ_INSTS_VALU*2/SIMDs/GRBM_GUI_ACTIVE per XCD, gfx950's 2-cycle "
                                 "wave64 issue; profiles/pmc_valu_c4.json) replaces the HBM fraction"},
            "cpu_baseline": cpu,
            "failed_replications": summary["failed"],
            "reference_abort": {"ref_aborted_replications": summary["ref_aborted"], "replications": args.R_total,
                                "ref_defined_decisions": ref_defined,
                                "decisions_per_step": args.R_total * T},
            "stats": {"decisions": summary["decisions"], "queueTime_ms_mean": summary["queueTime_ms"].get("mean"),
                      "response_ms_mean": summary["response_ms"].get("mean"), "energy_j": summary["energy_j"],
                      "max_pending": summary["max_pending"], "hist_counts": [int(hist[0].sum()), int(hist[1].sum())]},
        }
        line["roofline"].update(rocprof_kernel_avg(args, line))  # (the committed kernel trace of this library)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def bench_c1(args, ctx, dev, dist, world, rank):
    """Config C1 on the v2 model replay (fognet_run_v2_dev)."""
    from fognetsimpp_amd import formats
    from fognetsimpp_amd.dist import shard
    MS = 10**9
    stop = 1000 * 10**12  # wirelessNet.ini:50 stopTime = 1000 s
    n_nodes = args.v2_nodes  # wirelessNet.ini: 5 ComputeBrokers (more: a timing of the v2 kernel's wider node sets)
    r0, R = shard(args.R_total, world, rank)
    t0 = time.time()
    gens = [formats.gen_trace_mqtt(r0 + r + 1, [0], [50 * MS], [MS], [-1], stop) for r in range(R)]  # :48 sendInterval
    T = max(g["arrive"].size for g in gens)
    arrive = np.full((R, T), stop, np.int64)  # padding publishes at the stop tick never run
    req = np.zeros((R, T), np.int32)
    for r, g in enumerate(gens):
        arrive[r, :g["arrive"].size] = g["arrive"]
        req[r, :g["req"].size] = g["req"]
    tr = fa.as_device_trace(dict(arrive=arrive, req=req, mips=np.full(n_nodes, 1000, np.int32),
                                 dl=np.full(n_nodes, MS, np.int64), ul=np.full(n_nodes, MS, np.int64),
                                 first_adv=np.full(n_nodes, 20 * MS, np.int64)), dev)
    torch.cuda.synchronize()
    log(f"[rank {rank}] c1: {R} replications x {T} publishes generated in {time.time() - t0:.1f}s")

    def step():
        return fa.run_v2(ctx, tr, 1000, stop, 0.01)  # wirelessNet.ini:58,64 MIPS = 1000; mqttApp2.cc:372

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        ev[i][0].record()
        out = step()
        ev[i][1].record()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if dist is not None:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kern_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    st = out.rep_stats()
    decisions_rank = int(st["n_tasks"].sum())
    total = torch.tensor([decisions_rank, int(st["events"].sum()), int((st["status"] != 0).sum())],
                         dtype=torch.int64, device=dev)
    if dist is not None:
        dist.all_reduce(total)
    decisions, events, failed = (int(x) for x in total.cpu().tolist())
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import oracle_lib
        reps = min(R, 1024)  # ~10-30 s of single-core work in total
        threads = host_cpu_info()[3] if args.cpu_threads <= 0 else args.cpu_threads
        t1 = time.perf_counter()
        o = oracle_lib.run_v2(arrive[:reps], req[:reps], 1000, np.full(n_nodes, 1000, np.int32), np.full(n_nodes, MS),
                              np.full(n_nodes, MS), np.full(n_nodes, 20 * MS), stop, 0.01, threads=threads)
        dt = time.perf_counter() - t1
        same = bool(np.array_equal(o["node"], out.node[:reps].cpu().numpy()) and
                    np.array_equal(o["done"], out.done_tick[:reps].cpu().numpy()))
        share_value = float(o["stats"]["n_tasks"].sum()) / dt
        model, nproc, avail, _ = host_cpu_info()
        acc = {}

        def run_all(n, th):
            acc["o"] = oracle_lib.run_v2(arrive[:n], req[:n], 1000, np.full(n_nodes, 1000, np.int32),
                                         np.full(n_nodes, MS), np.full(n_nodes, MS), np.full(n_nodes, 20 * MS), stop,
                                         0.01, threads=th)

        n_all, r_all, dt_all = cpu_all_cores(run_all, R, per_thread=4)
        v_all = float(acc["o"]["stats"]["n_tasks"].sum()) / dt_all
        s1 = min(max(16, args.cpu_reps_1t), R)
        t1 = time.perf_counter()
        run_all(s1, 1)
        dt1 = time.perf_counter() - t1
        cpu = cpu_line(v_all, n_all, dt_all,
                       f"{r_all} replications of the same C1 traces (v2 oracle DES)", share_value, threads,
                       {"share_sample": f"{reps} replications, outputs identical to the device: {same}",
                        "share_wall_s": dt, "parity": same,
                        "single_thread_value": float(acc["o"]["stats"]["n_tasks"].sum()) / dt1,
                        "single_thread_sample": f"{s1} replications", "single_thread_wall_s": dt1,
                        "host_cpu": model, "host_nproc": nproc, "job_cpus": avail})
    if rank == 0:
        line = {
            "metric": METRIC, "value": decisions * args.steps / elapsed, "unit": "decisions/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (mqttApp2 task source, glibc rand() per replication)",
            "config": {"workload": "C1 example General run, v2 modules (BASELINE.json configs[0])",
                       "R_total": args.R_total, "T_max": T, "N": n_nodes, "model": "BrokerBaseApp2 + ComputeBrokerApp2",
                       "parallelism": f"replications sharded over {world} GPU(s)"},
            "roofline": {"bound": "latency", "achieved": None, "peak": None, "unit": None, "frac": None,
                         "traffic": None, "kernel": "replay_v2_rows_kernel<16, 2> (N <= 16: two replications per wavefront, two wavefronts per SIMD)",
                         "kernel_ms_per_step": kern_ms,
                         "events_per_s": events * args.steps / elapsed,
                         "note": "event-driven (~53 reference FES events per publish, counted in events_per_s; "
                                 "no-op adverts are left out of the queues and simple timer firings "
                                 "batched, DESIGN.md section 9); no HBM roofline applies"},
            "cpu_baseline": cpu, "failed_replications": failed,
            "stats": {"decisions": decisions, "events": events, "local": int(st["n_local"].sum()),
                      "forwarded": int(st["n_forwarded"].sum())},
        }
        line["roofline"].update(rocprof_kernel_avg(args, line))  # (the committed kernel trace of this library)
        print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def host_cpu_info():
    """CPU model, host logical CPUs, the CPUs in this process's affinity mask,
    and the share the GPU box allots this job (OMP_NUM_THREADS when set, else
    the mask)."""
    model = ""
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                model = ln.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    nproc = os.cpu_count() or 1
    avail = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else nproc
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    cores = min(avail, share) if share > 0 else avail
    return model, nproc, avail, cores


def cpu_all_cores(run, reps_max, per_thread=8):
    """Time ``run(reps, threads)`` (the oracle over the first ``reps``
    replications, statistics only) on EVERY CPU of this job's affinity mask
    ("with 1 thread, and with all cores"), one replication per
    thread at a time, ``per_thread`` replications per thread when the sample
    allows.  Returns (threads, reps, seconds)."""
    _, _, avail, _ = host_cpu_info()
    reps = min(reps_max, max(avail * per_thread, 1))
    t0 = time.perf_counter()
    run(reps, avail)
    return avail, reps, time.perf_counter() - t0


def cpu_baseline(trace, args, R, T, N, out=None):
    """Oracle (tests/oracle_lib: the CPU restatement, kind "port") timed on this
    host on a bounded sample of the same workload: on every CPU of this job's
    affinity mask (``value``), on the job's CPU share (OMP_NUM_THREADS; also the
    parity sample) and on 1 thread.  With ``out`` (the device outputs of the
    timed steps) the oracle's outputs on the share sample are compared with the
    device's: ``parity``."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import oracle_lib

    reps = min(args.cpu_reps, R)
    keys = ("arrive", "req", "mips", "dl", "ul", "init")
    model, nproc, avail, cores = host_cpu_info()
    reps_all = min(R, max(reps, 8 * avail))
    h = {k: trace[k][:reps_all].cpu().numpy() for k in keys}
    # the power model rides along when the device run used it (energy_j is part of the record compared),
    # and so do the policy and its inputs
    pw = {k: trace[k][:reps_all].cpu().numpy() for k in ("p_busy", "p_idle")} if "p_busy" in trace else {}
    pw["policy"] = oracle_lib.POLICIES[args.policy]
    if args.policy == "EXT_HIER":
        pw.update(region=trace["region"][:reps_all].cpu().numpy(), hier_threshold_s=args.hier_threshold_s,
                  hier_up_tick=args.hier_up_ms * 10**9)

    def cut(n):
        return {k: (v[:n] if isinstance(v, np.ndarray) and v.ndim >= 1 and v.shape[0] == reps_all else v)
                for k, v in pw.items()}

    threads = max(1, min(args.cpu_threads, cores)) if args.cpu_threads > 0 else cores
    log(f"cpu baseline: {reps} replications on {threads} threads (host {nproc} CPUs, {avail} in this job's mask) ...")
    t0 = time.perf_counter()
    o = oracle_lib.run_batch(*(h[k][:reps] for k in keys), threads=threads, outputs=True, **cut(reps))
    dt = time.perf_counter() - t0
    ok = int((o["stats"]["status"] == 0).sum())
    parity = None
    if out is not None and out.node is None:  # statistics-only device run: the records
        parity = o["stats"].tobytes() == out.stats[: reps * _abi.REP_STATS_DTYPE.itemsize].cpu().numpy().tobytes()
    elif out is not None:
        parity = bool(np.array_equal(o["node"], out.node[:reps].cpu().numpy())
                      and np.array_equal(o["status"], out.status[:reps].cpu().numpy())
                      and np.array_equal(o["start"], out.start_tick[:reps].cpu().numpy())
                      and np.array_equal(o["done"], out.done_tick[:reps].cpu().numpy())
                      and o["stats"].tobytes() == out.stats[: reps * _abi.REP_STATS_DTYPE.itemsize].cpu().numpy().tobytes())
    del o
    log(f"cpu baseline: {reps_all} replications on all {avail} CPUs of the mask ...")
    n_all, r_all, dt_all = cpu_all_cores(
        lambda n, th: oracle_lib.run_batch(*(h[k][:n] for k in keys), threads=th, outputs=False, **cut(n)), reps_all)
    s1 = min(max(16, args.cpu_reps_1t), reps)
    t1 = time.perf_counter()
    oracle_lib.run_batch(*(h[k][:s1] for k in keys), threads=1, outputs=False, **cut(s1))  # same policy/power/regions
    dt1 = time.perf_counter() - t1
    return cpu_line(r_all * T / dt_all, n_all, dt_all,
                    f"{r_all} replications x {T} tasks x {N} nodes (rank 0's first replications of the same trace, "
                    f"statistics only), one replication per thread at a time",
                    reps * T / dt, threads, {
            "share_sample": f"{reps} replications with per-task outputs on the job's CPU share ({threads} threads), "
                            f"{ok}/{reps} completed",
            "share_wall_s": dt,
            "single_thread_value": s1 * T / dt1, "single_thread_sample": f"{s1} replications",
            "single_thread_wall_s": dt1, "host_cpu": model, "host_nproc": nproc, "job_cpus": avail,
            "parity": parity,
            "parity_sample": f"oracle vs device outputs (node, status, start, done, stats record) on the {reps} "
                             f"replications of the share sample",
            "parity_scope": "device == oracle (the CPU restatement) over the whole replay. 'Bit-exact versus the "
                            "reference' is claimed only for the reference-defined prefix: where a replication's "
                            "reference run aborts at an overflowing queueTime emission (ComputeBrokerApp3.cc:238, "
                            "uncaught up to :84-86; reference_abort), the decisions after its abort_tick are the "
                            "engine's continuation (an extension the oracle restates identically), counted in "
                            "value but not in value_ref_defined; the oracle's stop-at-abort mode reproduces the "
                            "reference's end of run (tests)"})


def cpu_quota():
    """CPUs' worth of time the job's cgroup allows (cpu.max), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else float(q) / float(p)
    except (OSError, ValueError):
        return None


def cpu_line(v_all, n_all, dt_all, sample, v_share, n_share, extra):
    """The cpu_baseline object: ``value`` is the better of the all-CPU run (every
    CPU of the job's affinity mask) and the share run (OMP_NUM_THREADS), so the
    GPU is compared with the fastest CPU configuration measured; both are listed."""
    best_all = v_all >= v_share
    d = {"value": max(v_all, v_share), "unit": "decisions/s", "cores": n_all if best_all else n_share,
         "kind": "port",
         "sample": sample + (f" on all {n_all} CPUs of this job's affinity mask" if best_all
                             else f" on the job's CPU share of {n_share} threads (faster here than all {n_all} "
                                  f"CPUs of the mask: cgroup quota {cpu_quota()} CPUs)"),
         "all_cores": {"value": v_all, "threads": n_all, "wall_s": dt_all, "cgroup_cpu_quota": cpu_quota()},
         "share_value": v_share, "share_cores": n_share}
    d.update(extra)
    return d


if __name__ == "__main__":
    main()
