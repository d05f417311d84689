"""Multi-rank path on CPU (gloo, world size 2): sharding covers every
replication once, and the all-gathered job record merged with the product's
exact merge equals the single-process record."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from fognetsimpp_amd import _abi
from fognetsimpp_amd.dist import allgather_job_stats, allreduce_hist_energy, job_record_tensor, shard
from fognetsimpp_amd.engine import merge_job_stats


def job_from_rep_stats(st):
    """Test-side exact rep -> job record (what reduce_kernel computes on the device)."""
    rec = np.zeros(1, dtype=_abi.JOB_STATS_DTYPE)[0]
    rec["n_reps"] = len(st)
    ok = st[st["status"] == 0]
    rec["n_failed"] = len(st) - len(ok)
    for f in ("n_tasks", "n_queued", "n_started", "events", "busy_s"):
        rec[f] = int(ok[f].sum())
    rec["energy_j"] = float(np.sum(ok["energy_j"]))
    big = np.iinfo(np.int64)
    rec["last_tick"] = int(ok["last_tick"].max()) if len(ok) else big.min
    rec["queue_min_raw"] = int(ok["queue_min_raw"].min()) if len(ok) else big.max
    rec["resp_min_ticks"] = int(ok["resp_min_ticks"].min()) if len(ok) else big.max
    rec["queue_max_raw"] = int(ok["queue_max_raw"].max()) if len(ok) else big.min
    rec["n_qtime"] = int(ok["n_qtime"].sum())
    rec["n_qtime_overflow"] = int(ok["n_qtime_overflow"].sum())
    ab = st[(st["status"] == 0) | (st["status"] == _abi.FOGNET_REF_ABORTED)]  # counted under the flag too
    rec["n_ref_aborted"] = int((ab["abort_tick"] != np.iinfo(np.int64).max).sum())
    rec["resp_max_ticks"] = int(ok["resp_max_ticks"].max()) if len(ok) else big.min
    rec["max_pending"] = int(ok["max_pending"].max()) if len(ok) else 0
    for name, lo, hi in (("queue_sum", "queue_sum_lo", "queue_sum_hi"), ("queue_sq", "queue_sq_lo", "queue_sq_hi"),
                         ("resp_sum", "resp_sum_lo", "resp_sum_hi"), ("resp_sq", "resp_sq_lo", "resp_sq_hi")):
        vals = [int(a) | (int(b) << 64) for a, b in zip(ok[lo], ok[hi])]
        if name == "queue_sum":  # signed two's complement
            vals = [v - (1 << 128) if v >> 127 else v for v in vals]
        if name == "queue_sq":
            vals = [v | (int(t) << 128) for v, t in zip(vals, ok["queue_sq_top"])]
        tot = sum(vals) % (1 << 192)
        rec[name] = [(tot >> (64 * i)) & (2**64 - 1) for i in range(3)]
    return rec


def test_shard_partitions():
    for total in (0, 1, 7, 4096, 1_000_000):
        for world in (1, 2, 3, 8):
            seen = []
            for rank in range(world):
                r0, n = shard(total, world, rank)
                seen.extend(range(r0, r0 + n))
            assert seen == list(range(total))


def _worker(rank, world, port, reps, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle_lib as ol
    import tracegen as tg
    r0, n = shard(reps, world, rank)
    recs = []
    hist = torch.zeros((_abi.HIST_METRICS, _abi.HIST_BINS), dtype=torch.int64)
    for r in range(r0, r0 + n):
        o = _replicate(ol, tg, r)
        recs.append(o["stats"])
        hist += torch.from_numpy(o["hist"].sum(axis=0))
    st = np.concatenate(recs).view(_abi.REP_STATS_DTYPE) if recs else np.zeros(0, _abi.REP_STATS_DTYPE)
    merged = allgather_job_stats(job_record_tensor(job_from_rep_stats(st), torch.device("cpu")))
    energy = torch.tensor([float(np.sum(st["energy_j"]))], dtype=torch.float64)
    allreduce_hist_energy(hist, energy)
    if rank == 0:
        q.put((merged.tobytes(), hist.numpy().copy(), float(energy[0])))
    dist.destroy_process_group()


def _replicate(ol, tg, r):
    import fognetsimpp_amd as fa
    rp = tg.make_replication(77, r, 16, 400, rho=(0.5, 0.9)[r % 2])
    pb, pi = fa.power_model(rp["mips"])
    return ol.run_batch(rp["arrive"], rp["req"], rp["mips"], rp["dl"], rp["ul"], rp["init"], p_busy=pb, p_idle=pi,
                        hist=True)


def free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(120)
def test_gloo_world2_job_stats_match_single_process():
    import oracle_lib as ol
    import tracegen as tg
    reps = 5
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, reps, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, got_hist, got_energy = q.get(timeout=110)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    outs = [_replicate(ol, tg, r) for r in range(reps)]
    st = np.concatenate([o["stats"] for o in outs]).view(_abi.REP_STATS_DTYPE)
    np.testing.assert_array_equal(got_hist, sum(o["hist"].sum(axis=0) for o in outs))
    assert got_hist[1].sum() == reps * 400
    np.testing.assert_allclose(got_energy, float(np.sum(st["energy_j"])), rtol=1e-12)
    assert got_energy > 0
    single = job_from_rep_stats(st)
    assert got == merge_job_stats([single]).tobytes()
    # and the merge is associative: per-replication records merged one by one
    one_by_one = merge_job_stats([job_from_rep_stats(st[i:i + 1]) for i in range(reps)])
    assert one_by_one.tobytes() == got


# ------------------------------------------------------------------ C-ABI stats exchange (fognet_allreduce_stats)

def test_comm_unique_id_and_argument_checks():
    """RCCL is loaded on first use; ids are 128 opaque bytes; a communicator
    needs a context and a valid (world, rank)."""
    import ctypes as C

    from fognetsimpp_amd import _abi, dist

    a, b = dist.StatsComm.unique_id(), dist.StatsComm.unique_id()
    assert len(a) == _abi.COMM_ID_BYTES and a != b
    lib = _abi.load()
    h = C.c_void_p()
    uid = (C.c_uint8 * _abi.COMM_ID_BYTES).from_buffer_copy(a)
    assert lib.fognet_comm_create(None, 1, 0, uid, C.byref(h)) == _abi.FOGNET_ERR_ARG
    assert lib.fognet_allreduce_stats(None, None, None, None, None) == _abi.FOGNET_ERR_ARG
    lib.fognet_comm_destroy(None)  # no-op


@pytest.mark.gpu
def test_comm_allreduce_world1_is_identity(ctx):
    """World 1 over the library's own RCCL communicator: the merged record is
    this rank's record and the histogram is unchanged."""
    import torch

    import fognetsimpp_amd as fa
    import tracegen as tg
    from fognetsimpp_amd import dist

    dev = torch.device("cuda", 0)
    tr = tg.make_batch(0x5EED0001, 4, 64, 3000)
    out = fa.run_batch(ctx, fa.as_device_trace(tr, dev), hist=True)
    torch.cuda.synchronize()
    job = fa.job_from_reps(out.rep_stats())
    hist0 = out.hist.clone()
    comm = dist.StatsComm(ctx, 1, 0, dist.StatsComm.unique_id())
    try:
        merged = comm.allreduce(job, out.hist)
    finally:
        comm.close()
    assert merged.tobytes() == job.tobytes()
    assert torch.equal(out.hist, hist0)


# ------------------------------------------------------------------ HIP engine in every rank (world 2, one GPU)

def _gpu_worker(rank, world, port, R_total, T, N, q):
    """One rank: replay its contiguous block of the global replications on the
    GPU (device Philox traces keyed by the global index), reduce on the device,
    all-gather the job record and all-reduce the histogram + energy over gloo
    (both ranks share cuda:0 on a one-GPU box, which RCCL does not allow)."""
    import fognetsimpp_amd as fa
    from fognetsimpp_amd import engine
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        dev = torch.device("cuda", 0)
        ctx = fa.Context(0)
        r0, n = shard(R_total, world, rank)
        mg, sc = fa.sweep_params(np.arange(r0, r0 + n), N)
        tr = fa.generate_trace(ctx, 0x5EED0003, n, T, N, mg, sc, r0=r0)
        pb, pi = fa.power_model(tr["mips"].cpu().numpy())
        tr["p_busy"], tr["p_idle"] = torch.from_numpy(pb).to(dev), torch.from_numpy(pi).to(dev)
        out = fa.run_batch(ctx, tr, hist=True)
        job = fa.reduce_stats(ctx, out.stats, n)
        torch.cuda.synchronize()
        hist = out.hist.cpu()
        energy = torch.tensor([float(job["energy_j"])], dtype=torch.float64)
        merged = allgather_job_stats(job_record_tensor(job, torch.device("cpu")))
        allreduce_hist_energy(hist, energy)
        if rank == 0:
            q.put((merged.tobytes(), hist.numpy().copy(), float(energy[0])))
        del out, tr
        ctx.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.timeout(240)
def test_gloo_world2_hip_engine_matches_single_rank(ctx):
    """two ranks each replay their block of C3-recipe
    replications through libfognet_hip; the merged job record and histogram
    equal one rank replaying all of them (integer fields bit-exact, the fp64
    energy sum within 1e-12 relative), and the histogram counts every task."""
    import fognetsimpp_amd as fa
    R_total, T, N = 6, 3000, 256
    dev = torch.device("cuda", 0)
    mg, sc = fa.sweep_params(np.arange(R_total), N)
    tr = fa.generate_trace(ctx, 0x5EED0003, R_total, T, N, mg, sc)
    pb, pi = fa.power_model(tr["mips"].cpu().numpy())
    tr["p_busy"], tr["p_idle"] = torch.from_numpy(pb).to(dev), torch.from_numpy(pi).to(dev)
    out = fa.run_batch(ctx, tr, hist=True)
    single = fa.reduce_stats(ctx, out.stats, R_total)
    torch.cuda.synchronize()
    single_hist = out.hist.cpu().numpy()

    mpx = mp.get_context("spawn")
    q = mpx.Queue()
    port = free_port()
    procs = [mpx.Process(target=_gpu_worker, args=(r, 2, port, R_total, T, N, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got, got_hist, got_energy = q.get(timeout=200)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.exitcode is None:
                p.kill()
    assert all(p.exitcode == 0 for p in procs)
    got_rec = np.frombuffer(got, dtype=_abi.JOB_STATS_DTYPE)[0]
    assert int(got_rec["n_reps"]) == R_total and int(got_rec["n_failed"]) == 0
    assert int(got_rec["n_tasks"]) == R_total * T
    np.testing.assert_array_equal(got_hist, single_hist)
    assert got_hist[1].sum() == R_total * T
    np.testing.assert_allclose(got_energy, float(single["energy_j"]), rtol=1e-12)
    a, b = got_rec.copy(), np.array(single).copy().reshape(-1)[0]
    a["energy_j"] = b["energy_j"] = 0.0
    assert a.tobytes() == b.tobytes()
