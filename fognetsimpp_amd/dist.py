"""Multi-GPU plumbing for the replay engine.

Replications are independent, so a job is sharded by contiguous blocks of
the global replication index; each rank generates and replays its own block
(trace keys depend on the global index only, so results do not depend on the
number of GPUs).  The only collective is one all-gather of the per-rank
``fognet_job_stats`` record, merged with exact integer arithmetic
(``fognet_job_stats_merge``), so the integer job statistics (counts, 192-bit
moments, minima/maxima, histograms) are bit-identical for any sharding.  The
builder-defined energy ``energy_j`` is an fp64 sum whose rounding depends on
the sharding and the merge order: equal within 1e-9 relative, not bitwise
(include/fognet_hip.h).  Works with the ``nccl`` (RCCL) backend on device tensors and with
``gloo`` on CPU tensors.
"""
from __future__ import annotations

import numpy as np
import torch

from . import _abi
from .engine import merge_job_stats


def shard(r_total: int, world: int, rank: int) -> tuple[int, int]:
    """(first global replication, count) of ``rank``'s contiguous block;
    the first ``r_total % world`` ranks take one extra replication."""
    if world <= 0 or not 0 <= rank < world or r_total < 0:
        raise ValueError("bad shard request")
    q, rem = divmod(r_total, world)
    r0 = rank * q + min(rank, rem)
    return r0, q + (1 if rank < rem else 0)


def job_record_tensor(job, device) -> torch.Tensor:
    """A job record (JOB_STATS_DTYPE) as a uint8 tensor for collectives."""
    raw = np.frombuffer(np.ascontiguousarray(job).tobytes(), dtype=np.uint8).copy()
    return torch.from_numpy(raw).to(device)


def allgather_job_stats(job_bytes: torch.Tensor, group=None) -> np.ndarray:
    """All-gather each rank's job record (uint8 tensor of one JOB_STATS_DTYPE)
    and return the merge over ranks in rank order (the integer fields' merge
    is associative, so any order gives the same values; energy_j is an fp64
    sum taken in rank order)."""
    import torch.distributed as dist

    world = dist.get_world_size(group)
    parts = [torch.empty_like(job_bytes) for _ in range(world)]
    dist.all_gather(parts, job_bytes.contiguous(), group=group)
    recs = [p.cpu().numpy().view(_abi.JOB_STATS_DTYPE)[0] for p in parts]
    return merge_job_stats(recs)


def allreduce_hist_energy(hist: torch.Tensor, energy: torch.Tensor, group=None) -> None:
    """In-place sum over ranks of the job latency histograms (int64
    [FOGNET_HIST_METRICS, FOGNET_HIST_BINS], exact) and of the energy
    statistics (float64 tensor: job energy and per-node energy totals).  This
    is the one RCCL collective of the data path (north star: "RCCL over xGMI
    used only for the final all-reduce of latency histograms and energy
    statistics"); ~1 KB + 8 B x nodes, so it is latency-bound."""
    import torch.distributed as dist

    dist.all_reduce(hist, op=dist.ReduceOp.SUM, group=group)
    dist.all_reduce(energy, op=dist.ReduceOp.SUM, group=group)


class StatsComm:
    """The library's own stats exchange (``fognet_allreduce_stats``, the C-ABI
    path a C++/OMNeT++ host uses without PyTorch): one RCCL communicator per
    rank; the 128-byte id from :meth:`unique_id` on rank 0 reaches the other
    ranks over any channel (here typically ``torch.distributed.broadcast_object_list``)."""

    def __init__(self, ctx, world: int, rank: int, uid: bytes):
        import ctypes as C

        if len(uid) != _abi.COMM_ID_BYTES:
            raise ValueError("comm id must be 128 bytes")
        self._ctx = ctx
        self._lib = ctx._lib
        buf = (C.c_uint8 * _abi.COMM_ID_BYTES).from_buffer_copy(uid)
        h = C.c_void_p()
        ctx.check(self._lib.fognet_comm_create(ctx.handle, world, rank, buf, C.byref(h)), "comm_create")
        self._h = h

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C

        buf = (C.c_uint8 * _abi.COMM_ID_BYTES)()
        rc = _abi.load().fognet_comm_unique_id(buf)
        if rc != _abi.FOGNET_OK:
            raise _abi.FognetError(rc, "fognet_comm_unique_id")
        return bytes(buf)

    def allreduce(self, job, hist: torch.Tensor | None = None) -> np.ndarray:
        """Exact job record over all ranks (all-gather + rank-order merge);
        ``hist`` (device int64 [2, 64]) is summed in place."""
        import ctypes as C

        from .engine import _ptr, _stream_ptr

        js = _abi.JobStats.from_buffer_copy(np.ascontiguousarray(job).tobytes())
        dev = torch.device("cuda", self._ctx.device)
        self._ctx.check(self._lib.fognet_allreduce_stats(self._ctx.handle, self._h, C.byref(js),
                                                         _ptr(hist), _stream_ptr(dev)), "allreduce_stats")
        return np.frombuffer(bytes(js), dtype=_abi.JOB_STATS_DTYPE)[0]

    def close(self):
        if self._h:
            self._lib.fognet_comm_destroy(self._h)
            self._h = None
