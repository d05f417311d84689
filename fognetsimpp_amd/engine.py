"""Host-side mirror of FogNetSim++'s offload-decision interface over libfognet_hip.

Device memory, streams and (for multi-GPU) RCCL come from PyTorch; every
decision, node update and statistic is computed by the gfx950 kernels in
``csrc/``.  Names follow the reference:

* :class:`BrokerBaseApp3` — the broker's allocation policy plug-in
  (``simple BrokerBaseApp3 like IUDPApp``, src/mqttapp/BrokerBaseApp3.ned:20);
  :meth:`BrokerBaseApp3.sendPubAck` is the decision core of
  ``BrokerBaseApp3::sendPubAck(..., status=false)`` (BrokerBaseApp3.cc:265-281).
* :class:`BrokerBaseApp2` — the v2 broker's local-first / "max-MIPS" forward
  (BrokerBaseApp2.cc:180-192, 235-286).
* :func:`run_v2` — replays of the v2 model (BrokerBaseApp2 + ComputeBrokerApp2).
* :class:`Context` + :func:`run_batch` — R independent trace replays of the
  broker/fog-node loop (BrokerBaseApp3.cc:123-158, ComputeBrokerApp3.cc:205-320).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass

import numpy as np
import torch

from . import _abi
from ._abi import FognetError

_TENSOR_DTYPES = {
    "arrive": torch.int64, "req": torch.int32, "mips": torch.int32,
    "dl": torch.int64, "ul": torch.int64, "init": torch.int64, "first_adv": torch.int64,
    "p_busy": torch.float64, "p_idle": torch.float64,  # optional power model (a11)
    "down": torch.int64,  # optional node crash ticks (node-down extension)
    "region": torch.int32,  # EXT_HIER: regional broker of each publish [R, T]
}
NEVER = np.iinfo(np.int64).max  # down tick of a node that never crashes
POLICIES = {"REF_V3": _abi.FOGNET_POLICY_REF_V3, "EXT_LAT": _abi.FOGNET_POLICY_EXT_LAT,
            "EXT_HIER": _abi.FOGNET_POLICY_EXT_HIER}


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _stream_ptr(device) -> C.c_void_p:
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


class Context:
    """A fognet_ctx bound to one HIP device (gfx950 required)."""

    def __init__(self, device: int | torch.device = 0):
        if isinstance(device, torch.device):
            device = device.index or 0
        self.device = int(device)
        self._lib = _abi.load()
        h = C.c_void_p()
        rc = self._lib.fognet_create(C.byref(h), self.device)
        if rc != _abi.FOGNET_OK:
            raise FognetError(rc, f"fognet_create(device={self.device}) failed: {_abi.status_string(rc)}")
        self._h = h

    @property
    def handle(self):
        return self._h

    def close(self):
        if getattr(self, "_h", None):
            self._lib.fognet_destroy(self._h)
            self._h = None

    def __del__(self):  # pragma: no cover - best effort
        try:
            self.close()
        except Exception:
            pass

    def check(self, rc: int, what: str = ""):
        if rc != _abi.FOGNET_OK:
            msg = self._lib.fognet_last_error(self._h).decode()
            raise FognetError(rc, f"{what}: {msg}" if what else msg)

    def sync(self):
        self.check(self._lib.fognet_sync(self._h), "sync")

    def hier_path_stats(self) -> tuple[int, int]:
        """EXT_HIER launches (N > 1024) that took the region pass / went straight to the
        sequential replay (fognet_hier_path_stats; FOGNET_HIER_REGIONS in fognet_hip.h)."""
        a, b = C.c_int64(0), C.c_int64(0)
        self.check(self._lib.fognet_hier_path_stats(self._h, C.byref(a), C.byref(b)), "hier_path_stats")
        return int(a.value), int(b.value)


class BrokerBaseApp3:
    """Allocation policy of BrokerBaseApp3 (src/mqttapp/BrokerBaseApp3.cc).

    ``brokers`` is the broker's view of the registered fog nodes in CONNECT
    order: advertised busy time (double) and MIPS (int) per node
    (Broker.cc:21-22, updated only by adverts, BrokerBaseApp3.cc:123-130).
    """

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def sendPubAck(self, adv_busy, adv_mips, MIPSRequired: int) -> int:  # noqa: N802,N803 (reference names)
        """Index of the node the task is offloaded to (BrokerBaseApp3.cc:267-281).

        Raises FognetError(FOGNET_ERR_NO_NODES) for an empty view (the reference
        dereferences brokers[0], UB) and FognetError(FOGNET_ERR_DIV0) when node 0
        has not advertised yet (MIPS 0: SIGFPE in the reference).
        """
        busy = np.ascontiguousarray(adv_busy, dtype=np.float64)
        mips = np.ascontiguousarray(adv_mips, dtype=np.int32)
        if busy.shape != mips.shape or busy.ndim != 1:
            raise FognetError(_abi.FOGNET_ERR_ARG, "adv_busy/adv_mips must be 1-D and equal length")
        out = C.c_int32(-1)
        lib = self.ctx._lib
        rc = lib.fognet_decide(self.ctx.handle, _abi.FOGNET_POLICY_REF_V3, len(busy),
                               busy.ctypes.data_as(C.c_void_p), mips.ctypes.data_as(C.c_void_p),
                               int(MIPSRequired), C.byref(out))
        self.ctx.check(rc, "sendPubAck")
        return out.value

    def sendPubAck_window(self, adv_busy, adv_mips, MIPSRequired) -> np.ndarray:  # noqa: N802,N803
        """The publishes of one window (no advert in between: one view) decided
        together (fognet_decide_window); equals one sendPubAck per request."""
        busy = np.ascontiguousarray(adv_busy, dtype=np.float64)
        mips = np.ascontiguousarray(adv_mips, dtype=np.int32)
        req = np.ascontiguousarray(MIPSRequired, dtype=np.int32).reshape(-1)
        if busy.shape != mips.shape or busy.ndim != 1:
            raise FognetError(_abi.FOGNET_ERR_ARG, "adv_busy/adv_mips must be 1-D and equal length")
        out = np.empty(len(req), np.int32)
        rc = self.ctx._lib.fognet_decide_window(self.ctx.handle, _abi.FOGNET_POLICY_REF_V3, len(busy),
                                                busy.ctypes.data_as(C.c_void_p), mips.ctypes.data_as(C.c_void_p),
                                                len(req), req.ctypes.data_as(C.c_void_p),
                                                out.ctypes.data_as(C.c_void_p))
        self.ctx.check(rc, "sendPubAck_window")
        return out

    def sendPubAck_batch(self, adv_busy: torch.Tensor, adv_mips: torch.Tensor, req: torch.Tensor):  # noqa: N802
        """M independent decisions on device tensors [M, n]; returns (node, status) int32 [M]."""
        m, n = adv_busy.shape
        node = torch.empty(m, dtype=torch.int32, device=adv_busy.device)
        status = torch.empty(m, dtype=torch.int32, device=adv_busy.device)
        rc = self.ctx._lib.fognet_decide_batch_dev(
            self.ctx.handle, _abi.FOGNET_POLICY_REF_V3, m, n,
            _ptr(adv_busy.contiguous()), _ptr(adv_mips.contiguous()), _ptr(req.contiguous()),
            _ptr(node), _ptr(status), _stream_ptr(adv_busy.device))
        self.ctx.check(rc, "decide_batch")
        return node, status


class BrokerBaseApp2:
    """Allocation policy of BrokerBaseApp2 (src/mqttapp/BrokerBaseApp2.cc, the
    module simulations/example/wirelessNet.ini:56 selects).

    Serves a task itself when MIPSRequired < its own remaining MIPS
    (``local_mips``: par MIPS minus its reservations, :181, :211); otherwise
    forwards to the LAST node whose advertised MIPS exceeds node 0's (the
    reference's "best broker" loop never updates its threshold, :241-248),
    and only if MIPSRequired < that node's MIPS (:262).
    """

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def sendPubAck(self, adv_mips, local_mips: int, MIPSRequired: int) -> tuple[int, int]:  # noqa: N802,N803
        """(action, node): action is _abi.V2_LOCAL / V2_FORWARD / V2_DROPPED /
        V2_NO_NODES; node is -1 for LOCAL and NO_NODES."""
        mips = np.ascontiguousarray(adv_mips, dtype=np.int32).reshape(-1)
        node, act = C.c_int32(-1), C.c_int32(0)
        rc = self.ctx._lib.fognet_decide_v2(self.ctx.handle, len(mips), mips.ctypes.data_as(C.c_void_p),
                                            int(local_mips), int(MIPSRequired), C.byref(node), C.byref(act))
        self.ctx.check(rc, "sendPubAck(v2)")
        return act.value, node.value

    def sendPubAck_batch(self, adv_mips: torch.Tensor, local_mips: torch.Tensor, req: torch.Tensor):  # noqa: N802
        """M independent decisions on device tensors adv_mips [M, n], local_mips [M],
        req [M]; returns (action, node) int32 [M]."""
        m, n = adv_mips.shape
        node = torch.empty(m, dtype=torch.int32, device=adv_mips.device)
        act = torch.empty(m, dtype=torch.int32, device=adv_mips.device)
        rc = self.ctx._lib.fognet_decide_v2_batch_dev(
            self.ctx.handle, m, n, _ptr(adv_mips.contiguous()), _ptr(local_mips.contiguous()), _ptr(req.contiguous()),
            _ptr(node), _ptr(act), _stream_ptr(adv_mips.device))
        self.ctx.check(rc, "decide_v2_batch")
        return act, node


@dataclass
class BatchResult:
    node: torch.Tensor | None        # [R, T] int32 (None: statistics only)
    status: torch.Tensor | None      # [R, T] uint8 (5 started / 4 queued)
    start_tick: torch.Tensor | None  # [R, T] int64
    done_tick: torch.Tensor | None   # [R, T] int64
    stats: torch.Tensor       # [R * sizeof(fognet_rep_stats)] uint8 (device)
    node_energy: torch.Tensor | None = None  # [R, N] float64 (power model only)
    hist: torch.Tensor | None = None         # [2, 64] int64 job histogram (queueTime, response), added to

    def rep_stats(self) -> np.ndarray:
        return self.stats.cpu().numpy().view(_abi.REP_STATS_DTYPE)


def allocate_outputs(R: int, T: int, device, N: int | None = None, energy: bool = False,
                     hist: bool = False, per_task: bool = True) -> BatchResult:
    """Output buffers; ``per_task=False``: statistics only (no per-task arrays:
    the replay writes nothing per task, fognet_batch_out)."""
    mk = (lambda shape, dt: torch.empty(shape, dtype=dt, device=device)) if per_task else (lambda shape, dt: None)
    return BatchResult(
        node=mk((R, T), torch.int32),
        status=mk((R, T), torch.uint8),
        start_tick=mk((R, T), torch.int64),
        done_tick=mk((R, T), torch.int64),
        stats=torch.zeros(R * _abi.REP_STATS_DTYPE.itemsize, dtype=torch.uint8, device=device),
        node_energy=torch.zeros((R, N), dtype=torch.float64, device=device) if energy else None,
        hist=torch.zeros((_abi.HIST_METRICS, _abi.HIST_BINS), dtype=torch.int64, device=device) if hist else None,
    )


def as_device_trace(trace: dict, device) -> dict:
    """numpy/torch trace dict -> contiguous device tensors of the ABI dtypes."""
    out = {}
    for k, dt in _TENSOR_DTYPES.items():
        if k not in trace or trace[k] is None:
            continue
        v = trace[k]
        t = v if isinstance(v, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(v))
        out[k] = t.to(device=device, dtype=dt).contiguous()
    if out["arrive"].dim() == 1:
        out["arrive"] = out["arrive"].unsqueeze(0)
        out["req"] = out["req"].unsqueeze(0)
        if "region" in out:
            out["region"] = out["region"].unsqueeze(0)
    return out


def run_batch(ctx: Context, trace: dict, out: BatchResult | None = None, ring_capacity: int = 0,
              stream=None, stage: str = "all", policy: str | int = "REF_V3", hist: bool = False,
              hier_threshold_s: int = 60, hier_up_tick: int = 20 * 10**9, ref_abort: bool = False) -> BatchResult:
    """Enqueue R trace replays (fognet_run_batch_dev) on the current stream.

    ``trace``: device tensors arrive/req [R, T], node params mips/dl/ul/init
    [R, N] (per replication) or [N] (shared), optional power model
    p_busy/p_idle (W, same shape as mips), optional node crash ticks ``down``
    (same shape as mips, NEVER = no crash; ComputeBrokerApp3::handleNodeCrash,
    ComputeBrokerApp3.cc:423-427: lost tasks get status 9).  ``stage``: "all", "replay"
    (fognet_replay_dev) or "stats" (fognet_rep_stats_dev).  ``policy``:
    "REF_V3" (BrokerBaseApp3), "EXT_LAT" (north-star cost) or "EXT_HIER"
    (hierarchical brokers with mobility handoff: needs ``trace["region"]``
    [R, T], see :func:`mobility_regions`; escalation above
    ``hier_threshold_s`` busy seconds, extra hop ``hier_up_tick``); the two
    extensions are not in the reference.  ``hist``: allocate the job
    histogram when ``out`` is None.  ``ref_abort`` (FOGNET_FLAG_REF_ABORT): a
    replication the reference run would end at a queueTime overflow gets status
    FOGNET_REF_ABORTED (its abort point, ``abort_tick``/``abort_task``, is in
    every record either way).
    """
    arrive, req = trace["arrive"], trace["req"]
    R, T = arrive.shape
    mips = trace["mips"]
    N = mips.shape[-1]
    stride = N if mips.dim() == 2 else 0
    pol = POLICIES[policy] if isinstance(policy, str) else int(policy)
    energy = trace.get("p_busy") is not None
    # host-side shape checks: the kernels index every array with these strides
    down = trace.get("down")
    for k in ("dl", "ul", "init") + (("p_busy", "p_idle") if energy else ()) + (("down",) if down is not None else ()):
        if tuple(trace[k].shape) != tuple(mips.shape):
            raise FognetError(_abi.FOGNET_ERR_ARG, f"{k} has shape {tuple(trace[k].shape)}, mips {tuple(mips.shape)}")
    if tuple(req.shape) != (R, T) or (mips.dim() == 2 and mips.shape[0] != R):
        raise FognetError(_abi.FOGNET_ERR_ARG, "trace arrays disagree on R/T")
    if out is not None and ((out.node is not None and tuple(out.node.shape) != (R, T))
                            or out.stats.numel() < R * _abi.REP_STATS_DTYPE.itemsize):
        raise FognetError(_abi.FOGNET_ERR_ARG, "output buffers too small for the trace")
    if out is None:
        out = allocate_outputs(R, T, arrive.device, N=N, energy=energy, hist=hist)
    region = trace.get("region")
    if pol == _abi.FOGNET_POLICY_EXT_HIER and (region is None or tuple(region.shape) != (R, T)):
        raise FognetError(_abi.FOGNET_ERR_ARG, "EXT_HIER needs trace['region'] of shape [R, T]")
    bi = _abi.BatchIn(R, T, N, pol, stride, ring_capacity,
                      _ptr(arrive), _ptr(req), _ptr(mips), _ptr(trace["dl"]), _ptr(trace["ul"]),
                      _ptr(trace["init"]), _ptr(trace.get("p_busy")), _ptr(trace.get("p_idle")), _ptr(down),
                      _ptr(region), int(hier_up_tick), int(hier_threshold_s),
                      _abi.FLAG_REF_ABORT if ref_abort else 0)
    bo = _abi.BatchOut(_ptr(out.node), _ptr(out.status), _ptr(out.start_tick), _ptr(out.done_tick),
                       _ptr(out.stats), _ptr(out.node_energy), _ptr(out.hist))
    s = C.c_void_p(stream.cuda_stream) if stream is not None else _stream_ptr(arrive.device)
    fn = {"all": ctx._lib.fognet_run_batch_dev, "replay": ctx._lib.fognet_replay_dev,
          "stats": ctx._lib.fognet_rep_stats_dev}[stage]
    ctx.check(fn(ctx.handle, C.byref(bi), C.byref(bo), s), f"run_batch[{stage}]")
    return out


def run_generated(ctx: Context, seed: int, R: int, T: int, N: int, mean_gap_ticks, lat_scale, r0: int = 0,
                  req_lo: int = 1000, req_hi: int = 64000, out: BatchResult | None = None, ring_capacity: int = 0,
                  policy: str | int = "REF_V3", power=None, hist: bool = True, energy: bool = False,
                  device=None, stream=None, hier_threshold_s: int = 60, hier_up_tick: int = 20 * 10**9) -> BatchResult:
    """Statistics-only replay of generated replications r0 .. r0+R-1
    (fognet_run_generated_dev): the trace recipe of
    :func:`generate_trace` is computed inside the replay kernel 64 publishes at
    a time, so neither the trace nor per-task outputs exist in memory.  The
    records equal ``generate_trace`` + ``run_batch`` on the same replications.
    ``power``: optional (p_busy, p_idle) device tensors [R, N] or [N].
    ``policy="EXT_HIER"``: each publish's regional broker is the one
    :func:`mobility_regions` (defaults) gives, computed in the kernel."""
    device = device if device is not None else torch.device("cuda", ctx.device)
    if isinstance(mean_gap_ticks, torch.Tensor):
        mg, ls = mean_gap_ticks.reshape(R).contiguous(), lat_scale.reshape(R).contiguous()
    else:
        mg = torch.as_tensor(np.asarray(mean_gap_ticks, dtype=np.float64).reshape(R), device=device)
        ls = torch.as_tensor(np.asarray(lat_scale, dtype=np.int64).reshape(R), device=device)
    pb, pi = power if power is not None else (None, None)
    stride = 0
    if pb is not None:
        if tuple(pb.shape) != tuple(pi.shape) or pb.shape[-1] != N or (pb.dim() == 2 and pb.shape[0] != R):
            raise FognetError(_abi.FOGNET_ERR_ARG, "power model arrays must be [R, N] or [N]")
        stride = N if pb.dim() == 2 else 0
    if out is None:
        out = allocate_outputs(R, T, device, N=N, energy=energy and pb is not None, hist=hist, per_task=False)
    elif out.stats.numel() < R * _abi.REP_STATS_DTYPE.itemsize:
        raise FognetError(_abi.FOGNET_ERR_ARG, "stats buffer too small")
    pol = POLICIES[policy] if isinstance(policy, str) else int(policy)
    gp = _abi.GenParams(seed & 0xFFFFFFFF, req_lo, req_hi, 0, _ptr(mg), _ptr(ls))
    hier = pol == _abi.FOGNET_POLICY_EXT_HIER
    bi = _abi.BatchIn(R, T, N, pol, stride, ring_capacity, None, None, None, None, None, None,
                      _ptr(pb), _ptr(pi), None, None, hier_up_tick if hier else 0, hier_threshold_s if hier else 0, 0)
    bo = _abi.BatchOut(None, None, None, None, _ptr(out.stats), _ptr(out.node_energy), _ptr(out.hist))
    s = C.c_void_p(stream.cuda_stream) if stream is not None else _stream_ptr(device)
    ctx.check(ctx._lib.fognet_run_generated_dev(ctx.handle, C.byref(gp), r0, C.byref(bi), C.byref(bo), s),
              "run_generated")
    out._keep = (mg, ls)
    return out


def user_stats(ctx: Context, trace: dict, out: BatchResult, user_ul, user_dl) -> np.ndarray:
    """User-side signals (fognet_user_stats_dev) of a finished replay: broker
    ``delay`` and mqttApp2's ``latency`` / ``latencyH1`` / ``taskTime`` as exact
    tick moments per replication (USER_STATS_DTYPE [R]).  ``user_ul`` /
    ``user_dl``: the publishing user's links, [R] (one user per replication)
    or [R, T] (per task), host arrays or device tensors."""
    arrive = trace["arrive"]
    R, T = arrive.shape
    dev = arrive.device
    uu = torch.as_tensor(np.asarray(user_ul) if not isinstance(user_ul, torch.Tensor) else user_ul,
                         dtype=torch.int64).to(dev).contiguous()
    ud = torch.as_tensor(np.asarray(user_dl) if not isinstance(user_dl, torch.Tensor) else user_dl,
                         dtype=torch.int64).to(dev).contiguous()
    per_task = 1 if uu.dim() == 2 else 0
    want = (R, T) if per_task else (R,)
    if tuple(uu.shape) != want or tuple(ud.shape) != want:
        raise FognetError(_abi.FOGNET_ERR_ARG, f"user links must both have shape [R] or [R, T], got "
                                               f"{tuple(uu.shape)} / {tuple(ud.shape)}")
    mips = trace["mips"]
    N = mips.shape[-1]
    res = torch.zeros(R * _abi.USER_STATS_DTYPE.itemsize, dtype=torch.uint8, device=dev)
    bi = _abi.BatchIn(R, T, N, _abi.FOGNET_POLICY_REF_V3, N if mips.dim() == 2 else 0, 0,
                      _ptr(arrive), _ptr(trace["req"]), _ptr(mips), _ptr(trace["dl"]), _ptr(trace["ul"]),
                      _ptr(trace["init"]), None, None)
    bo = _abi.BatchOut(_ptr(out.node), _ptr(out.status), _ptr(out.start_tick), _ptr(out.done_tick),
                       _ptr(out.stats), None, None)
    ctx.check(ctx._lib.fognet_user_stats_dev(ctx.handle, C.byref(bi), C.byref(bo), _ptr(uu), _ptr(ud), per_task,
                                             _ptr(res), _stream_ptr(dev)), "user_stats")
    return res.cpu().numpy().view(_abi.USER_STATS_DTYPE)


@dataclass
class V2Result:
    node: torch.Tensor        # [R, T] int32 (-1: served by the broker / no node)
    status: torch.Tensor      # [R, T] uint8 (_abi.V2_ST_*; 0: not published before the stop)
    start_tick: torch.Tensor  # [R, T] int64 reservation tick (-1: never reserved)
    done_tick: torch.Tensor   # [R, T] int64 release tick (-1: not released)
    stats: torch.Tensor       # [R * sizeof(fognet_v2_stats)] uint8

    def rep_stats(self) -> np.ndarray:
        return self.stats.cpu().numpy().view(_abi.V2_STATS_DTYPE)


def run_v2(ctx: Context, trace: dict, broker_mips, stop_tick, required_time_s=0.01, queue_capacity: int = 0,
           stream=None) -> V2Result:
    """R replays of the v2 model (BrokerBaseApp2 + ComputeBrokerApp2, the modules
    simulations/example/wirelessNet.ini:56,62 select) on the device
    (fognet_run_v2_dev).  ``trace``: device tensors arrive/req [R, T], node
    parameters mips/dl/ul and first_adv (first ADVERTISEMIPS firing) [R, N] or
    [N]; ``broker_mips``, ``stop_tick``, ``required_time_s``: scalars or [R]."""
    arrive, req = trace["arrive"], trace["req"]
    R, T = arrive.shape
    dev = arrive.device
    mips = trace["mips"]
    N = mips.shape[-1]
    for k in ("dl", "ul", "first_adv"):
        if tuple(trace[k].shape) != tuple(mips.shape):
            raise FognetError(_abi.FOGNET_ERR_ARG, f"{k} has shape {tuple(trace[k].shape)}, mips {tuple(mips.shape)}")
    per = lambda v, dt: torch.as_tensor(np.array(np.broadcast_to(np.asarray(v), (R,))), dtype=dt).to(dev)
    bm, st_, rt = per(broker_mips, torch.int32), per(stop_tick, torch.int64), per(required_time_s, torch.float64)
    out = V2Result(torch.empty((R, T), dtype=torch.int32, device=dev), torch.empty((R, T), dtype=torch.uint8, device=dev),
                   torch.empty((R, T), dtype=torch.int64, device=dev), torch.empty((R, T), dtype=torch.int64, device=dev),
                   torch.zeros(R * _abi.V2_STATS_DTYPE.itemsize, dtype=torch.uint8, device=dev))
    vi = _abi.V2In(R, T, N, N if mips.dim() == 2 else 0, queue_capacity, 0, _ptr(arrive), _ptr(req), _ptr(bm), _ptr(rt),
                   _ptr(st_), _ptr(mips), _ptr(trace["dl"]), _ptr(trace["ul"]), _ptr(trace["first_adv"]))
    vo = _abi.V2Out(_ptr(out.node), _ptr(out.status), _ptr(out.start_tick), _ptr(out.done_tick), _ptr(out.stats))
    s = C.c_void_p(stream.cuda_stream) if stream is not None else _stream_ptr(dev)
    ctx.check(ctx._lib.fognet_run_v2_dev(ctx.handle, C.byref(vi), C.byref(vo), s), "run_v2")
    out._keep = (bm, st_, rt)
    return out


def _signed(v: int, bits: int) -> int:
    return v - (1 << bits) if v >> (bits - 1) else v


def _fields(n, s, q, lo, hi, unit) -> dict:
    """cStdDev's `.sca` fields (count/mean/stddev/sum/sqrsum/min/max) of n values
    with exact sum s and sum of squares q, in units of ``unit`` ms."""
    if n == 0:
        return dict(count=0)
    var = (q - s * s / n) / (n - 1) if n > 1 else 0.0
    return dict(count=n, mean=s / n * unit, stddev=max(var, 0.0) ** 0.5 * unit, sum=s * unit, sqrsum=q * unit * unit,
                min=int(lo) * unit, max=int(hi) * unit)


def summarize_moments(m, raw_ms: bool = True) -> dict:
    """count/mean/stddev/sum/sqrsum/min/max of one signal-moments record
    (fognet_moments) like cStdDev's `.sca` fields.  ``raw_ms``: the values are
    raw emitted simtime_t of a ms signal (recorded value raw * 1e-12 ms); False
    for ``delay`` (raw ticks, reported in ms)."""
    n = int(m["count"])
    s = _signed(int(m["sum_lo"]) | (int(m["sum_hi"]) << 64), 128)
    q = int(m["sq_lo"]) | (int(m["sq_hi"]) << 64) | (int(m["sq_top"]) << 128)
    d = _fields(n, s, q, m["min_raw"], m["max_raw"], 1e-12 if raw_ms else 1e-9)
    d["overflow"] = int(m["overflow"])
    return d


def reduce_stats(ctx: Context, stats: torch.Tensor, R: int) -> np.ndarray:
    """Exact job-level reduction on the device; returns a JOB_STATS_DTYPE record."""
    out = torch.zeros(_abi.JOB_STATS_DTYPE.itemsize, dtype=torch.uint8, device=stats.device)
    ctx.check(ctx._lib.fognet_reduce_stats_dev(ctx.handle, _ptr(stats), R, _ptr(out), _stream_ptr(stats.device)),
              "reduce_stats")
    return out.cpu().numpy().view(_abi.JOB_STATS_DTYPE)[0]


def merge_job_stats(records) -> np.ndarray:
    """Exact host merge of job records (e.g. one per GPU after an all-gather)."""
    lib = _abi.load()
    acc = _abi.JobStats()
    lib.fognet_job_stats_init(C.byref(acc))
    for rec in records:
        b = _abi.JobStats.from_buffer_copy(np.ascontiguousarray(rec).tobytes())
        lib.fognet_job_stats_merge(C.byref(acc), C.byref(b))
    return np.frombuffer(bytes(acc), dtype=_abi.JOB_STATS_DTYPE)[0]


def job_from_reps(reps) -> np.ndarray:
    """Exact host reduction of per-replication records (REP_STATS_DTYPE) into a
    job record (fognet_job_stats_add_rep, the host twin of fognet_reduce_stats_dev)."""
    lib = _abi.load()
    acc = _abi.JobStats()
    lib.fognet_job_stats_init(C.byref(acc))
    for rec in np.atleast_1d(reps):
        b = _abi.RepStats.from_buffer_copy(np.ascontiguousarray(rec).tobytes())
        lib.fognet_job_stats_add_rep(C.byref(acc), C.byref(b))
    return np.frombuffer(bytes(acc), dtype=_abi.JOB_STATS_DTYPE)[0]


def _u192(limbs) -> int:
    return int(limbs[0]) | (int(limbs[1]) << 64) | (int(limbs[2]) << 128)


def summarize(job) -> dict:
    """`.sca`-style fields (count/mean/stddev/sum/sqrsum/min/max, ms) of a job record:
    queueTime as the reference records it (ComputeBrokerApp3.cc:238,
    ComputeBrokerApp3.ned:45-46; raw values * 1e-12), response in ticks / 1e9."""
    qs = _signed(_u192(job["queue_sum"]), 192)
    queue = _fields(int(job["n_qtime"]), qs, _u192(job["queue_sq"]), job["queue_min_raw"], job["queue_max_raw"], 1e-12)
    queue["overflow"] = int(job["n_qtime_overflow"])
    return {
        "replications": int(job["n_reps"]), "failed": int(job["n_failed"]),
        "decisions": int(job["n_tasks"]), "queued": int(job["n_queued"]), "started": int(job["n_started"]),
        "queueTime_ms": queue,
        "response_ms": _fields(int(job["n_tasks"]), _u192(job["resp_sum"]), _u192(job["resp_sq"]),
                               job["resp_min_ticks"], job["resp_max_ticks"], 1e-9),
        "max_pending": int(job["max_pending"]),
        "busy_s": int(job["busy_s"]),
        "energy_j": float(job["energy_j"]),
        # replications the reference run would have ended at a queueTime overflow (fognet_hip.h)
        "ref_aborted": int(job["n_ref_aborted"]),
    }


def allocate_trace(R: int, T: int, N: int, device) -> dict:
    """Device buffers of one trace batch (arrive/req [R, T], node params [R, N])."""
    return {
        "arrive": torch.empty((R, T), dtype=torch.int64, device=device),
        "req": torch.empty((R, T), dtype=torch.int32, device=device),
        "mips": torch.empty((R, N), dtype=torch.int32, device=device),
        "dl": torch.empty((R, N), dtype=torch.int64, device=device),
        "ul": torch.empty((R, N), dtype=torch.int64, device=device),
        "init": torch.empty((R, N), dtype=torch.int64, device=device),
    }


def generate_trace(ctx: Context, seed: int, R: int, T: int, N: int, mean_gap_ticks, lat_scale,
                   r0: int = 0, req_lo: int = 1000, req_hi: int = 64000, device=None, out: dict | None = None) -> dict:
    """Device trace generator (recipe: csrc/tracegen.hip); per-replication
    ``mean_gap_ticks`` (float64 [R]) and ``lat_scale`` (int64 [R]), host arrays
    or device tensors.  ``out``: reuse these buffers (allocate_trace layout)."""
    device = device if device is not None else torch.device("cuda", ctx.device)
    if isinstance(mean_gap_ticks, torch.Tensor):
        mg, ls = mean_gap_ticks.reshape(R).contiguous(), lat_scale.reshape(R).contiguous()
    else:
        mg = torch.as_tensor(np.asarray(mean_gap_ticks, dtype=np.float64).reshape(R), device=device)
        ls = torch.as_tensor(np.asarray(lat_scale, dtype=np.int64).reshape(R), device=device)
    tr = out if out is not None else allocate_trace(R, T, N, device)
    gp = _abi.GenParams(seed & 0xFFFFFFFF, req_lo, req_hi, 0, _ptr(mg), _ptr(ls))
    rc = ctx._lib.fognet_gen_trace_dev(ctx.handle, C.byref(gp), r0, R, T, N, _ptr(tr["arrive"]), _ptr(tr["req"]),
                                       _ptr(tr["mips"]), _ptr(tr["dl"]), _ptr(tr["ul"]), _ptr(tr["init"]),
                                       _stream_ptr(device))
    ctx.check(rc, "gen_trace")
    tr["_keep"] = (mg, ls)
    return tr


def sweep_params(r_global: np.ndarray, N: int, rho=None, lat_scale=None, req_lo=1000, req_hi=64000):
    """Per-replication (mean_gap_ticks, lat_scale) for the C3 policy sweep:
    rho = (0.5, 0.8, 0.95)[r % 3], latency x(1, 10, 100)[(r // 3) % 3]
    unless fixed values are given.  mips pattern 1000*(1 + j % 4)."""
    r_global = np.asarray(r_global, dtype=np.int64)
    mips = 1000.0 * (1 + (np.arange(N) % 4))
    es = 0.5 * (req_lo + req_hi) * float(np.mean(1.0 / mips))
    rho_r = np.full(r_global.shape, rho, np.float64) if rho is not None else np.array((0.5, 0.8, 0.95))[r_global % 3]
    sc = (np.full(r_global.shape, lat_scale, np.int64) if lat_scale is not None
          else np.array((1, 10, 100), np.int64)[(r_global // 3) % 3])
    mean_gap = es / (N * rho_r) * _abi.TICKS_PER_SECOND
    return mean_gap, sc


def c5_params(r_global: np.ndarray, N: int, req_lo=1000, req_hi=64000):
    """Per-replication (mean_gap_ticks, lat_scale) of the C5 large-topology
    recipe (builder-defined: the reference has no C5 parameters):
    rho = (0.002, 0.01, 0.05)[r % 3], latency x(1, 10, 100)[(r // 3) % 3].
    Light loads: under REF_V3 the C3 loads herd all of T onto node 0 when N is
    in the thousands (the stale view keeps every node at busy 0 until its first
    completion advert), so C5 uses loads at which decisions spread over nodes."""
    r_global = np.asarray(r_global, dtype=np.int64)
    mg, sc = sweep_params(r_global, N, req_lo=req_lo, req_hi=req_hi)
    rho = np.array((0.002, 0.01, 0.05))[r_global % 3]
    mips = 1000.0 * (1 + (np.arange(N) % 4))
    es = 0.5 * (req_lo + req_hi) * float(np.mean(1.0 / mips))
    return es / (N * rho) * _abi.TICKS_PER_SECOND, sc


def mobility_regions(arrive, N: int, users: int = 256, period_s=(30, 45, 60, 75)):
    """Regional broker of every publish under a builder-defined mobility model
    (FOGNET_POLICY_EXT_HIER; not in the reference, whose only mobility is the
    users' radio mobility, simulations/example/wirelessNet.ini:13-29): publish i
    of a replication comes from user u = i mod ``users``; user u starts in
    region u mod B (B = ceil(N / 1024) regions of 1024 consecutive nodes) and
    hands off to the next region (+1 for even u, -1 for odd u, mod B) every
    period_s[u mod 4] seconds from the replication's first publish.  Integer
    arithmetic only, so numpy (host) and torch (device) give the same regions.
    ``arrive``: [R, T] int64 ticks (numpy array or tensor); returns int32 [R, T]."""
    B = -(-N // _abi.HIER_REGION_NODES)
    torch_in = isinstance(arrive, torch.Tensor)
    xp = torch if torch_in else np
    R, T = arrive.shape
    i = xp.arange(T, device=arrive.device) if torch_in else np.arange(T)
    u = (i % users).to(torch.int64) if torch_in else (i % users).astype(np.int64)
    per = [p * _abi.TICKS_PER_SECOND for p in period_s]
    period = (torch.tensor(per, device=arrive.device, dtype=torch.int64) if torch_in else np.array(per, np.int64))[u % 4]
    sign = 1 - 2 * (u % 2)
    t0 = arrive[:, :1]
    hops = (arrive - t0) // period
    reg = (u % B) + sign * hops
    reg = reg % B  # floor modulo in both numpy and torch
    return reg.to(torch.int32) if torch_in else reg.astype(np.int32)


def _saturation_template(arrive0: np.ndarray, region: np.ndarray, sizes: list[int], lat_max: int):
    """Roles of the publishes of one region sequence (saturating_trace): per
    region, walk its publishes; a free publish p starts a pair on the region's
    next fresh node (small task of S1 seconds, the region's next publish q a
    giant task), S1 the smallest whole second above q's gap, so q reaches the
    node before p completes; every publish up to p's completion advert (S1 + the
    link latencies, bounded by ``lat_max``) is a zero-service filler.  Once every
    node of the region has its pair, the publishes are zero-service tasks, which
    the saturated regional broker escalates.
    Returns role [T] (0 filler / escalation, 1 small, 2 giant), the pair's node
    offset within its region [T] (-1 for fillers) and S1 [T]."""
    T = arrive0.shape[0]
    role = np.zeros(T, np.int8)
    node = np.full(T, -1, np.int64)
    s1 = np.zeros(T, np.int64)
    tps = TICKS_PER_SECOND_I
    for b, size in enumerate(sizes):
        idx = np.flatnonzero(region == b)
        m = 0
        i = 0
        while i + 1 < len(idx) and m < size:
            p, q = idx[i], idx[i + 1]
            S1 = (int(arrive0[q]) - int(arrive0[p])) // tps + 1
            role[p], role[q] = 1, 2
            node[p] = node[q] = m
            s1[p] = S1
            adv = int(arrive0[p]) + S1 * tps + lat_max  # the advert has reached the broker by then
            i += 2
            while i < len(idx) and int(arrive0[idx[i]]) <= adv:
                i += 1
            m += 1
    return role, node, s1


TICKS_PER_SECOND_I = 10**12


def saturating_trace(seed: int, R: int, T: int, N: int, gap_s: float = 0.1, giant_s=(4000, 6000),
                     users: int = 256, lat_ticks=(10**9, 10**10), escalate=None, r0: int = 0) -> dict:
    """Builder-defined overload recipe for EXT_HIER at the C5 topology, host
    numpy (the reference has no hierarchy; DESIGN.md §3.8 "Escalations at
    N = 10,000").  Under the reference's stale view a regional broker herds its
    publishes onto its lowest-index node until that node's first completion
    advert arrives (BrokerBaseApp3.cc:123-130, 265-281), and it escalates only
    when every node of its region advertises more than the threshold, so an
    i.i.d. trace needs ~1024^2 publishes per region to saturate one.  This trace
    saturates every region within ~3 publishes per node: each node gets one
    pair -- a short task, then a giant one (giant_s seconds, more than the whole
    filling phase) that reaches it before the short one completes, so its first
    advert carries the giant's backlog -- and zero-service fillers until that
    advert lands; afterwards every publish is a zero-service task escalated to
    the parent's global argmin (the smallest advertised giant).  Publishes every
    ``gap_s`` seconds (plus jitter), regions from :func:`mobility_regions`
    (``users`` users), per-node link latencies in ``lat_ticks``, MIPS
    1000 * (1 + j % 4).  The publish ticks and regions are shared by all
    replications; global replication r0 + i gets its own giants and latencies
    (Philox-free numpy streams keyed by (seed, r0 + i), so a shard equals the
    same rows of the whole job), and its smallest giant sits in region
    3 + (r0 + i) % 7 (B = 10), so escalations land in the wide kernel's upper
    rows.  ``escalate`` ([R] bools, default all): a replication given False
    gets 30-s tasks instead of giants, so its nodes advertise at most 30 s
    (below the bench's 60-s threshold) and no region escalates (the region pass
    finishes it).  Returns host arrays (make_batch layout) + ``region`` [R, T]."""
    tps = TICKS_PER_SECOND_I
    B = -(-N // _abi.HIER_REGION_NODES)
    sizes = [min(_abi.HIER_REGION_NODES, N - b * _abi.HIER_REGION_NODES) for b in range(B)]
    lo, hi = lat_ticks
    shared = np.random.default_rng([seed & 0xFFFFFFFF, T, N])
    g = int(gap_s * tps)
    base = 2 * hi  # after every first advert (init = ul < hi)
    arrive0 = base + np.arange(T, dtype=np.int64) * g + shared.integers(0, g // 2, size=T, dtype=np.int64)
    region0 = mobility_regions(arrive0[None, :], N, users=users)[0]
    role, off, s1 = _saturation_template(arrive0, region0, sizes, 2 * hi)
    k = np.where(off >= 0, region0.astype(np.int64) * _abi.HIER_REGION_NODES + off, 0)
    mips1 = (1000 * (1 + np.arange(N) % 4)).astype(np.int32)
    mk = mips1[k].astype(np.int64)  # [T]: the MIPS of the pair's node
    esc = np.ones(R, bool) if escalate is None else np.asarray(escalate, bool)
    dl = np.empty((R, N), np.int64)
    ul = np.empty((R, N), np.int64)
    req = np.empty((R, T), np.int32)
    for i in range(R):
        rng = np.random.default_rng([seed & 0xFFFFFFFF, r0 + i])
        dl[i] = rng.integers(lo, hi, size=N, dtype=np.int64)
        ul[i] = rng.integers(lo, hi, size=N, dtype=np.int64)
        giant = rng.integers(giant_s[0] + 1, giant_s[1], size=N, dtype=np.int64)
        b = (3 + (r0 + i) % 7) % B  # the smallest giant of this replication
        giant[b * _abi.HIER_REGION_NODES + int(rng.integers(0, sizes[b]))] = giant_s[0]
        if not esc[i]:
            giant[:] = 30
        zero = rng.integers(0, 1000, size=T, dtype=np.int64)  # below every MIPS: zero service
        req[i] = np.where(role == 1, s1 * mk, np.where(role == 2, giant[k] * mk, zero))
    return dict(arrive=np.broadcast_to(arrive0, (R, T)).copy(), req=req, mips=np.broadcast_to(mips1, (R, N)).copy(),
                dl=dl, ul=ul, init=ul.copy(), region=np.broadcast_to(region0, (R, T)).copy())


def power_model(mips) -> tuple[np.ndarray, np.ndarray]:
    """Synthetic node power model for the a11 energy statistic (builder-defined;
    the reference has no fog-node energy model): busy power
    grows with MIPS, idle power is 35% of it.  Same shape as ``mips``."""
    m = np.asarray(mips, dtype=np.float64)
    p_busy = 20.125 + 0.02 * m
    return p_busy, 0.35 * p_busy
