"""Host-side formats on either side of the decision path (include/fognet_io.h).

* :func:`save_trace` / :func:`load_trace` — binary SoA trace files
  ("FOGNTRC1"): node parameters in CONNECT order + the broker-side publish
  trace, the exact inputs of :func:`fognetsimpp_amd.run_batch`.
* :func:`write_sca` / :func:`write_vec` — OMNeT++ 4.6 result files in the
  layout of simulations/example/results/General-0.sca / General-0.vec.
* :func:`gen_trace_mqtt` — the reference task source (mqttApp2.cc:198-409):
  one glibc rand() stream shared by all users in FES order,
  MIPSRequired = 200 + rand() % 701.

All of it is host C++ in libfognet_hip (no GPU, no context).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import FognetError

_NODE_KEYS = (("mips", np.int32), ("dl", np.int64), ("ul", np.int64), ("init", np.int64))


def _p(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def _check(rc: int, what: str):
    if rc != _abi.FOGNET_OK:
        raise FognetError(rc, f"{what}: {_abi.load().fognet_io_last_error().decode()}")


def trace_info(path: str) -> dict:
    info = _abi.TraceInfo()
    _check(_abi.load().fognet_trace_info_read(path.encode(), C.byref(info)), "trace_info")
    return dict(R=info.R, T=info.T, N=info.N, node_stride=info.node_stride, flags=info.flags,
                version=info.version, payload_bytes=info.payload_bytes, checksum=info.checksum,
                note=info.note.decode())


def save_trace(path: str, trace: dict, node_id=None, note: str = "") -> None:
    """Write a trace dict (arrive/req [R, T] or [T]; mips/dl/ul/init [R, N] or
    [N] shared; optional p_busy/p_idle like mips) to ``path``."""
    arrive = np.ascontiguousarray(np.atleast_2d(np.asarray(trace["arrive"])), dtype=np.int64)
    req = np.ascontiguousarray(np.atleast_2d(np.asarray(trace["req"])), dtype=np.int32)
    R, T = arrive.shape
    if req.shape != (R, T):
        raise FognetError(_abi.FOGNET_ERR_ARG, "arrive/req shapes differ")
    nodes = {k: np.ascontiguousarray(trace[k], dtype=dt) for k, dt in _NODE_KEYS}
    shared = nodes["mips"].ndim == 1
    N = nodes["mips"].shape[-1]
    for k, a in nodes.items():
        if a.shape != nodes["mips"].shape or (not shared and a.shape[0] != R):
            raise FognetError(_abi.FOGNET_ERR_ARG, f"{k} has shape {a.shape}")
    pb = pi = None
    if trace.get("p_busy") is not None:
        pb = np.ascontiguousarray(trace["p_busy"], dtype=np.float64)
        pi = np.ascontiguousarray(trace["p_idle"], dtype=np.float64)
    nid = np.ascontiguousarray(node_id, dtype=np.int32) if node_id is not None else None
    bi = _abi.BatchIn(R, T, N, _abi.FOGNET_POLICY_REF_V3, 0 if shared else N, 0,
                      _p(arrive), _p(req), _p(nodes["mips"]), _p(nodes["dl"]), _p(nodes["ul"]), _p(nodes["init"]),
                      _p(pb), _p(pi))
    _check(_abi.load().fognet_trace_write(path.encode(), C.byref(bi), _p(nid), note.encode()), "save_trace")


def load_trace(path: str) -> dict:
    """Read a trace file into numpy arrays (the save_trace layout; node arrays
    are [N] when the file stores them shared).  Verifies the checksum."""
    info = trace_info(path)
    R, T, N, stride = info["R"], info["T"], info["N"], info["node_stride"]
    nshape = (R, N) if stride else (N,)
    out = {"arrive": np.empty((R, T), np.int64), "req": np.empty((R, T), np.int32)}
    for k, dt in _NODE_KEYS:
        out[k] = np.empty(nshape, dt)
    pw = bool(info["flags"] & _abi.TRACE_FLAG_POWER)
    if pw:
        out["p_busy"] = np.empty(nshape, np.float64)
        out["p_idle"] = np.empty(nshape, np.float64)
    nid = np.empty(nshape, np.int32) if info["flags"] & _abi.TRACE_FLAG_NODE_ID else None
    bi = _abi.BatchIn(0, 0, 0, 0, 0, 0, _p(out["arrive"]), _p(out["req"]), _p(out["mips"]), _p(out["dl"]),
                      _p(out["ul"]), _p(out["init"]), _p(out.get("p_busy")), _p(out.get("p_idle")))
    _check(_abi.load().fognet_trace_read(path.encode(), C.byref(bi), _p(nid)), "load_trace")
    if nid is not None:
        out["node_id"] = nid
    out["note"] = info["note"]
    return out


def write_sca(path: str, job, hist=None, run_id: str = "General-0-fognet", network: str = "FogNet") -> None:
    """OMNeT++ .sca of a job record (JOB_STATS_DTYPE) and optional histogram [2, 64]."""
    js = _abi.JobStats.from_buffer_copy(np.ascontiguousarray(job).tobytes())
    h = np.ascontiguousarray(hist, dtype=np.int64) if hist is not None else None
    if h is not None and h.shape != (_abi.HIST_METRICS, _abi.HIST_BINS):
        raise FognetError(_abi.FOGNET_ERR_ARG, f"hist shape {h.shape}")
    _check(_abi.load().fognet_write_sca(path.encode(), run_id.encode(), network.encode(), C.byref(js), _p(h)),
           "write_sca")


def write_vec(path: str, arrive, dl, node, status, start, node_id=None, run_id: str = "General-0-fognet",
              network: str = "FogNet") -> None:
    """OMNeT++ .vec of ONE replication: arrive/node/status/start [T], dl [N]."""
    a = np.ascontiguousarray(arrive, dtype=np.int64).reshape(-1)
    d = np.ascontiguousarray(dl, dtype=np.int64).reshape(-1)
    n = np.ascontiguousarray(node, dtype=np.int32).reshape(-1)
    s = np.ascontiguousarray(status, dtype=np.uint8).reshape(-1)
    st = np.ascontiguousarray(start, dtype=np.int64).reshape(-1)
    nid = np.ascontiguousarray(node_id, dtype=np.int32).reshape(-1) if node_id is not None else None
    T, N = a.size, d.size
    if not (n.size == s.size == st.size == T) or (nid is not None and nid.size != N):
        raise FognetError(_abi.FOGNET_ERR_ARG, "write_vec: array lengths differ")
    _check(_abi.load().fognet_write_vec(path.encode(), run_id.encode(), network.encode(), T, N, _p(a), _p(d), _p(n),
                                        _p(s), _p(st), _p(nid)), "write_vec")


def gen_trace_mqtt(seed: int, start, interval, uplink, downlink, stop: int, req_base: int = 200, req_span: int = 701,
                   cap: int | None = None) -> dict:
    """Reference task source (fognet_gen_trace_mqtt): per-user tick arrays
    start/interval/uplink/downlink (downlink < 0: no CONNACK); returns
    arrive [T] (broker arrival ticks), req [T], user [T]."""
    st, iv, up, dn = (np.ascontiguousarray(x, dtype=np.int64).reshape(-1) for x in (start, interval, uplink, downlink))
    U = st.size
    if not (iv.size == up.size == dn.size == U):
        raise FognetError(_abi.FOGNET_ERR_ARG, "per-user arrays differ in length")
    if U and (iv.min() <= 0 or st.min() < 0 or up.min() < 0):
        raise FognetError(_abi.FOGNET_ERR_ARG, "need start >= 0, interval > 0, uplink >= 0")
    if cap is None:  # upper bound: CONNACK + every timer before stop
        span = np.maximum(stop - st, 0)
        cap = int((span // iv + 2).sum()) if U else 0
    arrive = np.empty(cap, np.int64)
    req = np.empty(cap, np.int32)
    user = np.empty(cap, np.int32)
    t = C.c_int32(0)
    _check(_abi.load().fognet_gen_trace_mqtt(seed & 0xFFFFFFFF, U, _p(st), _p(iv), _p(up), _p(dn), int(stop), req_base,
                                             req_span, cap, _p(arrive), _p(req), _p(user), C.byref(t)),
           "gen_trace_mqtt")
    n = t.value
    return dict(arrive=arrive[:n], req=req[:n], user=user[:n])
