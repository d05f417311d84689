"""ctypes loader for the CPU restatement in oracle/ (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg use this.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "build", "liboracle.so")


class OrcRepStats(C.Structure):
    _fields_ = [
        ("n_tasks", C.c_int64), ("n_queued", C.c_int64), ("n_started", C.c_int64),
        ("last_tick", C.c_int64),
        ("queue_min_raw", C.c_int64), ("queue_max_raw", C.c_int64),
        ("resp_min_ticks", C.c_int64), ("resp_max_ticks", C.c_int64),
        ("queue_sum_lo", C.c_uint64), ("queue_sum_hi", C.c_uint64),
        ("queue_sq_lo", C.c_uint64), ("queue_sq_hi", C.c_uint64),
        ("resp_sum_lo", C.c_uint64), ("resp_sum_hi", C.c_uint64),
        ("resp_sq_lo", C.c_uint64), ("resp_sq_hi", C.c_uint64),
        ("events", C.c_int64), ("max_pending", C.c_int32), ("status", C.c_int32),
        ("busy_s", C.c_int64), ("energy_j", C.c_double),
        ("queue_sq_top", C.c_uint64), ("n_qtime", C.c_int64), ("n_qtime_overflow", C.c_int64),
        ("abort_tick", C.c_int64), ("abort_task", C.c_int64),
    ]


_NP = {C.c_int64: np.int64, C.c_uint64: np.uint64, C.c_int32: np.int32, C.c_double: np.float64}
ORC_STATS_DTYPE = np.dtype([(n, _NP[t]) for n, t in OrcRepStats._fields_])
assert ORC_STATS_DTYPE.itemsize == C.sizeof(OrcRepStats)
MOMENTS_DTYPE = np.dtype([("count", np.int64), ("min_raw", np.int64), ("max_raw", np.int64),
                          ("sum_lo", np.uint64), ("sum_hi", np.uint64), ("sq_lo", np.uint64), ("sq_hi", np.uint64),
                          ("sq_top", np.uint64), ("overflow", np.int64)])
USER_SIGNALS = ("delay", "latency", "latencyH1", "taskTime")
USER_STATS_DTYPE = np.dtype([(n, MOMENTS_DTYPE) for n in USER_SIGNALS])
POLICY_REF_V3, POLICY_EXT_LAT, POLICY_EXT_HIER = 1, 16, 32
POLICIES = {"REF_V3": POLICY_REF_V3, "EXT_LAT": POLICY_EXT_LAT, "EXT_HIER": POLICY_EXT_HIER}

_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = C.CDLL(LIB)
        p = C.c_void_p
        _lib.orc_run_batch.argtypes = [C.c_int32, C.c_int64, C.c_int32, C.c_int32] + [p] * 11 + [C.c_int]
        _lib.orc_run_batch.restype = C.c_int
        _lib.orc_run_batch2.argtypes = [C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_int32] + [p] * 15 + [C.c_int]
        _lib.orc_run_batch2.restype = C.c_int
        _lib.orc_run_batch3.argtypes = ([C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_int32] + [p] * 10 +
                                        [C.c_int32] + [p] * 8 + [C.c_int])
        _lib.orc_run_batch3.restype = C.c_int
        _lib.orc_run_batch4.argtypes = ([C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_int32] + [p] * 10 +
                                        [C.c_int32] + [p] * 9 + [C.c_int])
        _lib.orc_run_batch4.restype = C.c_int
        _lib.orc_run_batch5.argtypes = ([C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_int32] + [p] * 10 +
                                        [C.c_int32, p, p, C.c_int32, C.c_int64] + [p] * 8 + [C.c_int])
        _lib.orc_run_batch5.restype = C.c_int
        _lib.orc_run_batch6.argtypes = ([C.c_int32, C.c_int64, C.c_int32, C.c_int32, C.c_int32] + [p] * 10 +
                                        [C.c_int32, p, p, C.c_int32, C.c_int64, C.c_int32] + [p] * 8 + [C.c_int])
        _lib.orc_run_batch6.restype = C.c_int
        _lib.orc_decide_hier.argtypes = [C.c_int32, p, p, C.c_int32, C.c_int32, C.c_int32, C.POINTER(C.c_int32),
                                         C.POINTER(C.c_int32)]
        _lib.orc_decide_hier.restype = C.c_int
        _lib.orc_decide_ext_lat.argtypes = [C.c_int32, p, p, p, C.c_int32, C.POINTER(C.c_int32)]
        _lib.orc_decide_ext_lat.restype = C.c_int
        _lib.orc_hist_bin.argtypes = [C.c_int64]
        _lib.orc_hist_bin.restype = C.c_int
        _lib.orc_hist_bin_raw.argtypes = [C.c_int64]
        _lib.orc_hist_bin_raw.restype = C.c_int
        _lib.orc_qtime_raw.argtypes = [C.c_int64, C.c_int64, C.POINTER(C.c_int64)]
        _lib.orc_qtime_raw.restype = C.c_int
        _lib.orc_ms_raw.argtypes = [C.c_int64, C.POINTER(C.c_int64)]
        _lib.orc_ms_raw.restype = C.c_int
        _lib.orc_decide_v3.argtypes = [C.c_int32, p, p, C.c_int32, C.POINTER(C.c_int32)]
        _lib.orc_decide_v3.restype = C.c_int
        _lib.orc_decide_v2.argtypes = [C.c_int32, p, C.c_int32, C.c_int32, C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        _lib.orc_decide_v2.restype = C.c_int
        _lib.orc_run_v2_batch.argtypes = [p, C.c_int]
        _lib.orc_run_v2_batch.restype = C.c_int
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def qtime_raw(now: int, qstart: int):
    """Raw simtime_t the node emits as queueTime (ComputeBrokerApp3.cc:238), or None
    where the reference's simtime_t arithmetic throws (orc_qtime_raw)."""
    out = C.c_int64(0)
    return out.value if lib().orc_qtime_raw(int(now), int(qstart), C.byref(out)) else None


def ms_raw(diff_ticks: int):
    out = C.c_int64(0)
    return out.value if lib().orc_ms_raw(int(diff_ticks), C.byref(out)) else None


def decide_v3(adv_busy, adv_mips, req):
    adv_busy = np.ascontiguousarray(adv_busy, dtype=np.float64)
    adv_mips = np.ascontiguousarray(adv_mips, dtype=np.int32)
    out = C.c_int32(-7)
    rc = lib().orc_decide_v3(len(adv_busy), _ptr(adv_busy), _ptr(adv_mips), int(req), C.byref(out))
    return rc, out.value


def decide_v2(adv_mips, local_mips, req):
    """BrokerBaseApp2 decision: (action ORC_V2_*, node)."""
    adv_mips = np.ascontiguousarray(adv_mips, dtype=np.int32)
    node, act = C.c_int32(-7), C.c_int32(-7)
    lib().orc_decide_v2(len(adv_mips), _ptr(adv_mips) if len(adv_mips) else None, int(local_mips), int(req),
                        C.byref(node), C.byref(act))
    return act.value, node.value


V2_LOCAL, V2_FORWARD, V2_DROPPED, V2_NO_NODES = 3, 4, 5, 6


def decide_ext_lat(adv_busy, mips, dl, req):
    adv_busy = np.ascontiguousarray(adv_busy, dtype=np.float64)
    mips = np.ascontiguousarray(mips, dtype=np.int32)
    dl = np.ascontiguousarray(dl, dtype=np.int64)
    out = C.c_int32(-7)
    rc = lib().orc_decide_ext_lat(len(adv_busy), _ptr(adv_busy), _ptr(mips), _ptr(dl), int(req), C.byref(out))
    return rc, out.value


def decide_hier(adv_busy, adv_mips, region, threshold_s, req):
    """EXT_HIER decision: (rc, node, escalated)."""
    adv_busy = np.ascontiguousarray(adv_busy, dtype=np.float64)
    adv_mips = np.ascontiguousarray(adv_mips, dtype=np.int32)
    k, esc = C.c_int32(-7), C.c_int32(-7)
    rc = lib().orc_decide_hier(len(adv_busy), _ptr(adv_busy), _ptr(adv_mips), int(region), int(threshold_s), int(req),
                               C.byref(k), C.byref(esc))
    return rc, k.value, esc.value


def run_batch(arrive, req, mips, dl, ul, init, threads: int = 1, outputs: bool = True, policy: int = 1,
              p_busy=None, p_idle=None, hist: bool = False, user_ul=None, user_dl=None, down=None, region=None,
              hier_threshold_s: int = 60, hier_up_tick: int = 20 * 10**9, stop_at_ref_abort: bool = False):
    """Replay R replications.  arrive/req: [R,T]; node params [R,N] or [N] (shared).
    ``p_busy``/``p_idle`` (same shape as mips) enable the energy model; ``hist``
    returns per-replication histograms [R, 2, 64]; ``user_ul``/``user_dl``
    ([R] one user per replication, or [R, T] per task) model the publishing
    users' links and return the user-side signals as ``user`` [R] (USER_STATS_DTYPE).
    ``down`` (same shape as mips, INT64_MAX = never): node crash ticks.
    ``region`` ([R, T] int32): the EXT_HIER regional broker of each publish.
    ``stop_at_ref_abort``: end each replication where the reference ends it, at
    the first queueTime emission that overflows (orc_rep_in.stop_at_ref_abort);
    outputs the run never reached stay -1 (status 0)."""
    arrive = np.ascontiguousarray(np.atleast_2d(arrive), dtype=np.int64)
    req = np.ascontiguousarray(np.atleast_2d(req), dtype=np.int32)
    R, T = arrive.shape
    mips = np.ascontiguousarray(mips, dtype=np.int32)
    dl = np.ascontiguousarray(dl, dtype=np.int64)
    ul = np.ascontiguousarray(ul, dtype=np.int64)
    init = np.ascontiguousarray(init, dtype=np.int64)
    N = mips.shape[-1]
    stride = N if mips.ndim == 2 else 0
    node = np.empty((R, T), np.int32) if outputs else None
    status = np.zeros((R, T), np.uint8) if outputs else None
    start = np.zeros((R, T), np.int64) if outputs else None
    done = np.zeros((R, T), np.int64) if outputs else None
    pb = np.ascontiguousarray(p_busy, dtype=np.float64) if p_busy is not None else None
    pi = np.ascontiguousarray(p_idle, dtype=np.float64) if p_idle is not None else None
    energy = np.zeros((R, N), np.float64) if pb is not None else None
    h = np.zeros((R, 2, 64), np.int64) if hist else None
    uu = ud = user = None
    per_task = 0
    if user_ul is not None:
        uu = np.ascontiguousarray(user_ul, dtype=np.int64)
        ud = np.ascontiguousarray(user_dl, dtype=np.int64)
        per_task = 1 if uu.ndim == 2 else 0
        user = np.zeros(R, USER_STATS_DTYPE)
    stats = (OrcRepStats * R)()
    dn = np.ascontiguousarray(down, dtype=np.int64) if down is not None else None
    rg = np.ascontiguousarray(np.atleast_2d(region), dtype=np.int32) if region is not None else None
    lib().orc_run_batch6(R, T, N, stride, policy, _ptr(arrive), _ptr(req), _ptr(mips), _ptr(dl), _ptr(ul),
                         _ptr(init), _ptr(pb), _ptr(pi), _ptr(uu), _ptr(ud), per_task, _ptr(dn), _ptr(rg),
                         int(hier_threshold_s), int(hier_up_tick), 1 if stop_at_ref_abort else 0, _ptr(node),
                         _ptr(status),
                         _ptr(start), _ptr(done), C.cast(stats, C.c_void_p), _ptr(energy), _ptr(h), _ptr(user),
                         threads)
    st = np.frombuffer(stats, dtype=ORC_STATS_DTYPE, count=R).copy()
    return dict(node=node, status=status, start=start, done=done, stats=st, node_energy=energy, hist=h, user=user)


# ---------------------------------------------------------------- v2 model (fognet_oracle_v2.c)

V2_ST_LOCAL, V2_ST_FORWARDED, V2_ST_DROPPED, V2_ST_NO_NODES, V2_ST_ACCEPTED, V2_ST_REJECTED = 3, 4, 5, 6, 7, 8


class OrcV2Stats(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("n_tasks", "n_local", "n_forwarded", "n_accepted", "n_rejected",
                                         "n_dropped", "n_no_nodes", "n_released_broker", "n_inflated",
                                         "n_released_node", "n_relayed", "events", "node_mips_final_sum")] + \
               [("broker_mips_final", C.c_int32), ("status", C.c_int32)]


V2_STATS_DTYPE = np.dtype([(n, _NP[t]) for n, t in OrcV2Stats._fields_])
assert V2_STATS_DTYPE.itemsize == C.sizeof(OrcV2Stats)


class OrcV2Batch(C.Structure):
    _fields_ = [("R", C.c_int32), ("N", C.c_int32), ("node_stride", C.c_int32), ("T", C.c_int64),
                ("arrive_tick", C.c_void_p), ("req_mips", C.c_void_p), ("required_time", C.c_void_p),
                ("broker_mips", C.c_void_p), ("stop_tick", C.c_void_p), ("mips", C.c_void_p), ("dl_tick", C.c_void_p),
                ("ul_tick", C.c_void_p), ("first_adv_tick", C.c_void_p), ("node", C.c_void_p), ("status", C.c_void_p),
                ("start_tick", C.c_void_p), ("done_tick", C.c_void_p), ("stats", C.c_void_p)]


def run_v2(arrive, req, broker_mips, mips, dl, ul, first_adv, stop_tick, required_time=0.01, threads: int = 1):
    """Replay the v2 model (BrokerBaseApp2 + ComputeBrokerApp2).  arrive/req
    [R,T]; broker_mips, stop_tick, required_time scalars or [R]; node params
    [R,N] or [N] (shared).  Returns node/status/start/done [R,T] and stats [R]."""
    arrive = np.ascontiguousarray(np.atleast_2d(arrive), dtype=np.int64)
    req = np.ascontiguousarray(np.atleast_2d(req), dtype=np.int32)
    R, T = arrive.shape
    mips = np.ascontiguousarray(mips, dtype=np.int32)
    N = mips.shape[-1]
    stride = N if mips.ndim == 2 else 0
    dl, ul, fa = (np.ascontiguousarray(x, dtype=np.int64) for x in (dl, ul, first_adv))
    bm = np.ascontiguousarray(np.broadcast_to(broker_mips, (R,)), dtype=np.int32)
    st_ = np.ascontiguousarray(np.broadcast_to(stop_tick, (R,)), dtype=np.int64)
    rt = np.ascontiguousarray(np.broadcast_to(required_time, (R,)), dtype=np.float64)
    node = np.empty((R, T), np.int32)
    status = np.empty((R, T), np.uint8)
    start = np.empty((R, T), np.int64)
    done = np.empty((R, T), np.int64)
    stats = (OrcV2Stats * R)()
    b = OrcV2Batch(R, N, stride, T, _ptr(arrive), _ptr(req), _ptr(rt), _ptr(bm), _ptr(st_), _ptr(mips), _ptr(dl),
                   _ptr(ul), _ptr(fa), _ptr(node), _ptr(status), _ptr(start), _ptr(done), C.cast(stats, C.c_void_p))
    lib().orc_run_v2_batch(C.byref(b), threads)
    return dict(node=node, status=status, start=start, done=done,
                stats=np.frombuffer(stats, dtype=V2_STATS_DTYPE, count=R).copy())
