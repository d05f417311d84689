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
        ("queue_min_ticks", C.c_int64), ("queue_max_ticks", C.c_int64),
        ("resp_min_ticks", C.c_int64), ("resp_max_ticks", C.c_int64),
        ("queue_sum_lo", C.c_uint64), ("queue_sum_hi", C.c_uint64),
        ("queue_sq_lo", C.c_uint64), ("queue_sq_hi", C.c_uint64),
        ("resp_sum_lo", C.c_uint64), ("resp_sum_hi", C.c_uint64),
        ("resp_sq_lo", C.c_uint64), ("resp_sq_hi", C.c_uint64),
        ("events", C.c_int64), ("max_pending", C.c_int32), ("status", C.c_int32),
    ]


ORC_STATS_DTYPE = np.dtype([(n, np.int64 if t in (C.c_int64,) else np.uint64 if t is C.c_uint64 else np.int32)
                            for n, t in OrcRepStats._fields_])

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
        _lib.orc_decide_v3.argtypes = [C.c_int32, p, p, C.c_int32, C.POINTER(C.c_int32)]
        _lib.orc_decide_v3.restype = C.c_int
    return _lib


def _ptr(a):
    return a.ctypes.data_as(C.c_void_p) if a is not None else None


def decide_v3(adv_busy, adv_mips, req):
    adv_busy = np.ascontiguousarray(adv_busy, dtype=np.float64)
    adv_mips = np.ascontiguousarray(adv_mips, dtype=np.int32)
    out = C.c_int32(-7)
    rc = lib().orc_decide_v3(len(adv_busy), _ptr(adv_busy), _ptr(adv_mips), int(req), C.byref(out))
    return rc, out.value


def run_batch(arrive, req, mips, dl, ul, init, threads: int = 1, outputs: bool = True):
    """Replay R replications.  arrive/req: [R,T]; node params [R,N] or [N] (shared)."""
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
    stats = (OrcRepStats * R)()
    lib().orc_run_batch(R, T, N, stride, _ptr(arrive), _ptr(req), _ptr(mips), _ptr(dl), _ptr(ul), _ptr(init),
                        _ptr(node), _ptr(status), _ptr(start), _ptr(done), C.cast(stats, C.c_void_p), threads)
    st = np.frombuffer(stats, dtype=ORC_STATS_DTYPE, count=R).copy()
    return dict(node=node, status=status, start=start, done=done, stats=st)
