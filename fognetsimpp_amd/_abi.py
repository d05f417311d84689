"""ctypes mirror of include/fognet_hip.h (libfognet_hip C ABI).

The library is built in-tree by ``make`` (see __graft_entry__.build()).  There
is no CPU fallback: importing the package without the built library raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(PKG_DIR, "libfognet_hip.so")

FOGNET_OK = 0
FOGNET_ERR_ARG = 1
FOGNET_ERR_NO_NODES = 2
FOGNET_ERR_DIV0 = 3
FOGNET_ERR_STATE = 4
FOGNET_ERR_DEVICE = 5
FOGNET_ERR_OOM = 6
FOGNET_ERR_CAPACITY = 7
FOGNET_ERR_UNSUPPORTED = 8
FOGNET_REF_ABORTED = 9  # replication status under FLAG_REF_ABORT
FLAG_REF_ABORT = 1  # fognet_batch_in.flags
FOGNET_ERR_INTERNAL = 10  # an internal invariant check failed
TASK_QUEUED, TASK_STARTED, TASK_LOST = 4, 5, 9  # fognet_task_status

FOGNET_POLICY_REF_V3 = 1
FOGNET_POLICY_REF_V2 = 2
FOGNET_POLICY_EXT_LAT = 16
FOGNET_POLICY_EXT_HIER = 32
HIER_REGION_NODES = 1024
TICKS_PER_SECOND = 10**12
# fognet_v2_action (BrokerBaseApp2 decision outcome)
V2_LOCAL, V2_FORWARD, V2_DROPPED, V2_NO_NODES = 3, 4, 5, 6
ABI_VERSION = 10
HIST_METRICS = 2  # 0 queueTime, 1 response
HIST_BINS = 64
COMM_ID_BYTES = 128  # FOGNET_COMM_ID_BYTES


class RepStats(C.Structure):
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


def _np_dtype(struct):
    m = {C.c_int64: np.int64, C.c_uint64: np.uint64, C.c_int32: np.int32, C.c_uint32: np.uint32,
         C.c_double: np.float64}
    fields = []
    for name, t in struct._fields_:
        if hasattr(t, "_length_"):
            fields.append((name, m[t._type_], (t._length_,)))
        else:
            fields.append((name, m[t]))
    dt = np.dtype(fields)
    assert dt.itemsize == C.sizeof(struct), (dt.itemsize, C.sizeof(struct))
    return dt


REP_STATS_DTYPE = _np_dtype(RepStats)


class JobStats(C.Structure):
    _fields_ = [
        ("n_reps", C.c_int64), ("n_failed", C.c_int64),
        ("n_tasks", C.c_int64), ("n_queued", C.c_int64), ("n_started", C.c_int64),
        ("last_tick", C.c_int64),
        ("queue_min_raw", C.c_int64), ("queue_max_raw", C.c_int64),
        ("resp_min_ticks", C.c_int64), ("resp_max_ticks", C.c_int64),
        ("queue_sum", C.c_uint64 * 3), ("queue_sq", C.c_uint64 * 3),
        ("resp_sum", C.c_uint64 * 3), ("resp_sq", C.c_uint64 * 3),
        ("events", C.c_int64), ("max_pending", C.c_int64),
        ("busy_s", C.c_int64), ("energy_j", C.c_double),
        ("n_qtime", C.c_int64), ("n_qtime_overflow", C.c_int64), ("n_ref_aborted", C.c_int64),
    ]


JOB_STATS_DTYPE = _np_dtype(JobStats)


class Moments(C.Structure):
    _fields_ = [("count", C.c_int64), ("min_raw", C.c_int64), ("max_raw", C.c_int64),
                ("sum_lo", C.c_uint64), ("sum_hi", C.c_uint64), ("sq_lo", C.c_uint64), ("sq_hi", C.c_uint64),
                ("sq_top", C.c_uint64), ("overflow", C.c_int64)]


USER_SIGNALS = ("delay", "latency", "latencyH1", "taskTime")


class UserStats(C.Structure):
    _fields_ = [(n, Moments) for n in USER_SIGNALS]


MOMENTS_DTYPE = _np_dtype(Moments)
USER_STATS_DTYPE = np.dtype([(n, MOMENTS_DTYPE) for n in USER_SIGNALS])
assert USER_STATS_DTYPE.itemsize == C.sizeof(UserStats)


class BatchIn(C.Structure):
    _fields_ = [
        ("R", C.c_int32), ("T", C.c_int32), ("N", C.c_int32), ("policy", C.c_int32),
        ("node_stride", C.c_int32), ("ring_capacity", C.c_int32),
        ("arrive_tick", C.c_void_p), ("req_mips", C.c_void_p), ("mips", C.c_void_p),
        ("dl_tick", C.c_void_p), ("ul_tick", C.c_void_p), ("init_adv_tick", C.c_void_p),
        ("p_busy_w", C.c_void_p), ("p_idle_w", C.c_void_p), ("down_tick", C.c_void_p),
        ("region", C.c_void_p), ("hier_up_tick", C.c_int64), ("hier_threshold_s", C.c_int32),
        ("flags", C.c_int32),
    ]


class BatchOut(C.Structure):
    _fields_ = [("node", C.c_void_p), ("status", C.c_void_p), ("start_tick", C.c_void_p),
                ("done_tick", C.c_void_p), ("stats", C.c_void_p), ("node_energy_j", C.c_void_p),
                ("hist", C.c_void_p)]


class GenParams(C.Structure):
    _fields_ = [("seed", C.c_uint32), ("req_lo", C.c_int32), ("req_hi", C.c_int32), ("pad", C.c_int32),
                ("mean_gap_ticks", C.c_void_p), ("lat_scale", C.c_void_p)]


V2_MAX_NODES = 16384
V2_ST_LOCAL, V2_ST_FORWARDED, V2_ST_DROPPED, V2_ST_NO_NODES, V2_ST_ACCEPTED, V2_ST_REJECTED = 3, 4, 5, 6, 7, 8


class V2In(C.Structure):
    _fields_ = [("R", C.c_int32), ("T", C.c_int32), ("N", C.c_int32), ("node_stride", C.c_int32),
                ("queue_capacity", C.c_int32), ("pad", C.c_int32),
                ("arrive_tick", C.c_void_p), ("req_mips", C.c_void_p), ("broker_mips", C.c_void_p),
                ("required_time_s", C.c_void_p), ("stop_tick", C.c_void_p), ("mips", C.c_void_p),
                ("dl_tick", C.c_void_p), ("ul_tick", C.c_void_p), ("first_adv_tick", C.c_void_p)]


class V2Stats(C.Structure):
    _fields_ = [(n, C.c_int64) for n in ("n_tasks", "n_local", "n_forwarded", "n_accepted", "n_rejected",
                                         "n_dropped", "n_no_nodes", "n_released_broker", "n_inflated",
                                         "n_released_node", "n_relayed", "events", "node_mips_final_sum")] + \
               [("broker_mips_final", C.c_int32), ("status", C.c_int32)]


V2_STATS_DTYPE = _np_dtype(V2Stats)


class V2Out(C.Structure):
    _fields_ = [("node", C.c_void_p), ("status", C.c_void_p), ("start_tick", C.c_void_p), ("done_tick", C.c_void_p),
                ("stats", C.c_void_p)]


TRACE_NOTE_BYTES = 160
TRACE_FLAG_POWER = 1
TRACE_FLAG_NODE_ID = 2


class TraceInfo(C.Structure):
    _fields_ = [("R", C.c_int32), ("T", C.c_int32), ("N", C.c_int32), ("node_stride", C.c_int32),
                ("flags", C.c_uint32), ("version", C.c_uint32), ("payload_bytes", C.c_uint64),
                ("checksum", C.c_uint64), ("note", C.c_char * TRACE_NOTE_BYTES)]


# name -> (restype, argtypes); every function declared in include/*.h
P = C.c_void_p
SIGNATURES = {
    "fognet_abi_version": (C.c_int, []),
    "fognet_status_string": (C.c_char_p, [C.c_int]),
    "fognet_create": (C.c_int, [C.POINTER(C.c_void_p), C.c_int]),
    "fognet_destroy": (None, [P]),
    "fognet_last_error": (C.c_char_p, [P]),
    "fognet_decide": (C.c_int, [P, C.c_int, C.c_int32, P, P, C.c_int32, C.POINTER(C.c_int32)]),
    "fognet_decide_window": (C.c_int, [P, C.c_int, C.c_int32, P, P, C.c_int32, P, P]),
    "fognet_decide_batch_dev": (C.c_int, [P, C.c_int, C.c_int64, C.c_int32, P, P, P, P, P, P]),
    "fognet_decide_v2": (C.c_int, [P, C.c_int32, P, C.c_int32, C.c_int32, C.POINTER(C.c_int32),
                                   C.POINTER(C.c_int32)]),
    "fognet_decide_v2_batch_dev": (C.c_int, [P, C.c_int64, C.c_int32, P, P, P, P, P, P]),
    "fognet_run_batch_dev": (C.c_int, [P, C.POINTER(BatchIn), C.POINTER(BatchOut), P]),
    "fognet_run_batch": (C.c_int, [P, C.POINTER(BatchIn), C.POINTER(BatchOut)]),
    "fognet_replay_dev": (C.c_int, [P, C.POINTER(BatchIn), C.POINTER(BatchOut), P]),
    "fognet_rep_stats_dev": (C.c_int, [P, C.POINTER(BatchIn), C.POINTER(BatchOut), P]),
    "fognet_user_stats_dev": (C.c_int, [P, C.POINTER(BatchIn), C.POINTER(BatchOut), P, P, C.c_int32, P, P]),
    "fognet_run_v2_dev": (C.c_int, [P, C.POINTER(V2In), C.POINTER(V2Out), P]),
    "fognet_reduce_stats_dev": (C.c_int, [P, P, C.c_int32, P, P]),
    "fognet_job_stats_init": (None, [C.POINTER(JobStats)]),
    "fognet_job_stats_merge": (None, [C.POINTER(JobStats), C.POINTER(JobStats)]),
    "fognet_job_stats_add_rep": (None, [C.POINTER(JobStats), C.POINTER(RepStats)]),
    "fognet_gen_trace_dev": (C.c_int, [P, C.POINTER(GenParams), C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                       P, P, P, P, P, P, P]),
    "fognet_run_generated_dev": (C.c_int, [P, C.POINTER(GenParams), C.c_int64, C.POINTER(BatchIn),
                                           C.POINTER(BatchOut), P]),
    "fognet_sync": (C.c_int, [P]),
    "fognet_hier_path_stats": (C.c_int, [P, C.POINTER(C.c_int64), C.POINTER(C.c_int64)]),
    "fognet_comm_unique_id": (C.c_int, [C.POINTER(C.c_uint8)]),
    "fognet_comm_create": (C.c_int, [P, C.c_int32, C.c_int32, C.POINTER(C.c_uint8), C.POINTER(P)]),
    "fognet_comm_destroy": (None, [P]),
    "fognet_allreduce_stats": (C.c_int, [P, P, C.POINTER(JobStats), P, P]),
    # include/fognet_io.h (host only, no context)
    "fognet_io_last_error": (C.c_char_p, []),
    "fognet_trace_write": (C.c_int, [C.c_char_p, C.POINTER(BatchIn), P, C.c_char_p]),
    "fognet_trace_info_read": (C.c_int, [C.c_char_p, C.POINTER(TraceInfo)]),
    "fognet_trace_read": (C.c_int, [C.c_char_p, C.POINTER(BatchIn), P]),
    "fognet_write_sca": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.POINTER(JobStats), P]),
    "fognet_write_vec": (C.c_int, [C.c_char_p, C.c_char_p, C.c_char_p, C.c_int32, C.c_int32, P, P, P, P, P, P]),
    "fognet_gen_trace_mqtt": (C.c_int, [C.c_uint32, C.c_int32, P, P, P, P, C.c_int64, C.c_int32, C.c_int32,
                                        C.c_int32, P, P, P, C.POINTER(C.c_int32)]),
}

_lib = None


class FognetError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"fognet status {code}: {msg}")
        self.code = code


def load():
    """Load the in-tree libfognet_hip.so; raises if it has not been built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} is missing: run `make` (or __graft_entry__.build()) first; "
                              "there is no CPU fallback")
        lib = C.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def status_string(code: int) -> str:
    return load().fognet_status_string(code).decode()
