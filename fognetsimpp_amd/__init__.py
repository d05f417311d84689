"""fognetsimpp_amd — MI355X-native engine for FogNetSim++'s offload-decision hot path.

Scope (BASELINE.json north_star): the broker's task-to-fog-node
argmin (BrokerBaseApp3.cc:265-304) and the fog node's queue update that follows
each decision (ComputeBrokerApp3.cc:205-320), replayed for thousands of
independent what-if replications on gfx950 behind the C ABI in
include/fognet_hip.h (libfognet_hip.so, built in-tree).
"""
from ._abi import FognetError, load as _load_lib  # noqa: F401
from .engine import (NEVER, BatchResult, BrokerBaseApp2, BrokerBaseApp3, Context, allocate_outputs, allocate_trace, as_device_trace, c5_params,  # noqa: F401
                     generate_trace, job_from_reps, merge_job_stats, mobility_regions, power_model, reduce_stats, run_batch, run_generated, run_v2, saturating_trace, summarize,
                     summarize_moments, user_stats, sweep_params)
from . import formats  # noqa: E402,F401

__all__ = ["Context", "BrokerBaseApp2", "BrokerBaseApp3", "BatchResult", "run_batch", "run_generated", "reduce_stats", "merge_job_stats", "power_model",
           "run_v2", "summarize", "summarize_moments", "user_stats", "generate_trace", "c5_params", "mobility_regions", "saturating_trace", "job_from_reps", "formats", "sweep_params", "allocate_outputs", "as_device_trace", "FognetError", "NEVER"]
