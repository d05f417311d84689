"""libfognet_hip loads and exports exactly the C ABI declared in include/*.h.
CPU only: no compute entry point is called without a GPU."""
import ctypes
import glob
import os
import re

import pytest
import torch

import fognetsimpp_amd._abi as abi

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_functions():
    names = set()
    for h in glob.glob(os.path.join(ROOT, "include", "*.h")):
        src = open(h).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][A-Za-z0-9_ ]*?[\s\*]+(fognet_[a-z0-9_]+)\s*\(", src, re.M):
            names.add(m.group(1))
    return sorted(names)


def test_header_declares_the_boundary():
    names = declared_functions()
    for n in ("fognet_create", "fognet_decide", "fognet_decide_batch_dev", "fognet_run_batch",
              "fognet_run_batch_dev", "fognet_reduce_stats_dev", "fognet_gen_trace_dev"):
        assert n in names


def test_library_exports_every_declared_symbol():
    lib = abi.load()
    for n in declared_functions():
        assert hasattr(lib, n), n
    assert set(declared_functions()) == set(abi.SIGNATURES), "ctypes mirror out of sync with the header"


def test_struct_sizes_match_header():
    # sizes fixed by the header's field lists (all naturally aligned)
    assert ctypes.sizeof(abi.RepStats) == 8 * 17 + 4 * 2 + 8 * 2
    assert ctypes.sizeof(abi.JobStats) == 8 * 10 + 8 * 12 + 8 * 2 + 8 * 2
    assert ctypes.sizeof(abi.BatchIn) == 4 * 6 + 8 * 9
    assert ctypes.sizeof(abi.BatchOut) == 8 * 7


def test_status_strings_and_version():
    lib = abi.load()
    assert lib.fognet_abi_version() == abi.ABI_VERSION == 6
    assert lib.fognet_status_string(abi.FOGNET_ERR_CAPACITY) == b"pending-task ring capacity exceeded"
    assert lib.fognet_status_string(99) == b"unknown status"


def test_job_stats_merge_is_exact_host_code():
    lib = abi.load()
    a, b = abi.JobStats(), abi.JobStats()
    lib.fognet_job_stats_init(ctypes.byref(a))
    lib.fognet_job_stats_init(ctypes.byref(b))
    b.n_reps, b.n_tasks = 3, 10
    b.queue_sum[0], b.queue_sum[1] = 2**64 - 1, 5
    b.queue_min_ticks, b.queue_max_ticks = 7, 9
    lib.fognet_job_stats_merge(ctypes.byref(a), ctypes.byref(b))
    lib.fognet_job_stats_merge(ctypes.byref(a), ctypes.byref(b))
    assert a.n_reps == 6 and a.n_tasks == 20
    assert (a.queue_sum[0], a.queue_sum[1], a.queue_sum[2]) == (2**64 - 2, 11, 0)
    assert a.queue_min_ticks == 7 and a.queue_max_ticks == 9


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU refusal")
def test_create_refuses_without_gpu():
    lib = abi.load()
    h = ctypes.c_void_p()
    assert lib.fognet_create(ctypes.byref(h), 0) == abi.FOGNET_ERR_DEVICE
    assert not h.value
