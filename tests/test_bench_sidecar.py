"""bench.py quotes a committed rocprofv3 profile (``roofline.kernel_avg_ms_rocprof``) only for a
run of the very library that was profiled, with the same config, and only when the profile's
average does not exceed its own run's ms_per_step.  CPU only: the
sidecar logic reads files and hashes the loaded library; no kernel runs."""
import argparse
import hashlib
import importlib.util
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _args():
    return argparse.Namespace(workload="c3", policy=None, c5_recipe="light")


def _write(tmp_path, side):
    (tmp_path / "profiles").mkdir(exist_ok=True)
    (tmp_path / "profiles" / "kernel_profile_c3.json").write_text(json.dumps(side))


def test_sidecar_quoted_only_for_the_profiled_library(bench, tmp_path, monkeypatch):
    lib = tmp_path / "lib.so"
    lib.write_bytes(b"the profiled build")
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench._abi, "LIB_PATH", str(lib))
    cfg = {"workload": "c3", "R": 4096}
    line = {"n_gpus": 1, "config": cfg, "ms_per_step": 11.5}
    side = {"avg_ms": 11.37, "ms_per_step": 11.41, "config": cfg, "command": "rocprofv3 ... bench.py",
            "lib_sha256": hashlib.sha256(b"the profiled build").hexdigest()}
    _write(tmp_path, side)
    r = bench.rocprof_kernel_avg(_args(), line)
    assert r["kernel_avg_ms_rocprof"] == 11.37
    assert r["rocprof_ms_per_step"] == 11.41 and r["ms_per_step_this_run"] == 11.5
    # a faster box than the profiled one: still quoted (its own run bounds the average), both figures shown
    r = bench.rocprof_kernel_avg(_args(), dict(line, ms_per_step=11.2))
    assert r["kernel_avg_ms_rocprof"] == 11.37 and r["ms_per_step_this_run"] == 11.2
    # another build (a kernel changed since the profile): never quoted
    lib.write_bytes(b"a later build")
    r = bench.rocprof_kernel_avg(_args(), line)
    assert r["kernel_avg_ms_rocprof"] is None and "rocprof_profile_other_build" in r
    lib.write_bytes(b"the profiled build")
    # another config, or an average above the profiled run's own step: rejected
    r = bench.rocprof_kernel_avg(_args(), dict(line, config={"workload": "c3", "R": 64}))
    assert r["kernel_avg_ms_rocprof"] is None and "rocprof_profile_rejected" in r
    _write(tmp_path, dict(side, avg_ms=11.6))
    r = bench.rocprof_kernel_avg(_args(), line)
    assert r["kernel_avg_ms_rocprof"] is None and "rocprof_profile_rejected" in r
    # multi-GPU lines quote nothing
    _write(tmp_path, side)
    assert bench.rocprof_kernel_avg(_args(), dict(line, n_gpus=2)) == {"kernel_avg_ms_rocprof": None}
