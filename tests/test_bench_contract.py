"""The bench.py contract the driver depends on (one JSON line from rank 0 with
the metric, the roofline and the CPU-baseline objects), on small
configurations of every workload: C3 (the default), C4, C5 (both policies)
and C1.  Each run also checks the oracle against the device on its CPU sample
(``cpu_baseline.parity``)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOP_KEYS = {"metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"}
ROOFLINE_KEYS = {"bound", "achieved", "peak", "unit", "frac", "traffic"}
CPU_KEYS = {"value", "unit", "cores", "kind", "sample"}


def run_bench(*args):
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], cwd=ROOT, capture_output=True,
                       text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    assert TOP_KEYS <= d.keys()
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["unit"] == "decisions/s"
    assert d["value"] > 0 and d["ms_per_step"] > 0 and "workload" in d["config"]
    assert ROOFLINE_KEYS <= d["roofline"].keys()
    assert CPU_KEYS <= d["cpu_baseline"].keys() and d["cpu_baseline"]["kind"] == "port"
    assert d["failed_replications"] == 0
    return d


def test_bench_c3_small():
    d = run_bench("--R", "64", "--T", "4000", "--steps", "2", "--warmup", "1", "--cpu-reps", "16",
                  "--cpu-reps-1t", "2")
    assert d["scaling"] == "weak" and d["roofline"]["bound"] == "hbm"
    assert d["cpu_baseline"]["parity"] is True
    assert d["stats"]["decisions"] == 64 * 4000
    # N = 256: every replication's reference run ends at a queueTime overflow within its first few hundred
    # publishes (the stale view herds them onto node 0); the line says so
    ra = d["reference_abort"]
    assert ra["replications"] == 64 and 0 < ra["ref_aborted_replications"] <= 64
    assert 0 < ra["ref_defined_decisions"] <= 64 * 4000
    assert d["roofline"]["bytes_per_decision"] == 12 + 24 + 2 * 256 * 48 / 4000
    cb = d["cpu_baseline"]
    assert cb["all_cores"]["threads"] == cb["job_cpus"] and "share_value" in cb
    assert cb["value"] == max(cb["all_cores"]["value"], cb["share_value"])


@pytest.mark.parametrize("policy", ["EXT_HIER", "REF_V3"])
def test_bench_c5_small(policy):
    d = run_bench("--workload", "c5", "--policy", policy, "--R-total", "16", "--T", "2000", "--N", "2048",
                  "--steps", "2", "--warmup", "1", "--cpu-reps", "8", "--cpu-reps-1t", "2")
    assert d["scaling"] == "strong" and d["cpu_baseline"]["parity"] is True
    assert d["stats"]["decisions"] == 16 * 2000


def test_bench_c4_small():
    d = run_bench("--workload", "c4", "--R-total", "512", "--T", "1000", "--steps", "2", "--warmup", "1",
                  "--cpu-reps", "16", "--cpu-reps-1t", "2")
    assert d["roofline"]["bound"] == "valu" and d["cpu_baseline"]["parity"] is True
    assert d["stats"]["decisions"] == 512 * 1000


def test_bench_c1_small():
    d = run_bench("--workload", "c1", "--R-total", "8", "--steps", "1", "--warmup", "1", "--cpu-threads", "4")
    assert d["cpu_baseline"]["parity"] is True and "outputs identical to the device: True" in \
        d["cpu_baseline"]["share_sample"]
    assert d["cpu_baseline"]["all_cores"]["threads"] == d["cpu_baseline"]["job_cpus"]  # all CPUs of the mask
