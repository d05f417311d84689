"""The OMNeT++ modules (integration/BrokerBaseAppHip.{h,cc,ned} for the v3
broker, integration/BrokerBaseApp2Hip.{h,cc,ned} for the v2 broker C1's ini
selects; integration/BrokerBaseAppRec.{h,cc,ned}, the trace
exporter, §2) are real code: they type-check against a minimal stub of the
OMNeT++ / INET identifiers they touch (tests/adapter/stub: the reference's
member names, types and access, BrokerBaseApp3.h:24-64, BrokerBaseApp2.h:27-60),
and drivers feed each the broker's message stream: the adapters' offloaded
tasks are checked against the oracle on a GPU, the exporter's trace against the
ground truth it was recorded from and its replay (oracle, and the device on a
GPU) against the ground truth's decisions."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = ["-I", os.path.join(ROOT, "tests", "adapter", "stub"), "-I", os.path.join(ROOT, "include"),
       "-I", os.path.join(ROOT, "integration")]


ADAPTERS = {"v3": ("BrokerBaseAppHip.cc", "adapter_drive"), "v2": ("BrokerBaseApp2Hip.cc", "adapter2_drive"),
            "rec": ("BrokerBaseAppRec.cc", "recorder_drive")}


@pytest.mark.parametrize("which", sorted(ADAPTERS))
def test_adapter_type_checks_against_the_reference_interface(which):
    for std in ("c++11", "c++14", "c++17"):  # OMNeT++ 4.6 builds with C++11
        subprocess.run(["g++", f"-std={std}", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        *INC, os.path.join(ROOT, "integration", ADAPTERS[which][0])], check=True)


def build_driver(out_dir, which="v3") -> str:
    name = ADAPTERS[which][1]
    exe = os.path.join(str(out_dir), name)
    lib = os.path.join(ROOT, "fognetsimpp_amd")
    orc = os.path.join(ROOT, "oracle", "build")
    subprocess.run(["g++", "-std=c++14", "-O1", "-Wall", "-Werror", "-Wno-unused-parameter", *INC,
                    os.path.join(ROOT, "tests", "adapter", name + ".cpp"), "-o", exe,
                    "-L", orc, "-loracle", "-L", lib, "-lfognet_hip", "-L/opt/rocm/lib", "-lamdhip64",
                    f"-Wl,-rpath,{orc}", f"-Wl,-rpath,{lib}", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return exe


@pytest.mark.parametrize("which", sorted(ADAPTERS))
def test_adapter_driver_links(tmp_path, which):
    assert os.path.exists(build_driver(tmp_path, which))


@pytest.mark.gpu
def test_adapter_offloads_like_the_reference_on_gpu(tmp_path):
    """Every task the adapter sends goes to the node orc_decide_v3 picks on the
    broker's view at that moment (integer, fractional and NaN busy times,
    N = 1 .. 1000), and an integer view is decided once, not per publish."""
    p = subprocess.run([build_driver(tmp_path)], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "adapter: all checks passed" in p.stdout
    print(p.stdout)


@pytest.mark.gpu
def test_v2_adapter_forwards_like_the_reference_on_gpu(tmp_path):
    """Every publish the v2 adapter forwards is recorded and its task goes to the
    node orc_decide_v2 picks on the MIPS view at that moment (ties, zero MIPS,
    N = 0 .. 1000), or is not sent when that node's MIPS is too small (:262);
    local publishes reach the base class; one device decision per view."""
    p = subprocess.run([build_driver(tmp_path, "v2")], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "adapter2: all checks passed" in p.stdout
    print(p.stdout)


def test_recorder_trace_equals_what_the_broker_saw(tmp_path):
    """BrokerBaseAppRec records the QoS-1 publishes (QoS-0 ones left out) and the node table (CONNECT
    order, first-advert MIPS and tick, ul from the advert's creation, dl from the first status-4/5 ack)
    and writes them at finish(); the trace read back equals the ground truth it was recorded from, and
    the oracle's replay of it reproduces the ground truth's decisions, ticks and statistics (CPU)."""
    p = subprocess.run([build_driver(tmp_path, "rec"), str(tmp_path / "rec.fogntrc"), "--no-gpu"],
                       capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "recorder: all checks passed" in p.stdout


@pytest.mark.gpu
def test_recorder_trace_replays_on_gpu(tmp_path):
    """The exporter's trace through fognet_run_batch on the device: every decision, status, start and
    completion tick and the statistics record equal the ground truth (identical inputs on both paths)."""
    p = subprocess.run([build_driver(tmp_path, "rec"), str(tmp_path / "rec.fogntrc")], capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "recorder: all checks passed" in p.stdout
    print(p.stdout)
