"""The OMNeT++ adapter (integration/BrokerBaseAppHip.{h,cc,ned})
is real code: it type-checks against a minimal stub of the OMNeT++ / INET
identifiers it touches (tests/adapter/stub: the reference's member names,
types and access, BrokerBaseApp3.h:24-64), and on a GPU a driver feeds it
adverts and publishes and checks every offloaded task against the oracle."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = ["-I", os.path.join(ROOT, "tests", "adapter", "stub"), "-I", os.path.join(ROOT, "include"),
       "-I", os.path.join(ROOT, "integration")]


def test_adapter_type_checks_against_the_reference_interface():
    for std in ("c++11", "c++14", "c++17"):  # OMNeT++ 4.6 builds with C++11
        subprocess.run(["g++", f"-std={std}", "-fsyntax-only", "-Wall", "-Wextra", "-Werror", "-Wno-unused-parameter",
                        *INC, os.path.join(ROOT, "integration", "BrokerBaseAppHip.cc")], check=True)


def build_driver(out_dir) -> str:
    exe = os.path.join(str(out_dir), "adapter_drive")
    lib = os.path.join(ROOT, "fognetsimpp_amd")
    orc = os.path.join(ROOT, "oracle", "build")
    subprocess.run(["g++", "-std=c++14", "-O1", "-Wall", "-Werror", "-Wno-unused-parameter", *INC,
                    os.path.join(ROOT, "tests", "adapter", "adapter_drive.cpp"), "-o", exe,
                    "-L", orc, "-loracle", "-L", lib, "-lfognet_hip", "-L/opt/rocm/lib", "-lamdhip64",
                    f"-Wl,-rpath,{orc}", f"-Wl,-rpath,{lib}", "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return exe


def test_adapter_driver_links(tmp_path):
    assert os.path.exists(build_driver(tmp_path))


@pytest.mark.gpu
def test_adapter_offloads_like_the_reference_on_gpu(tmp_path):
    """Every task the adapter sends goes to the node orc_decide_v3 picks on the
    broker's view at that moment (integer, fractional and NaN busy times,
    N = 1 .. 1000), and an integer view is decided once, not per publish."""
    p = subprocess.run([build_driver(tmp_path)], capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "adapter: all checks passed" in p.stdout
    print(p.stdout)
