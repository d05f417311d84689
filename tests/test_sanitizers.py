"""Host C/C++ under AddressSanitizer + UBSan (SURVEY.md §5 "Race detection /
sanitizers"): `make asan` builds the CPU oracle, the trace / result-file I/O
(csrc/io.cpp) and the command-line driver (csrc/fognet_replay.cpp) with
-fsanitize=address,undefined and drives them through their paths
(tests/c/oracle_check.c, tests/c/io_check.cpp, driver --dry-run and error
exits).  Any sanitizer report fails the target.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_make_asan_is_clean():
    p = subprocess.run(["make", "-s", "-C", ROOT, "asan"], capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    assert "asan: oracle, io and driver clean" in p.stdout
