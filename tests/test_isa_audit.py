"""The replay kernel's inline-asm prefetch is only correct if no
compiler-generated instruction touches the prefetch registers inside the main
loop.  Rebuild the gfx950 ISA and audit it.  CPU only."""
import glob
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_prefetch_registers_only_touched_by_asm():
    subprocess.run(["make", "-s", "-C", ROOT, "asm"], check=True, capture_output=True)
    s = glob.glob(os.path.join(ROOT, "build", "asm", "replay-hip-amdgcn-amd-amdhsa-gfx950.s"))
    assert s, "ISA not generated"
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import check_nh_regs
    assert check_nh_regs.audit(s[0]) == 0
