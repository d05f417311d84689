"""bench.py against a variant build (tools/build_variant.sh): FOGNET_LIB=build/ab/X/libfognet_hip.so
python tools/bench_var.py <bench args>.  Diagnostics only; the product bench loads the in-tree library."""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from fognetsimpp_amd import _abi  # noqa: E402

_abi.LIB_PATH = os.environ["FOGNET_LIB"]
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
