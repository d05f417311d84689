"""libfognet_hip loads and exports exactly the C ABI declared in include/*.h.
CPU only: no compute entry point is called without a GPU."""
import ctypes
import glob
import os
import re
import subprocess

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


def test_struct_layouts_match_header(tmp_path):
    """sizeof/offsetof of every struct field as the C compiler lays out
    include/fognet_hip.h, against the ctypes mirror."""
    structs = {"fognet_rep_stats": abi.RepStats, "fognet_job_stats": abi.JobStats, "fognet_moments": abi.Moments,
               "fognet_user_stats": abi.UserStats, "fognet_batch_in": abi.BatchIn, "fognet_batch_out": abi.BatchOut,
               "fognet_gen_params": abi.GenParams, "fognet_v2_in": abi.V2In, "fognet_v2_stats": abi.V2Stats,
               "fognet_v2_out": abi.V2Out}
    lines = []
    for cname, st in structs.items():
        lines.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in st._fields_:
            lines.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    src = tmp_path / "layout.c"
    src.write_text("#include <stdio.h>\n#include <stddef.h>\n#include \"fognet_hip.h\"\nint main(void){" +
                   "\n".join(lines) + "return 0;}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    got = dict(ln.split() for ln in subprocess.run([str(exe)], check=True, capture_output=True,
                                                    text=True).stdout.splitlines())
    for cname, st in structs.items():
        assert int(got[cname]) == ctypes.sizeof(st), cname
        for f, _ in st._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(st, f).offset, f"{cname}.{f}"


def test_status_strings_and_version():
    lib = abi.load()
    assert lib.fognet_abi_version() == abi.ABI_VERSION == 10
    assert lib.fognet_status_string(abi.FOGNET_ERR_CAPACITY) == b"capacity exceeded"
    assert lib.fognet_status_string(99) == b"unknown status"


def test_job_stats_merge_is_exact_host_code():
    lib = abi.load()
    a, b = abi.JobStats(), abi.JobStats()
    lib.fognet_job_stats_init(ctypes.byref(a))
    lib.fognet_job_stats_init(ctypes.byref(b))
    b.n_reps, b.n_tasks = 3, 10
    b.queue_sum[0], b.queue_sum[1] = 2**64 - 1, 5
    b.queue_min_raw, b.queue_max_raw = 7, 9
    lib.fognet_job_stats_merge(ctypes.byref(a), ctypes.byref(b))
    lib.fognet_job_stats_merge(ctypes.byref(a), ctypes.byref(b))
    assert a.n_reps == 6 and a.n_tasks == 20
    assert (a.queue_sum[0], a.queue_sum[1], a.queue_sum[2]) == (2**64 - 2, 11, 0)
    assert a.queue_min_raw == 7 and a.queue_max_raw == 9


@pytest.mark.skipif(torch.cuda.is_available(), reason="checks the no-GPU refusal")
def test_create_refuses_without_gpu():
    lib = abi.load()
    h = ctypes.c_void_p()
    assert lib.fognet_create(ctypes.byref(h), 0) == abi.FOGNET_ERR_DEVICE
    assert not h.value


def build_c_client():
    """tests/c/abi_c_client.c: plain C99 against include/fognet_hip.h, linked to the library."""
    exe = os.path.join(ROOT, "build", "abi_c_client")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.run(["gcc", "-std=c99", "-pedantic", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "c", "abi_c_client.c"), "-o", exe,
                    "-L", os.path.join(ROOT, "fognetsimpp_amd"), "-lfognet_hip", "-L/opt/rocm/lib", "-lamdhip64",
                    "-Wl,-rpath," + os.path.join(ROOT, "fognetsimpp_amd"), "-Wl,-rpath,/opt/rocm/lib"], check=True)
    return exe


@pytest.mark.skipif(torch.cuda.is_available(), reason="the no-GPU path of the C client")
def test_plain_c_client_builds_and_refuses_without_gpu():
    p = subprocess.run([build_c_client(), "--no-gpu"], capture_output=True, text=True, timeout=60)
    assert p.returncode == 0, p.stderr


@pytest.mark.gpu
def test_plain_c_client_on_gpu():
    """fognet_decide / fognet_decide_window / fognet_run_batch called from C."""
    p = subprocess.run([build_c_client()], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "all checks passed" in p.stdout


def test_numeric_limits_match_header(tmp_path):
    """The ctypes mirror's constants (limits, ABI version, histogram shape, policy ids) equal the
    header's macros as the C compiler evaluates them."""
    pairs = {"FOGNET_ABI_VERSION": abi.ABI_VERSION, "FOGNET_HIST_METRICS": abi.HIST_METRICS,
             "FOGNET_HIST_BINS": abi.HIST_BINS, "FOGNET_HIER_REGION_NODES": abi.HIER_REGION_NODES,
             "FOGNET_V2_MAX_NODES": abi.V2_MAX_NODES, "FOGNET_COMM_ID_BYTES": abi.COMM_ID_BYTES,
             "FOGNET_TICKS_PER_SECOND": abi.TICKS_PER_SECOND, "FOGNET_FLAG_REF_ABORT": abi.FLAG_REF_ABORT,
             "FOGNET_POLICY_REF_V3": abi.FOGNET_POLICY_REF_V3, "FOGNET_POLICY_EXT_HIER": abi.FOGNET_POLICY_EXT_HIER,
             "FOGNET_ERR_UNSUPPORTED": abi.FOGNET_ERR_UNSUPPORTED}
    src = tmp_path / "limits.c"
    src.write_text("#include <stdio.h>\n#include \"fognet_hip.h\"\nint main(void){" +
                   "".join(f'printf("{k} %lld\\n", (long long)({k}));' for k in pairs) + "return 0;}\n")
    exe = tmp_path / "limits"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)],
                   check=True)
    got = dict(ln.split() for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines())
    for k, v in pairs.items():
        assert int(got[k]) == v, k


def test_missing_library_fails_loudly(monkeypatch, tmp_path):
    """No CPU fallback: without the built HIP library the package refuses to run."""
    monkeypatch.setattr(abi, "_lib", None)
    monkeypatch.setattr(abi, "LIB_PATH", str(tmp_path / "libfognet_hip.so"))
    with pytest.raises(ImportError, match="no CPU fallback"):
        abi.load()
    with pytest.raises(ImportError):
        abi.status_string(0)
