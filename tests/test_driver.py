"""fognet_replay, the command-line trace-replay driver (SURVEY.md §8(b) caller 2,
fognetsimpp_amd/csrc/fognet_replay.cpp): omnetpp.ini lookup, the trace it
builds from the ini keys, its errors, and (GPU) its outputs against the
Python path and the oracle on the same trace."""
import os
import subprocess

import numpy as np
import pytest

from fognetsimpp_amd import formats

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DRIVER = os.path.join(ROOT, "fognetsimpp_amd", "fognet_replay")
INI = os.path.join(ROOT, "tests", "scenarios", "fog5.ini")
MS = 10**9
SEC = 10**12


def drive(*args, check=True):
    p = subprocess.run([DRIVER, *args], capture_output=True, text=True, timeout=120)
    if check and p.returncode != 0:
        raise AssertionError(f"fognet_replay {' '.join(args)} -> {p.returncode}\n{p.stdout}\n{p.stderr}")
    return p


def shown(stdout):
    """--show lines -> {"node": [(mips, start, init)], "user": [(name, start, interval)], "stop": int}"""
    out = {"node": [], "user": [], "stop": None}
    for line in stdout.splitlines():
        f = line.split()
        if f[0] == "node":
            kv = dict(x.split("=") for x in f[3:])
            out["node"].append((int(kv["MIPS"]), int(kv["startTime_ticks"]), int(kv["first_advert_at_broker_ticks"])))
        elif f[0] == "user":
            kv = dict(x.split("=") for x in f[2:])
            out["user"].append((f[1], int(kv["startTime_ticks"]), int(kv["sendInterval_ticks"])))
        elif f[0].startswith("stop_ticks="):
            out["stop"] = int(f[0].split("=")[1])
    return out


@pytest.fixture(scope="module", autouse=True)
def built():
    if not os.path.exists(DRIVER):
        pytest.skip("fognet_replay not built (make)")


def test_general_section_lookup():
    s = shown(drive("-f", INI, "--users", "user[3]", "--dry-run", "--show").stdout)
    assert [m for m, _, _ in s["node"]] == [1000, 2000, 3000, 4000]  # literal ComputeBroker<k> keys
    # first advert at the broker: CONNECT (1 ms) + CONNACK (1 ms) + 0.01 s + advert (1 ms)
    assert all(st == 0 and init == 13 * MS for _, st, init in s["node"])
    assert s["user"] == [(f"user[{u}]", 200 * MS, 1500 * MS) for u in range(3)]
    assert s["stop"] == 300 * SEC


def test_config_extends_and_ranges():
    """[Config Heavy] extends General: its {2..3} range key comes first, the
    rest falls through to General; sim-time-limit bounds stopTime."""
    s = shown(drive("-f", INI, "-c", "Heavy", "--users", "user[2]", "--dry-run", "--show").stdout)
    assert [m for m, _, _ in s["node"]] == [1000, 500, 500, 4000]
    assert s["stop"] == 120 * SEC


def test_config_without_extends_falls_back_to_general():
    s = shown(drive("-f", INI, "-c", "Example", "--nodes", "5", "--dry-run", "--show").stdout)
    assert [m for m, _, _ in s["node"]] == [1000] * 5  # ComputeBroker* wildcard of [Config Example]
    assert s["user"] == [("user", 0, 50 * MS)]
    assert s["stop"] == 1000 * SEC


def test_trace_matches_task_source(tmp_path):
    """The exported trace is fognet_gen_trace_mqtt on the ini's user keys
    (mqttApp2.cc:198-409) with the driver's link options; node parameters in
    CONNECT (index) order."""
    p = str(tmp_path / "g.fogntrc")
    drive("-f", INI, "--users", "user[10]", "--dry-run", "--trace-out", p, "--reps", "2", "--seed", "7")
    tr = formats.load_trace(p)
    assert tr["arrive"].shape[0] == 2
    for r in range(2):
        g = formats.gen_trace_mqtt(7 + r, [200 * MS] * 10, [1500 * MS] * 10, [MS] * 10, [MS] * 10, 300 * SEC)
        np.testing.assert_array_equal(tr["arrive"][r], g["arrive"])
        np.testing.assert_array_equal(tr["req"][r], g["req"])
    np.testing.assert_array_equal(tr["mips"], [1000, 2000, 3000, 4000])
    np.testing.assert_array_equal(tr["dl"], [MS] * 4)
    np.testing.assert_array_equal(tr["init"], [13 * MS] * 4)
    assert "fog5.ini [General]" in tr["note"]


def test_example_publish_count():
    """config C1's publish stream: one user, 50 ms over 1000 s, no CONNACK
    under BrokerBaseApp2 -> 19,999 publishes."""
    out = drive("-f", INI, "-c", "Example", "--nodes", "5", "--dry-run").stdout
    assert "broker=BrokerBaseApp2" in out and "publishes/rep=19999" in out


@pytest.mark.parametrize("cfg,args,msg", [
    # users starting at 0 publish at their CONNACK (~3 ms), before the 13-ms first adverts
    ("Early", ["--users", "user[2]"], "divide by the unadvertised MIPS 0"),
    ("General", ["--users", "nobody"], "no sendInterval"),
    ("General", ["--users", "user[2]", "--stop", "1.0000000000001s"], "not a whole number of ticks"),
    ("General", ["--users", "user[2]", "--dl", "exponential(1s)"], "not a constant time value"),
    ("General", ["--users", "user[2]", "--bogus"], "unknown option"),
    ("Missing", ["--users", "user[2]"], "no [Config Missing] section"),
])
def test_errors(cfg, args, msg):
    """A publish before the last first advert would reach BrokerBaseApp3's
    decision with node 0's MIPS still 0 (SIGFPE, BrokerBaseApp3.cc:267)."""
    p = drive("-f", INI, "-c", cfg, *args, "--dry-run", check=False)
    assert p.returncode == 2 and msg in p.stderr, p.stderr


# ------------------------------------------------------------------ GPU: the driver's replay

@pytest.mark.gpu
def test_driver_replay_matches_python_and_oracle(ctx, tmp_path):
    """The driver's .sca/.vec equal the Python path's files on the same trace,
    and its per-node decisions equal the oracle's."""
    import torch
    import fognetsimpp_amd as fa
    import oracle_lib

    p = str(tmp_path / "g.fogntrc")
    sca, vec = str(tmp_path / "d.sca"), str(tmp_path / "d.vec")
    out = drive("-f", INI, "--users", "user[10]", "--reps", "3", "--trace-out", p, "--sca", sca, "--vec", vec).stdout
    tr = formats.load_trace(p)
    o = oracle_lib.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"])
    per = np.bincount(o["node"].ravel(), minlength=4)
    assert f"tasks_per_node={','.join(str(x) for x in per)}" in out
    assert "failed_reps=0" in out

    dev = torch.device("cuda", 0)
    res = fa.run_batch(ctx, fa.as_device_trace({k: tr[k] for k in ("arrive", "req", "mips", "dl", "ul", "init")}, dev),
                       hist=True)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(res.node.cpu().numpy(), o["node"])
    job = fa.job_from_reps(res.rep_stats())
    sca2, vec2 = str(tmp_path / "p.sca"), str(tmp_path / "p.vec")
    formats.write_sca(sca2, job, res.hist.cpu().numpy(),
                      run_id="General-0", network="FogNet5")
    formats.write_vec(vec2, tr["arrive"][0], tr["dl"], res.node.cpu().numpy()[0], res.status.cpu().numpy()[0],
                      res.start_tick.cpu().numpy()[0], run_id="General-0", network="FogNet5")
    assert open(sca).read() == open(sca2).read()
    assert open(vec).read() == open(vec2).read()


@pytest.mark.gpu
def test_driver_v2_example_all_to_node0():
    """config C1 as shipped through the driver: the v2 broker serves 9 tasks
    itself, then forwards everything to node 0."""
    out = drive("-f", INI, "-c", "Example", "--nodes", "5").stdout
    assert "local=9 forwarded=19990" in out and "failed_reps=0" in out
    assert "forwarded_per_node(rep0)=19990,0,0,0,0" in out


def test_rank_block_of_replications(tmp_path):
    """--world/--rank: rank k replays a contiguous block of the --reps
    replications (the first reps % world ranks take one more), each with its
    global glibc seed, so the job does not depend on the number of GPUs."""
    p = str(tmp_path / "r1.fogntrc")
    drive("-f", INI, "--users", "user[2]", "--reps", "5", "--seed", "3", "--world", "2", "--rank", "1",
          "--comm-id", str(tmp_path / "id"), "--dry-run", "--trace-out", p)
    tr = formats.load_trace(p)
    assert tr["arrive"].shape[0] == 2  # replications 3 and 4
    for i, r in enumerate((3, 4)):
        g = formats.gen_trace_mqtt(3 + r, [200 * MS] * 2, [1500 * MS] * 2, [MS] * 2, [MS] * 2, 300 * SEC)
        np.testing.assert_array_equal(tr["req"][i], g["req"])
    p = drive("-f", INI, "--users", "user[2]", "--world", "2", "--dry-run", check=False)
    assert p.returncode == 2 and "--comm-id" in p.stderr


@pytest.mark.gpu
def test_driver_stats_exchange_world1(ctx, tmp_path):
    """The RCCL exchange path (fognet_allreduce_stats) at world 1 writes the
    same .sca as the plain run, and removes the rendezvous file."""
    a, b, cid = str(tmp_path / "a.sca"), str(tmp_path / "b.sca"), str(tmp_path / "comm.id")
    drive("-f", INI, "--users", "user[10]", "--reps", "4", "--sca", a)
    drive("-f", INI, "--users", "user[10]", "--reps", "4", "--sca", b, "--comm-id", cid)
    assert open(a).read() == open(b).read()
    assert not os.path.exists(cid)


def test_ring_must_be_power_of_two():
    p = drive("-f", INI, "--users", "user[2]", "--ring", "1000", "--dry-run", check=False)
    assert p.returncode == 2 and "--ring must be a power of two" in p.stderr


@pytest.mark.skipif(__import__("torch").cuda.is_available(), reason="needs ranks that cannot open a device")
def test_failed_ranks_do_not_hang(tmp_path):
    """world 2 where no rank can open a gfx950 device (this CPU container): each
    rank reports the failure through the rendezvous files instead of entering
    RCCL, and both exit 1 promptly (no rank is left waiting in a collective)."""
    cid = str(tmp_path / "comm.id")
    procs = [subprocess.Popen([DRIVER, "-f", INI, "--users", "user[2]", "--reps", "2", "--world", "2", "--rank", str(k),
                               "--comm-id", cid], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
             for k in range(2)]
    for p in procs:
        _, err = p.communicate(timeout=60)
        assert p.returncode == 1, err
        assert "failed; skipping the statistics exchange" in err


@pytest.mark.gpu
def test_driver_tiny_ring_same_results(ctx, tmp_path):
    """--ring 4: replications with a node past 4 pending tasks are handed to the
    wide kernel; the run completes with the same .sca as the default ring."""
    a, b = str(tmp_path / "a.sca"), str(tmp_path / "b.sca")
    out_a = drive("-f", INI, "--users", "user[10]", "--reps", "4", "--sca", a).stdout
    out_b = drive("-f", INI, "--users", "user[10]", "--reps", "4", "--sca", b, "--ring", "4").stdout
    assert "failed_reps=0" in out_b
    assert open(a).read() == open(b).read()
    mp = int(out_a.split("max_pending=")[1].split()[0])
    assert mp > 4, "the scenario must overflow a 4-entry ring"
