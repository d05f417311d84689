"""Host-side formats (include/fognet_io.h), CPU only: binary trace files,
OMNeT++ .sca/.vec writers, and the reference task source (mqttApp2's glibc
rand() publish stream) against the system glibc and a Python restatement."""
import ctypes
import heapq
import os

import numpy as np
import pytest

import fognetsimpp_amd as fa
from fognetsimpp_amd import formats
import oracle_lib as ol
import tracegen as tg

libc = ctypes.CDLL("libc.so.6")
MS = 1_000_000_000  # ticks per ms


# ------------------------------------------------------------------ task source

def py_mqtt(seed, start, interval, uplink, downlink, stop, base=200, span=701):
    """Restatement of fognet_gen_trace_mqtt (mqttApp2.cc:198-409) on a heapq
    FES ordered by (tick, insertion seq); rand() from the system glibc."""
    libc.srand(seed)
    fes, seq, gen, pubs = [], 0, [0] * len(start), []

    def push(t, kind, u, g=0):
        nonlocal seq
        heapq.heappush(fes, (t, seq, kind, u, g))
        seq += 1

    def arm(u, now):
        if now + interval[u] < stop:
            gen[u] += 1
            push(now + interval[u], "data", u, gen[u])

    def publish(u, now):
        pubs.append((now + uplink[u], len(pubs), base + libc.rand() % span, u))
        arm(u, now)

    for u in range(len(start)):
        push(start[u], "start", u)
    while fes:
        t, _, kind, u, g = heapq.heappop(fes)
        if kind == "start":
            push(t + uplink[u], "connect", u)
            arm(u, t)
        elif kind == "connect":
            if downlink[u] >= 0:
                push(t + downlink[u], "connack", u)
        elif kind == "connack":
            publish(u, t)
        elif g == gen[u]:
            publish(u, t)
    pubs.sort(key=lambda p: (p[0], p[1]))
    return (np.array([p[0] for p in pubs], np.int64), np.array([p[2] for p in pubs], np.int32),
            np.array([p[3] for p in pubs], np.int32))


def test_glibc_rand_stream_matches_system_glibc():
    """One user, no CONNACK, 50 ms period over 1000 s (wirelessNet.ini:48-50):
    19,999 publishes at k * 50 ms with 200 + rand() % 701 of srand(1)."""
    g = formats.gen_trace_mqtt(1, [0], [50 * MS], [0], [-1], 1000 * 10**12)
    libc.srand(1)
    want = np.array([200 + libc.rand() % 701 for _ in range(19999)], np.int32)
    np.testing.assert_array_equal(g["req"], want)
    np.testing.assert_array_equal(g["arrive"], np.arange(1, 20000, dtype=np.int64) * 50 * MS)
    assert (g["user"] == 0).all()


@pytest.mark.parametrize("seed", [0, 1, 12345, 0xFFFFFFFF])
def test_glibc_rand_seeds(seed):
    g = formats.gen_trace_mqtt(seed, [0], [MS], [0], [-1], 400 * MS, req_base=0, req_span=2**31 - 1)
    libc.srand(seed)
    want = [libc.rand() % (2**31 - 1) for _ in range(g["req"].size)]
    assert g["req"].size == 399
    np.testing.assert_array_equal(g["req"], np.array(want, np.int32))


def test_connack_restarts_the_timer():
    """The CONNACK publishes at once and re-arms the timer from there
    (processConSubAck -> sendMqttData, mqttApp2.cc:319-325, 400-405)."""
    g = formats.gen_trace_mqtt(1, [0], [50 * MS], [3 * MS], [4 * MS], 1000 * MS)
    sends = g["arrive"] - 3 * MS
    np.testing.assert_array_equal(sends, 7 * MS + np.arange(sends.size) * 50 * MS)
    assert sends[-1] < 1000 * MS and sends[-1] + 50 * MS >= 1000 * MS


@pytest.mark.parametrize("case", range(6))
def test_multi_user_event_order_matches_restatement(case):
    rng = np.random.default_rng(100 + case)
    U = int(rng.integers(1, 9))
    # coarse grids make same-tick events (the FES insertion-order rule) common
    start = rng.integers(0, 4, U) * 10 * MS
    interval = rng.choice([10, 20, 30], U) * MS
    uplink = rng.integers(0, 3, U) * 5 * MS
    downlink = np.where(rng.random(U) < 0.7, rng.integers(0, 3, U) * 5 * MS, -1)
    stop = 2000 * MS
    g = formats.gen_trace_mqtt(7 + case, start, interval, uplink, downlink, stop)
    a, r, u = py_mqtt(7 + case, start.tolist(), interval.tolist(), uplink.tolist(), downlink.tolist(), stop)
    np.testing.assert_array_equal(g["arrive"], a)
    np.testing.assert_array_equal(g["req"], r)
    np.testing.assert_array_equal(g["user"], u)
    assert (np.diff(g["arrive"]) >= 0).all()


def test_mqtt_trace_capacity_and_args():
    with pytest.raises(fa.FognetError) as e:
        formats.gen_trace_mqtt(1, [0], [MS], [0], [-1], 100 * MS, cap=10)
    assert e.value.code == 7  # FOGNET_ERR_CAPACITY
    with pytest.raises(fa.FognetError):
        formats.gen_trace_mqtt(1, [0], [0], [0], [-1], 100 * MS)  # interval must be > 0
    assert formats.gen_trace_mqtt(1, [], [], [], [], 100 * MS)["arrive"].size == 0


def test_mqtt_trace_replays_like_c1():
    """C1 as the reference runs it: the generator's trace through the oracle
    sends every decision to node 0 (KAT-1)."""
    g = formats.gen_trace_mqtt(1, [0], [50 * MS], [2 * MS], [2 * MS], 1000 * 10**12)
    n = 5
    lat = np.array([120_000_000 + 7_000_000 * j for j in range(n)], np.int64)
    o = ol.run_batch(g["arrive"][None], g["req"][None], np.full(n, 1000, np.int32), lat, lat, lat)
    assert o["stats"]["status"][0] == 0 and (o["node"] == 0).all()


# ------------------------------------------------------------------ trace files

def _same(a, b):
    for k in ("arrive", "req", "mips", "dl", "ul", "init"):
        np.testing.assert_array_equal(np.asarray(a[k]).reshape(np.asarray(b[k]).shape), b[k], err_msg=k)


@pytest.mark.parametrize("shared,power,ids", [(False, False, False), (True, False, False), (False, True, True),
                                              (True, True, False)])
def test_trace_roundtrip(tmp_path, shared, power, ids):
    tr = tg.make_batch(0x5EED0003, 3, 7, 101, sweep=True)
    if shared:
        tr = dict(tr, mips=tr["mips"][0], dl=tr["dl"][0], ul=tr["ul"][0], init=tr["init"][0])
    if power:
        pb, pi = fa.power_model(tr["mips"])
        tr = dict(tr, p_busy=pb, p_idle=pi)
    nid = (np.arange(7, dtype=np.int32) * 3 + 100) if ids else None
    if ids and not shared:
        nid = np.tile(nid, (3, 1))
    p = str(tmp_path / "t.fnt")
    formats.save_trace(p, tr, node_id=nid, note="C3 sample")
    info = formats.trace_info(p)
    assert (info["R"], info["T"], info["N"]) == (3, 101, 7) and info["note"] == "C3 sample"
    assert info["node_stride"] == (0 if shared else 7)
    back = formats.load_trace(p)
    _same(back, tr)
    if power:
        np.testing.assert_array_equal(back["p_busy"], tr["p_busy"])
        np.testing.assert_array_equal(back["p_idle"], tr["p_idle"])
    else:
        assert "p_busy" not in back
    if ids:
        np.testing.assert_array_equal(back["node_id"], nid)
    # sections start on 64-byte boundaries: the file size is exact
    assert os.path.getsize(p) == 256 + info["payload_bytes"]


def test_trace_replay_identical_after_roundtrip(tmp_path):
    tr = tg.make_batch(0x5EED0001, 2, 16, 500)
    p = str(tmp_path / "t.fnt")
    formats.save_trace(p, tr)
    back = formats.load_trace(p)
    o1 = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"])
    o2 = ol.run_batch(back["arrive"], back["req"], back["mips"], back["dl"], back["ul"], back["init"])
    for k in ("node", "status", "start", "done"):
        np.testing.assert_array_equal(o1[k], o2[k])
    assert o1["stats"].tobytes() == o2["stats"].tobytes()


def test_trace_corruption_is_detected(tmp_path):
    tr = tg.make_batch(5, 2, 4, 50)
    p = str(tmp_path / "t.fnt")
    formats.save_trace(p, tr)
    raw = bytearray(open(p, "rb").read())
    bad = bytearray(raw)
    bad[-3] ^= 0x40  # payload bit flip -> checksum mismatch
    open(p, "wb").write(bad)
    with pytest.raises(fa.FognetError, match="checksum"):
        formats.load_trace(p)
    open(p, "wb").write(raw[:-8])  # truncated
    with pytest.raises(fa.FognetError, match="length"):
        formats.trace_info(p)
    bad = bytearray(raw)
    bad[0:8] = b"NOTATRCE"
    open(p, "wb").write(bad)
    with pytest.raises(fa.FognetError, match="magic"):
        formats.trace_info(p)
    with pytest.raises(fa.FognetError):
        formats.trace_info(str(tmp_path / "missing.fnt"))


def test_empty_trace_roundtrip(tmp_path):
    tr = dict(arrive=np.zeros((2, 0), np.int64), req=np.zeros((2, 0), np.int32), mips=np.full(3, 1000, np.int32),
              dl=np.ones(3, np.int64), ul=np.ones(3, np.int64), init=np.full(3, 2, np.int64))
    p = str(tmp_path / "e.fnt")
    formats.save_trace(p, tr)
    back = formats.load_trace(p)
    assert back["arrive"].shape == (2, 0)
    _same(back, tr)


# ------------------------------------------------------------------ result files

def parse_sca(path):
    """{(module, name): {field: value}} for statistic blocks, plus scalars and bins."""
    stats, scalars, bins, cur = {}, {}, {}, None
    for ln in open(path):
        ln = ln.rstrip("\n")
        if ln.startswith("statistic "):
            mod, name = ln[len("statistic "):].split(" \t")
            cur = (mod, name)
            stats[cur], bins[cur] = {}, []
        elif ln.startswith("field ") and cur:
            _, f, v = ln.split(" ")
            stats[cur][f] = float(v)
        elif ln.startswith("bin\t") and cur:
            _, lo, c = ln.split("\t")
            bins[cur].append((lo, int(c)))
        elif ln.startswith("scalar "):
            mod, name, v = ln[len("scalar "):].split(" \t")
            scalars[(mod, name.strip('"'))] = v
    return stats, scalars, bins


def test_sca_fields_match_exact_statistics(tmp_path):
    tr = tg.make_batch(0x5EED0003, 6, 32, 2000, sweep=True)
    pb, pi = fa.power_model(tr["mips"])
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=4,
                     p_busy=pb, p_idle=pi, hist=True)
    job = fa.job_from_reps(o["stats"])
    hist = o["hist"].sum(axis=0)
    p = str(tmp_path / "General-0.sca")
    formats.write_sca(p, job, hist, run_id="General-0-test", network="FogNet")
    text = open(p).read()
    assert text.startswith("version 2\nrun General-0-test\n")
    stats, scalars, bins = parse_sca(p)
    s = fa.summarize(job)
    q = stats[("FogNet.fogNodes.udpApp[0]", "queueTime:stats")]
    r = stats[("FogNet.broker.udpApp[0]", "response:stats")]
    for blk, ref in ((q, s["queueTime_ms"]), (r, s["response_ms"])):
        assert blk["count"] == ref["count"]
        for f in ("mean", "stddev", "sum", "sqrsum", "min", "max"):
            assert blk[f] == pytest.approx(ref[f], rel=1e-12), f
    assert int(scalars[("FogNet.broker.udpApp[0]", "decisions")]) == 6 * 2000
    assert float(scalars[("FogNet.fogNodes.udpApp[0]", "energy J")]) == pytest.approx(float(o["stats"]["energy_j"].sum()),
                                                                                      rel=1e-12)
    hb = bins[("FogNet.fogNodes.udpApp[0]", "queueTime:histogram")]
    assert hb[0] == ("-INF", 0) and [c for _, c in hb[1:]] == hist[0].tolist()
    assert [lo for lo, _ in hb[1:4]] == ["0", "1", "2"]
    # the stats block layout of General-0.sca:4957-4967
    i = text.index("statistic FogNet.fogNodes.udpApp[0] \tqueueTime:stats\n")
    block = text[i:].split("\n")[1:8]
    assert [b.split(" ")[1] for b in block] == ["count", "mean", "stddev", "sum", "sqrsum", "min", "max"]


def test_sca_empty_statistics_print_nan(tmp_path):
    tr = dict(arrive=np.zeros((1, 0), np.int64), req=np.zeros((1, 0), np.int32), mips=np.full(2, 1000, np.int32),
              dl=np.ones(2, np.int64), ul=np.ones(2, np.int64), init=np.full(2, 2, np.int64))
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"])
    p = str(tmp_path / "e.sca")
    formats.write_sca(p, fa.job_from_reps(o["stats"]))
    text = open(p).read()
    assert "field count 0\nfield mean -nan\nfield stddev -nan\nfield sum 0\nfield sqrsum 0\nfield min -nan\n" in text


def test_vec_queue_time_vectors(tmp_path):
    tr = tg.make_batch(0x5EED0002, 1, 8, 1500, rho=0.95)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"])
    p = str(tmp_path / "General-0.vec")
    formats.write_vec(p, tr["arrive"][0], tr["dl"][0], o["node"][0], o["status"][0], o["start"][0])
    decl, data = {}, {}
    for ln in open(p):
        if ln.startswith("vector "):
            f = ln.split()
            decl[int(f[1])] = (f[2], f[3], f[4])
        elif ln[:1].isdigit():
            vid, t, v = ln.rstrip("\n").split("\t")
            data.setdefault(int(vid), []).append((t, v))
    assert decl[0] == ("FogNet.broker.udpApp[0]", "decision:vector", "TV")
    assert decl[3] == ("FogNet.fogNode[2].udpApp[0]", "queueTime:vector", "TV")
    assert [int(v) for _, v in data[0]] == o["node"][0].tolist()
    n_q = sum(len(v) for k, v in data.items() if k > 0)
    assert n_q == int(o["stats"]["n_queued"][0]) > 0
    # values: (start - arrival at node) in ms; times: exact decimal seconds
    for j in range(8):
        idx = np.nonzero((o["node"][0] == j) & (o["status"][0] == 4))[0]
        got = data.get(1 + j, [])
        assert len(got) == idx.size
        for (t, v), i in zip(got, idx):
            q = int(o["start"][0][i]) - int(tr["arrive"][0][i] + tr["dl"][0][j])
            assert float(v) == pytest.approx(q / 1e9, rel=1e-13)
            sec, _, frac = t.partition(".")
            assert int(sec) * 10**12 + int((frac + "0" * 12)[:12]) == int(o["start"][0][i])
