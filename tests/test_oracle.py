"""The CPU restatement (oracle/) against the hand-traced known answers and the
reference's structural invariants.  CPU only."""
import ctypes

import numpy as np
import pytest

import golden_io
import oracle_lib as ol
import tracegen as tg

TPS = 10**12


@pytest.mark.parametrize("case", golden_io.decide_cases(), ids=lambda c: c[0])
def test_decide_known_answers(case):
    name, busy, mips, req, node, err = case
    rc, k = ol.decide_v3(busy, mips, req)
    if err is not None:
        assert rc == err
    else:
        assert rc == 0 and k == node


@pytest.mark.parametrize("case", golden_io.replay_cases(), ids=lambda c: c[0])
def test_replay_known_answers(case):
    name, tr, exp = case
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"])
    assert o["stats"]["status"][0] == 0
    np.testing.assert_array_equal(o["node"][0], exp["node"])
    np.testing.assert_array_equal(o["status"][0], exp["status"])
    np.testing.assert_array_equal(o["start"][0], exp["start"])
    np.testing.assert_array_equal(o["done"][0], exp["done"])
    assert o["stats"]["n_queued"][0] == exp["n_queued"]
    assert o["stats"]["n_started"][0] == exp["n_started"]


def c1_trace():
    """Config C1 (simulations/example/wirelessNet.ini): 5 nodes of MIPS 1000, one
    mqttApp2 user publishing every 50 ms from 0.05 s to 999.95 s (19,999 tasks)
    with MIPSRequired = 200 + rand() % 701 (mqttApp2.cc:370; glibc rand(), seed 1)."""
    libc = ctypes.CDLL("libc.so.6")
    libc.srand(1)
    req = np.array([200 + libc.rand() % 701 for _ in range(19999)], np.int32)
    arrive = (np.arange(1, 20000, dtype=np.int64) * 50_000_000_000)
    n = 5
    lat = np.array([120_000_000 + 7_000_000 * j for j in range(n)], np.int64)
    return dict(arrive=arrive, req=req, mips=np.full(n, 1000, np.int32), dl=lat, ul=lat, init=lat + 10_000_000_000)


def test_c1_example_run_all_to_node0():
    tr = c1_trace()
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"])
    st = o["stats"][0]
    assert st["status"] == 0 and st["n_tasks"] == 19999
    assert (o["node"][0] == 0).all()
    assert (o["status"][0] == 5).all()
    a = tr["arrive"] + tr["dl"][0]
    np.testing.assert_array_equal(o["start"][0], a)
    np.testing.assert_array_equal(o["done"][0], a)
    assert st["events"] == 2 * 5 + 4 * 19999


def check_fifo_invariants(tr, o):
    """Per-node FIFO single-server recurrence implied by ComputeBrokerApp3.cc:269-320,224-256."""
    arrive, req = np.atleast_2d(tr["arrive"]), np.atleast_2d(tr["req"])
    R, T = arrive.shape
    for r in range(R):
        mips = tr["mips"][r] if tr["mips"].ndim == 2 else tr["mips"]
        dl = tr["dl"][r] if tr["dl"].ndim == 2 else tr["dl"]
        node, start, done, status = o["node"][r], o["start"][r], o["done"][r], o["status"][r]
        S = req[r] // mips[node]
        a = arrive[r] + dl[node]
        np.testing.assert_array_equal(done - start, S.astype(np.int64) * TPS)
        assert (start >= a).all()
        assert ((status == 5) <= (start == a)).all()
        for k in np.unique(node):
            idx = np.nonzero(node == k)[0]
            prev = np.concatenate([[np.iinfo(np.int64).min], done[idx][:-1]])
            np.testing.assert_array_equal(start[idx], np.maximum(a[idx], prev))


def test_oracle_fifo_invariants_c2_like():
    b = tg.make_batch(0x5EED0001, 2, 64, 3000)
    o = ol.run_batch(b["arrive"], b["req"], b["mips"], b["dl"], b["ul"], b["init"], threads=2)
    assert (o["stats"]["status"] == 0).all()
    check_fifo_invariants(b, o)
    st = o["stats"]
    assert (st["events"] == 2 * 64 + 4 * 3000).all()
    assert (st["n_queued"] + st["n_started"] == 3000).all()


def test_oracle_threads_deterministic():
    b = tg.make_batch(7, 6, 16, 800, rho=0.9)
    o1 = ol.run_batch(b["arrive"], b["req"], b["mips"], b["dl"], b["ul"], b["init"], threads=1)
    o4 = ol.run_batch(b["arrive"], b["req"], b["mips"], b["dl"], b["ul"], b["init"], threads=4)
    for k in ("node", "status", "start", "done"):
        np.testing.assert_array_equal(o1[k], o4[k])
    assert o1["stats"].tobytes() == o4["stats"].tobytes()


def test_oracle_div0_when_node0_has_not_advertised():
    # node 0's first advert lands after the first publish -> brokers[0].MIPS == 0 (SIGFPE)
    tr = dict(arrive=np.array([100], np.int64), req=np.array([1000], np.int32), mips=np.array([1000, 1000], np.int32),
              dl=np.array([1, 1], np.int64), ul=np.array([10, 10], np.int64), init=np.array([500, 50], np.int64))
    o = ol.run_batch(**{k: tr[k] for k in ("arrive", "req", "mips", "dl", "ul", "init")})
    assert o["stats"]["status"][0] == 3


def test_oracle_state_error_when_task_meets_pending_advert_timer():
    # node 1's one-shot ADVERTISEMIPS self-message is still pending when a task
    # reaches it -> scheduleAt() on a scheduled message (ComputeBrokerApp3.cc:301)
    tr = dict(arrive=np.array([100, 101, 3 * TPS], np.int64), req=np.array([2000, 2000, 1000], np.int32),
              mips=np.array([1000, 1000], np.int32), dl=np.array([5, 5], np.int64), ul=np.array([10, 10], np.int64),
              init=np.array([10, 5 * TPS], np.int64))
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"])
    # t0, t1 -> node 0; node 0 advertises busy 2 at 2e12+115; t2 -> node 1 at 3e12+5
    assert o["node"][0][:2].tolist() == [0, 0]
    assert o["stats"]["status"][0] == 4


# ------------------------------------------------------------------ builder-defined rows (a10/a11, EXT_LAT)
# None of these is in the reference: the answers below are derived by hand from
# the definitions in include/fognet_hip.h (parity unpinned against FogNetSim++).

@pytest.mark.parametrize("ticks,b", [(0, 0), (999_999_999, 0), (10**9, 1), (2 * 10**9 - 1, 1), (2 * 10**9, 2),
                                     (3 * 10**9, 2), (4 * 10**9, 3), (1023 * 10**9, 10), (1024 * 10**9, 11),
                                     (2**62, 33), (-5, 0)])
def test_hist_bin_rule(ticks, b):
    assert ol.lib().orc_hist_bin(ticks) == b


def test_ext_lat_decide_known_answers():
    # cost_j = dl_j + (busy_j + min(req // mips_j, 2^20)) * 1e12
    busy = [3.0, 1.0, 1.0, 0.0]
    mips = [1000, 1000, 4000, 500]
    dl = [0, 5 * 10**11, 10**11, 0]
    # req 4000: costs 7e12, 5.5e12, 2.1e12, 8e12 -> node 2
    assert ol.decide_ext_lat(busy, mips, dl, 4000) == (0, 2)
    # req 0: costs 3e12, 1.5e12, 1.1e12, 0 -> node 3
    assert ol.decide_ext_lat(busy, mips, dl, 0) == (0, 3)
    # tie on cost -> lowest index
    assert ol.decide_ext_lat([1.0, 1.0], [1000, 1000], [7, 7], 2500) == (0, 0)
    # network delay decides between otherwise equal nodes
    assert ol.decide_ext_lat([0.0, 0.0], [1000, 1000], [9, 8], 2500) == (0, 1)
    # saturation: both service times exceed 2^20 s -> equal saturated service, busy decides
    assert ol.decide_ext_lat([5.0, 4.0], [1, 2], [0, 0], 2**31 - 1) == (0, 1)
    assert ol.decide_ext_lat([], [], [], 5)[0] == 2  # NO_NODES
    assert ol.decide_ext_lat([0.0], [0], [0], 5)[0] == 3  # DIV0


def test_energy_known_answer():
    """One node, two tasks of 3 s and 5 s back to back, plus an idle node:
    H = last completion; E_j = Pb*B_j + Pi*(H - B_j)."""
    dl = np.array([10**9, 10**9], np.int64)
    ul = np.array([10**9, 10**9], np.int64)
    init = ul.copy()
    arrive = np.array([10**10, 10**10 + 1], np.int64)
    req = np.array([3000, 5000], np.int32)
    mips = np.array([1000, 1000], np.int32)
    pb = np.array([50.5, 70.0])
    pi = np.array([10.25, 20.0])
    o = ol.run_batch(arrive, req, mips, dl, ul, init, p_busy=pb, p_idle=pi, hist=True)
    st = o["stats"][0]
    assert st["status"] == 0 and (o["node"][0] == 0).all()  # stale view: node 0 twice
    H = 10**10 + 10**9 + 8 * TPS
    assert st["last_tick"] == H and st["busy_s"] == 8
    e0 = 50.5 * 8 + 10.25 * ((H - 8 * TPS) / 1e12)
    e1 = 0.0 + 20.0 * (H / 1e12)
    assert o["node_energy"][0].tolist() == [e0, e1]
    assert st["energy_j"] == e0 + e1
    # histograms: task 1 queued 3 s - 1 tick (bin 12: 2048..4095 ms); responses 3.001 s and 8.001 s - 1 tick
    h = o["hist"][0]
    assert h[0].sum() == 1 and h[0][12] == 1
    assert h[1].sum() == 2 and h[1][12] == 1 and h[1][13] == 1


def test_ext_lat_replay_invariants():
    tr = tg.make_batch(77, 4, 64, 3000, sweep=True)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=4,
                     policy=ol.POLICY_EXT_LAT)
    assert (o["stats"]["status"] == 0).all()
    # spreads load (the reference policy herds onto one node between adverts)
    assert all(len(np.unique(o["node"][r])) > 8 for r in range(4))
    check_fifo_invariants(tr, o)


@pytest.mark.parametrize("case", golden_io.decide_v2_cases(), ids=lambda c: c[0])
def test_decide_v2_known_answers(case):
    """Oracle restatement of BrokerBaseApp2's decision pinned by hand-traced vectors."""
    name, mips, local, req, action, node = case
    assert ol.decide_v2(mips, local, req) == (action, node)


def test_user_side_known_answer():
    """One publish at tick 100, node 0 (MIPS 1000, dl 3, ul 5), MIPSRequired 2000
    (S = 2 s), user uplink 7 / downlink 11 ticks.  Hand-traced: broker `delay` =
    7 (BrokerBaseApp3.cc:143); its status-4 pubAck reaches the user at 111,
    created at 93 -> latencyH1 18; the node's status-5 ack leaves at 103,
    reaches the broker at 108, the user at 119 -> latency 26; status 6 leaves
    at 103 + 2e12 -> taskTime 2e12 + 26 (mqttApp2.cc:257-291).  The ms signals
    are emitted as (simTime() - created) * 1000: raw = 1000 x ticks here (exact
    in double below 2^53); delay is emitted unscaled (raw = ticks)."""
    tr = dict(arrive=np.array([[100]], np.int64), req=np.array([[2000]], np.int32), mips=np.array([1000], np.int32),
              dl=np.array([3], np.int64), ul=np.array([5], np.int64), init=np.array([5], np.int64))
    o = ol.run_batch(**tr, user_ul=np.array([7]), user_dl=np.array([11]))
    u = o["user"][0]
    got = {n: (int(u[n]["count"]), int(u[n]["min_raw"]), int(u[n]["max_raw"])) for n in ol.USER_SIGNALS}
    assert got == {"delay": (1, 7, 7), "latencyH1": (1, 18000, 18000), "latency": (1, 26000, 26000),
                   "taskTime": (1, (2 * 10**12 + 26) * 1000, (2 * 10**12 + 26) * 1000)}


def test_user_side_events_do_not_change_decisions():
    """The ack relay is modelled as real FES events; they carry no state back
    into the decision loop, so every output and record is unchanged."""
    tr = tg.make_batch(7, 3, 16, 2000, rho=0.9)
    a = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=3)
    rng = np.random.default_rng(3)
    uu, ud = rng.integers(0, 10**9, (2, 3, 2000))
    b = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=3, user_ul=uu,
                     user_dl=ud)
    for k in ("node", "status", "start", "done"):
        np.testing.assert_array_equal(a[k], b[k])
    assert a["stats"].tobytes() == b["stats"].tobytes()
    u = b["user"]
    np.testing.assert_array_equal(u["delay"]["count"], 2000)
    np.testing.assert_array_equal(u["taskTime"]["count"], 2000)
    np.testing.assert_array_equal(u["latency"]["count"], b["stats"]["n_started"])
    np.testing.assert_array_equal(u["latencyH1"]["count"], 2000 + b["stats"]["n_queued"])


@pytest.mark.parametrize("case", golden_io.replay_v2_cases(), ids=lambda c: c[0])
def test_v2_replay_known_answers(case):
    """The v2 model restatement (oracle/fognet_oracle_v2.c) on hand-traced traces."""
    name, tr, e = case
    o = ol.run_v2(tr["arrive"], tr["req"], tr["broker_mips"], tr["mips"], tr["dl"], tr["ul"], tr["first_adv"],
                  tr["stop"])
    assert o["node"][0].tolist() == e["node"]
    assert o["status"][0].tolist() == e["status"]
    assert o["start"][0].tolist() == e["start"]
    assert o["done"][0].tolist() == e["done"]
    st = o["stats"][0]
    assert int(st["status"]) == e.get("rep_status", 0)
    for k, v in e.items():
        if k.startswith("n_") or k.endswith("_final") or k.endswith("_sum"):
            assert int(st[k]) == v, k


def test_v2_c1_example_run_has_rounding_forwards():
    """C1 as shipped (wirelessNet.ini: 1 user, 50-ms interval, MIPSRequired 200 + rand() % 701,
    broker and 5 nodes at 1000 MIPS).  The broker's single timer fails to release a
    local reservation when dbl(t) + 0.01 > dbl(t + 0.01 s) (IEEE rounding); only a
    new local task re-arms it, and once the pool is below 200 MIPS no task is local
    again: the pool stays stuck and every later publish is forwarded -- to node 0,
    the only outcome of the v2 forward rule with equal MIPS (the General-0.sca fact
    that ComputeBroker1 received all forwarded tasks)."""
    from fognetsimpp_amd import formats
    MS = 10**9
    g = formats.gen_trace_mqtt(1, [0], [50 * MS], [MS], [-1], 1000 * 10**12)
    n = 5
    o = ol.run_v2(g["arrive"], g["req"], 1000, np.full(n, 1000, np.int32), np.full(n, MS), np.full(n, MS),
                  np.full(n, 20 * MS), 1000 * 10**12)
    st = o["stats"][0]
    assert int(st["status"]) == 0 and int(st["n_tasks"]) == 19999
    assert (int(st["n_local"]), int(st["n_forwarded"]), int(st["broker_mips_final"])) == (9, 19990, 101)
    assert int(st["n_accepted"]) == int(st["n_relayed"]) == 19990
    fw = o["node"][0][o["status"][0] != 3]
    assert (fw == 0).all()


@pytest.mark.parametrize("case", golden_io.replay_down_cases(), ids=lambda c: c[0])
def test_replay_down_known_answers(case):
    """Node-down extension (handleNodeCrash, ComputeBrokerApp3.cc:423-427): hand-traced cases."""
    name, tr, exp = case
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], down=tr["down"])
    st = o["stats"][0]
    assert st["status"] == 0
    np.testing.assert_array_equal(o["node"][0], exp["node"])
    np.testing.assert_array_equal(o["status"][0], exp["status"])
    np.testing.assert_array_equal(o["start"][0], exp["start"])
    np.testing.assert_array_equal(o["done"][0], exp["done"])
    for k in ("n_queued", "n_started", "busy_s", "events", "max_pending"):
        assert st[k] == exp[k], k
    assert st["n_tasks"] == len(exp["node"])
    # queueTime raw values = 1000 x the tick difference at these small ticks (exact round trip)
    assert st["queue_sum_lo"] == exp["queue_sum_ms"] * 10**12 and st["queue_sum_hi"] == 0
    assert st["resp_sum_lo"] == exp["resp_sum_ms"] * 10**9 and st["resp_sum_hi"] == 0


def test_replay_down_never_is_identity():
    """down = INT64_MAX everywhere reproduces the run without the extension."""
    rng = np.random.default_rng(5)
    T, N = 400, 6
    arrive = np.cumsum(rng.integers(0, 3 * 10**11, T)).astype(np.int64)
    req = rng.integers(0, 9000, T).astype(np.int32)
    mips = rng.integers(500, 4000, N).astype(np.int32)
    dl = rng.integers(0, 10**10, N).astype(np.int64)
    ul = rng.integers(0, 10**10, N).astype(np.int64)
    init = ul.copy()
    a = ol.run_batch(arrive + 10**10, req, mips, dl, ul, init)
    b = ol.run_batch(arrive + 10**10, req, mips, dl, ul, init, down=np.full(N, np.iinfo(np.int64).max))
    for k in ("node", "status", "start", "done"):
        np.testing.assert_array_equal(a[k], b[k])
    assert a["stats"].tobytes() == b["stats"].tobytes()


def test_replay_down_rejects_early_crash_and_energy():
    tr = golden_io.replay_down_cases()[0][1]
    bad = tr["down"].copy()
    bad[0] = tr["init"][0] - 1  # before the node's first advert reaches the broker
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], down=bad)
    assert o["stats"]["status"][0] == 1  # ORC_ERR_ARG
    pw = np.full(2, 30.0)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], down=tr["down"],
                     p_busy=pw, p_idle=pw)
    assert o["stats"]["status"][0] == 8  # ORC_ERR_UNSUPPORTED


def test_udiv_magic_exact():
    """replay_common.h udiv_magic/udiv (Granlund-Montgomery): the replay
    kernel's S = MIPSRequired / MIPS (ComputeBrokerApp3.cc:276) as a
    multiply-high and shifts, restated in numpy and checked against integer
    division for every divisor up to 2^16, large divisors and extreme numerators."""
    d = np.concatenate([np.arange(1, 1 << 16, dtype=np.uint64),
                        np.array([(1 << 31) - 1, 1 << 31, (1 << 32) - 1, 3 << 30, 123456789], np.uint64)])
    l = np.array([0 if x <= 1 else int(x - 1).bit_length() for x in d], np.uint64)
    m = ((np.uint64(1) << np.uint64(32)) * ((np.uint64(1) << l) - d)) // d + np.uint64(1)
    m &= np.uint64(0xFFFFFFFF)
    sh1 = np.minimum(l, 1)
    sh2 = np.where(l > 1, l - 1, 0).astype(np.uint64)
    rng = np.random.default_rng(5)
    for n in [np.uint64(0), np.uint64(1), np.uint64(0xFFFFFFFF), np.uint64(0x7FFFFFFF), np.uint64(64000), None]:
        nn = rng.integers(0, 1 << 32, d.size, dtype=np.uint64) if n is None else np.full(d.size, n, np.uint64)
        t = (m * nn) >> np.uint64(32)
        q = (t + ((nn - t) >> sh1)) >> sh2
        np.testing.assert_array_equal(q, nn // d)


@pytest.mark.parametrize("case", golden_io.qtime_cases(), ids=lambda c: c[0])
def test_qtime_known_answers(case):
    """queueTime as the reference emits it (ComputeBrokerApp3.cc:238, 306): the
    queueStartTime double round trip above 2^53 ticks, a negative value for a
    task queued and started in one tick, and the simtime_t overflow above ~9223 s."""
    name, tr, exp = case
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], hist=True)
    for k in ("node", "status", "start", "done"):
        np.testing.assert_array_equal(o[k][0], exp[k], err_msg=k)
    golden_io.check_qtime_record(o["stats"][0], exp)
    assert o["hist"][0][0].sum() == exp["n_qtime"]


@pytest.mark.parametrize("case", golden_io.qtime_cases(), ids=lambda c: c[0])
def test_qtime_stop_at_reference_abort(case):
    """The reference ends its run at the first queueTime emission that throws
    (ComputeBrokerApp3.cc:238, no handler up to :84-86): the oracle's stop mode
    reaches exactly the hand-traced prefix (kat_qtime.json stop_start /
    stop_done) and reports the same abort point as the continuing run."""
    name, tr, exp = case
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], stop_at_ref_abort=True)
    np.testing.assert_array_equal(o["node"][0], exp["node"])
    np.testing.assert_array_equal(o["status"][0], exp["status"])
    np.testing.assert_array_equal(o["start"][0], exp["stop_start"])
    np.testing.assert_array_equal(o["done"][0], exp["stop_done"])
    st = o["stats"][0]
    ab = np.iinfo(np.int64).max if exp["abort_tick"] is None else exp["abort_tick"]
    assert st["status"] == 0 and int(st["abort_tick"]) == ab and int(st["abort_task"]) == exp["abort_task"]
    assert int(st["n_qtime_overflow"]) == (1 if exp["abort_tick"] is not None else 0)


def test_reference_abort_prefix_on_sweep_trace():
    """C3-recipe replications (N = 256; the stale view herds the first
    publishes onto node 0, whose queue passes ~9223 s within a few hundred
    tasks, at every load of the sweep): the continuing oracle (the engine's
    extension) and the stop-at-abort oracle (the reference) agree on every
    value the reference defines -- the decisions of all publishes up to the
    abort tick, every status, start and completion the aborted run reached --
    and on the abort point; the prefix is exactly the publishes with
    arrive_tick <= abort_tick.  The N = 16 replication never overflows."""
    b = tg.make_batch(0x5EED0003, 3, 256, 3000, sweep=True)
    s16 = tg.make_replication(0x5EED0003, 3, 16, 3000, rho=0.95)
    full = ol.run_batch(b["arrive"], b["req"], b["mips"], b["dl"], b["ul"], b["init"], threads=3)
    stop = ol.run_batch(b["arrive"], b["req"], b["mips"], b["dl"], b["ul"], b["init"], threads=3,
                        stop_at_ref_abort=True)
    big = np.iinfo(np.int64).max
    n_abort = 0
    for r in range(3):
        fs, ss = full["stats"][r], stop["stats"][r]
        assert int(fs["abort_tick"]) == int(ss["abort_tick"]) and int(fs["abort_task"]) == int(ss["abort_task"])
        ab = int(fs["abort_tick"])
        if ab == big:
            assert int(fs["n_qtime_overflow"]) == 0
            continue
        n_abort += 1
        k = int(fs["abort_task"])
        assert full["status"][r][k] == 4 and full["start"][r][k] == ab  # the popped task starts at the abort tick
        prefix = b["arrive"][r] <= ab
        assert int(ss["n_tasks"]) == int(prefix.sum())
        np.testing.assert_array_equal(stop["node"][r][prefix], full["node"][r][prefix])
        assert (stop["node"][r][~prefix] == -1).all()
        reached = stop["status"][r] != 0
        np.testing.assert_array_equal(stop["status"][r][reached], full["status"][r][reached])
        for key in ("start", "done"):
            got = stop[key][r]
            np.testing.assert_array_equal(got[got >= 0], full[key][r][got >= 0])
            assert (got[got >= 0] <= ab).all()
        assert stop["start"][r][k] == -1 and int(ss["n_qtime_overflow"]) == 1
    assert n_abort == 3  # the recipe does reach the overflow
    o16 = ol.run_batch(s16["arrive"], s16["req"], s16["mips"], s16["dl"], s16["ul"], s16["init"],
                       stop_at_ref_abort=True)
    assert int(o16["stats"][0]["abort_tick"]) == big and int(o16["stats"][0]["abort_task"]) == -1
    assert int(o16["stats"][0]["n_tasks"]) == 3000 and (o16["done"][0] >= 0).all()


def test_qtime_raw_function():
    # below 2^51 ticks the round trip is exact: raw = 1000 x the tick difference
    assert ol.qtime_raw(5 * 10**12 + 7, 10**12) == (4 * 10**12 + 7) * 1000
    assert ol.qtime_raw(2**54 + 3, 2**54 + 3) == -1000
    assert ol.qtime_raw(10**16, 0) is None  # 10^4 s: (simTime() - qst) * 1000 leaves simtime_t's range
    assert ol.ms_raw(26) == 26000 and ol.ms_raw(9224 * 10**12) is None


def test_oracle_stats_layout_is_the_abi_layout():
    from fognetsimpp_amd import _abi
    assert ol.ORC_STATS_DTYPE.descr == _abi.REP_STATS_DTYPE.descr
    assert ol.MOMENTS_DTYPE.descr == _abi.MOMENTS_DTYPE.descr


def test_v2_node_reproduces_general0_recording():
    """Weak pin against the reference's own recorded run (General-0.sca/.vec,
    older user code): the fog node (ComputeBrokerApp2) receives the 4 forwarded
    tasks at the recorded ticks and releases them at the recorded double-send
    ticks of its 10-ms timer (one release + advert per firing after the last
    arrival re-armed it, ComputeBrokerApp2.cc:219-237, 290-293); every
    forwarded task goes to node 0 (CB1 received 5 packets, CB2-5 one each)."""
    tr, d = golden_io.general0_v2_node()
    assert d["packets_received"] == {"ComputeBroker1": 5, "ComputeBroker2": 1, "ComputeBroker3": 1,
                                     "ComputeBroker4": 1, "ComputeBroker5": 1}
    o = ol.run_v2(tr["arrive"], tr["req"], tr["broker_mips"], tr["mips"], tr["dl"], tr["ul"], tr["first_adv"],
                  tr["stop"], 0.01)
    assert (o["node"][0] == 0).all()
    assert (o["status"][0] == ol.V2_ST_ACCEPTED).all()
    np.testing.assert_array_equal(o["start"][0], d["task_arrival_ticks"])
    np.testing.assert_array_equal(o["done"][0], d["release_ticks"])
    assert o["stats"]["n_released_node"][0] == 4


def hier_kat():
    """Hand-traced EXT_HIER replay (hierarchical brokers; not in the reference):
    N = 1025 nodes -> region 0 = nodes 0..1023, region 1 = node 1024; MIPS 1000,
    dl = ul = 1 ms, escalation above 1 busy second, extra hop 5 ms.
      t0 1.0 s   r0 req 3000: view all 0 -> node 0, starts 1.001, done 4.001
      t1 1.5 s   r0 req 2000: view unchanged -> node 0, queued, 4.001 .. 6.001
      t2 5.0 s   r0 req 1000: node 0's advert (4.002) says busy 2 -> region
                 minimum node 1 (busy 0) -> 1.001 + ... starts 5.001, done 6.001
      t3 5.5 s   r1 req 4000: node 1024 (busy 0), starts 5.501, done 9.501
      t4 7.0 s   r1 req 3000: node 1024 (its view still 0), queued 9.501 .. 12.501
      t5 9.6 s   r1 req 1000: node 1024's advert (9.502) says busy 3 > 1 ->
                 escalated: the parent's minimum is node 0 (its 6.002 advert: 0),
                 arriving 9.6 + 1 ms + 5 ms = 9.606, idle -> starts at once."""
    ms, sec = 10**9, 10**12
    N = 1025
    tr = dict(arrive=np.array([[sec, 1500 * ms, 5 * sec, 5500 * ms, 7 * sec, 9600 * ms]], np.int64),
              req=np.array([[3000, 2000, 1000, 4000, 3000, 1000]], np.int32), mips=np.full(N, 1000, np.int32),
              dl=np.full(N, ms, np.int64), ul=np.full(N, ms, np.int64), init=np.full(N, ms, np.int64),
              region=np.array([[0, 0, 0, 1, 1, 1]], np.int32))
    exp = dict(node=[0, 0, 1, 1024, 1024, 0], status=[5, 4, 5, 5, 4, 5],
               start=[1001 * ms, 4001 * ms, 5001 * ms, 5501 * ms, 9501 * ms, 9606 * ms],
               done=[4001 * ms, 6001 * ms, 6001 * ms, 9501 * ms, 12501 * ms, 10606 * ms])
    return tr, exp, dict(hier_threshold_s=1, hier_up_tick=5 * ms)


def test_hier_decide_known_answers():
    busy = np.array([5.0] * 1024 + [1.0] + [9.0] * 10)
    mips = np.full(busy.size, 1000, np.int32)
    assert ol.decide_hier(busy, mips, 0, 3, 1000) == (0, 1024, 1)  # region 0 all above 3 s: the parent's minimum
    busy[:1024] = 2.0
    assert ol.decide_hier(busy, mips, 0, 3, 1000) == (0, 0, 0)  # region 0, lowest index among equal busy
    assert ol.decide_hier(busy, mips, 1, 3, 1000) == (0, 1024, 0)
    assert ol.decide_hier(busy, mips, 2, 3, 1000)[0] == 1  # no region 2 (ORC_ERR_ARG)


def test_hier_replay_known_answer():
    tr, exp, kw = hier_kat()
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], policy=ol.POLICY_EXT_HIER,
                     region=tr["region"], **kw)
    assert o["stats"]["status"][0] == 0
    for k in ("node", "status", "start", "done"):
        np.testing.assert_array_equal(o[k][0], exp[k], err_msg=k)


def test_mobility_model_host_equals_device_formula():
    """fa.mobility_regions: numpy and torch (CPU) give the same regions; every
    region is valid and users hand off over time."""
    import torch
    import fognetsimpp_amd as fa
    tr = tg.make_batch(3, 2, 3000, 4000, rho=0.01)
    a = fa.mobility_regions(tr["arrive"], 3000)
    b = fa.mobility_regions(torch.from_numpy(tr["arrive"]), 3000).numpy()
    np.testing.assert_array_equal(a, b)
    assert a.min() >= 0 and a.max() < 3 and len(np.unique(a)) == 3
