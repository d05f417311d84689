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
