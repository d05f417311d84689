"""Parity of the gfx950 engine (through the C ABI) with the CPU restatement and
the hand-traced known answers.  Integer/index outputs must be bit-exact."""
import numpy as np
import pytest
import torch

import fognetsimpp_amd as fa
import golden_io
import oracle_lib as ol
import tracegen as tg
from fognetsimpp_amd import _abi
from test_oracle import c1_trace, check_fifo_invariants, hier_kat

pytestmark = pytest.mark.gpu
TPS = 10**12


def run_gpu(ctx, tr, ring_capacity=0):
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace(tr, dev)
    out = fa.run_batch(ctx, d, ring_capacity=ring_capacity)
    torch.cuda.synchronize()
    return dict(node=out.node.cpu().numpy(), status=out.status.cpu().numpy(),
                start=out.start_tick.cpu().numpy(), done=out.done_tick.cpu().numpy(),
                stats=out.rep_stats(), raw=out)


def assert_parity(tr, g, o):
    st_g, st_o = g["stats"], o["stats"]
    np.testing.assert_array_equal(st_g["status"], st_o["status"])
    for k in ("node", "status", "start", "done"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)
    for f in ("n_tasks", "n_queued", "n_started", "last_tick", "queue_min_raw", "queue_max_raw",
              "resp_min_ticks", "resp_max_ticks", "queue_sum_lo", "queue_sum_hi", "queue_sq_lo", "queue_sq_hi",
              "queue_sq_top", "n_qtime", "n_qtime_overflow", "abort_tick", "abort_task",
              "resp_sum_lo", "resp_sum_hi", "resp_sq_lo", "resp_sq_hi", "events", "max_pending"):
        np.testing.assert_array_equal(st_g[f], st_o[f], err_msg=f)


# ------------------------------------------------------------------ decision core

@pytest.mark.parametrize("case", golden_io.decide_cases(), ids=lambda c: c[0])
def test_sendPubAck_known_answers(ctx, case):
    name, busy, mips, req, node, err = case
    broker = fa.BrokerBaseApp3(ctx)
    if err is not None:
        with pytest.raises(fa.FognetError) as e:
            broker.sendPubAck(busy, mips, req)
        assert e.value.code == err
    else:
        assert broker.sendPubAck(busy, mips, req) == node


def test_decide_batch_matches_oracle(ctx):
    rng = np.random.default_rng(5)
    for n in (1, 3, 64, 65, 256, 1000):
        m = 2000
        busy = rng.integers(0, 6, size=(m, n)).astype(np.float64) + rng.choice([0.0, 0.5, 1e-16], size=(m, n))
        busy[rng.random((m, n)) < 0.01] = np.nan
        mips = rng.integers(1, 3000, size=(m, n)).astype(np.int32)
        mips[rng.random(m) < 0.05, 0] = 0
        req = rng.integers(-5000, 70000, size=m).astype(np.int32)
        dev = torch.device("cuda", ctx.device)
        node, status = fa.BrokerBaseApp3(ctx).sendPubAck_batch(
            torch.from_numpy(busy).to(dev), torch.from_numpy(mips).to(dev), torch.from_numpy(req).to(dev))
        node, status = node.cpu().numpy(), status.cpu().numpy()
        for q in range(m):
            rc, k = ol.decide_v3(busy[q], mips[q], int(req[q]))
            assert status[q] == rc, (n, q)
            if rc == 0:
                assert node[q] == k, (n, q)


def test_decide_window_and_large_views_match_oracle(ctx):
    """fognet_decide_window (one view, m requests) and fognet_decide on views past
    the kernel-argument size (mapped host memory) against the reference scan."""
    rng = np.random.default_rng(8)
    broker = fa.BrokerBaseApp3(ctx)
    for n in (1, 4, 64, 256, 257, 3000):
        for _ in range(3):
            busy = rng.integers(0, 5, size=n).astype(np.float64) + rng.choice([0.0, 0.5, 1e-16, np.nan], size=n)
            mips = rng.integers(1, 3000, size=n).astype(np.int32)
            reqs = rng.integers(0, 10**6, size=50).astype(np.int32)
            got = broker.sendPubAck_window(busy, mips, reqs)
            want = [ol.decide_v3(busy, mips, int(q))[1] for q in reqs]
            np.testing.assert_array_equal(got, want)
            assert broker.sendPubAck(busy, mips, int(reqs[0])) == want[0]


def test_decide_latency(ctx):
    """Per-call latency of the scalar drop-in (one launch + one synchronisation,
    no copies) and of a window of 64 publishes; written to
    gpurun_out/decide_latency.json.  The bound only catches regressions."""
    import json
    import os
    import time
    broker = fa.BrokerBaseApp3(ctx)
    res = {}
    for n in (5, 256, 10_000):
        busy = np.arange(n, dtype=np.float64)[::-1].copy()
        mips = np.full(n, 1000, np.int32)
        for _ in range(50):
            broker.sendPubAck(busy, mips, 4000)
        k = 2000
        t0 = time.perf_counter()
        for _ in range(k):
            broker.sendPubAck(busy, mips, 4000)
        res[f"decide_n{n}_us"] = (time.perf_counter() - t0) / k * 1e6
        reqs = np.full(64, 4000, np.int32)
        t0 = time.perf_counter()
        for _ in range(200):
            broker.sendPubAck_window(busy, mips, reqs)
        res[f"window64_n{n}_us"] = (time.perf_counter() - t0) / 200 * 1e6
    os.makedirs(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out"), exist_ok=True)
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out",
                           "decide_latency.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(res)
    assert res["decide_n5_us"] < 2000


@pytest.mark.parametrize("case", golden_io.decide_v2_cases(), ids=lambda c: c[0])
def test_v2_sendPubAck_known_answers(ctx, case):
    name, mips, local, req, action, node = case
    assert fa.BrokerBaseApp2(ctx).sendPubAck(mips, local, req) == (action, node)


def test_decide_v2_batch_matches_oracle(ctx):
    rng = np.random.default_rng(17)
    dev = torch.device("cuda", ctx.device)
    for n in (0, 1, 2, 5, 64, 65, 300, 5000):
        m = 1500
        mips = rng.choice([0, 500, 999, 1000, 1001, 2000, 4000], size=(m, max(n, 1))).astype(np.int32)[:, :n]
        mips = np.ascontiguousarray(mips)
        local = rng.integers(-100, 3000, size=m).astype(np.int32)
        req = rng.integers(0, 4500, size=m).astype(np.int32)
        act, node = fa.BrokerBaseApp2(ctx).sendPubAck_batch(
            torch.from_numpy(mips).to(dev), torch.from_numpy(local).to(dev), torch.from_numpy(req).to(dev))
        act, node = act.cpu().numpy(), node.cpu().numpy()
        for q in range(m):
            assert (act[q], node[q]) == ol.decide_v2(mips[q], local[q], req[q]), (n, q)


# ------------------------------------------------------------------ replay engine

@pytest.mark.parametrize("case", golden_io.replay_cases(), ids=lambda c: c[0])
def test_replay_known_answers(ctx, case):
    name, tr, exp = case
    g = run_gpu(ctx, tr)
    assert g["stats"]["status"][0] == 0
    np.testing.assert_array_equal(g["node"][0], exp["node"])
    np.testing.assert_array_equal(g["status"][0], exp["status"])
    np.testing.assert_array_equal(g["start"][0], exp["start"])
    np.testing.assert_array_equal(g["done"][0], exp["done"])
    assert g["stats"]["n_queued"][0] == exp["n_queued"]
    assert g["stats"]["n_started"][0] == exp["n_started"]


def test_c1_example_run(ctx):
    tr = c1_trace()
    g = run_gpu(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"])
    assert_parity(tr, g, o)
    assert (g["node"] == 0).all()


def test_c2_trace_replay_bit_exact(ctx):
    """Config C2: 1 replication x 10,000 tasks x 64 nodes (BASELINE.json configs[1])."""
    tr = tg.make_batch(0x5EED0001, 1, 64, 10000)
    g = run_gpu(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"])
    assert_parity(tr, g, o)


@pytest.mark.parametrize("N", [1, 5, 63, 64, 100, 128, 200, 256])
def test_node_counts(ctx, N):
    tr = tg.make_batch(1000 + N, 3, N, 1500, rho=0.9)
    g = run_gpu(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=3)
    assert_parity(tr, g, o)


def test_policy_sweep_sample(ctx):
    """C3 recipe (rho x latency-scale sweep) at reduced T for the oracle."""
    tr = tg.make_batch(0x5EED0003, 18, 256, 4000, sweep=True)
    g = run_gpu(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8)
    assert_parity(tr, g, o)


def tie_heavy(seed, R, N, T):
    """Coarse ticks so arrivals, completions and adverts collide: latencies and
    gaps are small multiples of a base, service times often 0, and some
    downlinks are >= whole seconds so the arrival-first rule is exercised."""
    rng = np.random.default_rng(seed)
    base = 10**11
    mips = rng.choice([1000, 2000, 500], size=(R, N)).astype(np.int32)
    dl = rng.choice([0, base, 2 * base, 10 * base, 20 * base, 30 * base], size=(R, N)).astype(np.int64)
    ul = rng.choice([0, base, 3 * base], size=(R, N)).astype(np.int64)
    init = ul + rng.integers(0, 3, size=(R, N)) * base
    start = init.max(axis=1, keepdims=True) + base
    gaps = rng.choice([0, 0, base, 5 * base, 10 * base], size=(R, T)).astype(np.int64)
    arrive = start + np.cumsum(gaps, axis=1)
    req = rng.choice([0, 400, 999, 1000, 1500, 2000, 3000], size=(R, T)).astype(np.int32)
    return dict(arrive=arrive, req=req, mips=mips, dl=dl, ul=ul, init=init)


@pytest.mark.parametrize("seed", range(6))
def test_tie_heavy(ctx, seed):
    tr = tie_heavy(seed, 8, 1 + 37 * seed, 2000)
    g = run_gpu(ctx, tr, ring_capacity=4096)  # N = 1 is overloaded: up to ~1500 pending
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8)
    assert_parity(tr, g, o)


def test_shared_node_params_and_empty_trace(ctx):
    tr = tg.make_replication(3, 0, 32, 700)
    batch = dict(arrive=np.stack([tr["arrive"]] * 2), req=np.stack([tr["req"], tr["req"][::-1].copy()]),
                 mips=tr["mips"], dl=tr["dl"], ul=tr["ul"], init=tr["init"])
    g = run_gpu(ctx, batch)
    o = ol.run_batch(batch["arrive"], batch["req"], batch["mips"], batch["dl"], batch["ul"], batch["init"])
    assert_parity(batch, g, o)
    empty = dict(batch, arrive=np.zeros((2, 0), np.int64), req=np.zeros((2, 0), np.int32))
    g = run_gpu(ctx, empty)
    assert (g["stats"]["status"] == 0).all() and (g["stats"]["n_tasks"] == 0).all()


@pytest.mark.parametrize("ring", [4, 16, 4096])
def test_ring_capacity_exceeded(ctx, ring):
    """An overloaded trace (queues grow without bound) completes whatever the
    ring capacity: replications past it are replayed by the wide kernel inside
    the same call.  A mixed batch (3 overloaded replications among light ones),
    bit-exact against the oracle, histogram included."""
    over = tg.make_batch(11, 3, 4, 2000, rho=3.0)
    light = tg.make_batch(12, 5, 4, 2000, rho=0.3)
    tr = {k: np.concatenate([light[k][:2], over[k], light[k][2:]]) for k in over}
    g = run_gpu_full(ctx, tr, ring_capacity=ring)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8, hist=True)
    assert (g["stats"]["status"] == 0).all()
    assert g["stats"]["max_pending"].max() > ring or ring == 4096
    assert_parity(tr, g, o)
    np.testing.assert_array_equal(g["hist"], o["hist"].sum(axis=0))


def test_service_past_register_kernel_bound(ctx):
    """Service times past the register kernel's bound (2^24 / ring capacity s,
    8191 s at the default ring) up to the wide kernel's 65535 s: handed over,
    same results as the oracle; the separate statistics pass agrees."""
    tr = tg.make_batch(13, 4, 8, 600, rho=0.5)
    tr = {k: v.copy() for k, v in tr.items()}
    tr["req"][1, 10] = 9000 * int(tr["mips"][1, 0])  # 9000 s on node 0
    tr["req"][3, ::50] = 60000 * 1000  # up to 60,000 s
    g = run_gpu_full(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=4, hist=True)
    assert (g["stats"]["status"] == 0).all()
    assert_parity(tr, g, o)
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace(tr, dev)
    sep = fa.run_batch(ctx, d, stage="replay")
    fa.run_batch(ctx, d, out=sep, stage="stats")
    torch.cuda.synchronize()
    assert sep.rep_stats().tobytes() == g["stats"].tobytes()


@pytest.mark.parametrize("N", [8, 300])  # handed over by the register kernel / the wide kernel
def test_service_times_past_2_16_seconds(ctx, N):
    """The reference accepts any int / int service time (ComputeBrokerApp3.cc:276):
    tasks of 65,536 s to 1,000,000 s (11.6 days), runs of them on one node, all
    completing within the engine's 2^61-tick range, match the oracle; a task
    completing past it is refused (FOGNET_ERR_ARG) by both."""
    tr = tg.make_batch(29, 3, N, 500, rho=0.5)
    tr = {k: v.copy() for k, v in tr.items()}
    m0 = int(tr["mips"][0, 0])
    tr["req"][0, 40] = 65536 * m0            # exactly 2^16 s on node 0 (ties -> node 0 decides it)
    tr["req"][1, 10:14] = 300_000 * 1000     # a run of 300,000 s tasks
    tr["req"][1, 200] = 1_000_000 * 1000     # 11.6 days
    tr["req"][2, ::97] = 2**31 - 1           # up to 2^31 - 1 s: completes past 2^61 ticks
    g = run_gpu_full(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=3, hist=True)
    assert list(g["stats"]["status"][:2]) == [0, 0] and g["stats"]["status"][2] == _abi.FOGNET_ERR_ARG
    assert o["stats"]["status"][2] == 1  # ORC_ERR_ARG
    two = {k: (v[:2] if k in ("node", "status", "start", "done", "stats") else v) for k, v in g.items()}
    ref = {k: (v[:2] if k in ("node", "status", "start", "done", "stats") else v) for k, v in o.items()}
    assert_parity(tr, two, ref)
    assert (g["done"][1] - g["start"][1]).max() >= 250_000 * TPS  # (the 1e6-MIPS task ran at 1000-4000 MIPS)


def test_saturated_advertised_busy(ctx):
    """A node that advertises 2^32 s or more of queued service (2,200 tasks of
    2e6 s queued on it that its crash keeps from ever completing, node-down
    extension): the
    32-bit view saturates, the node is never the minimum, decisions equal the
    oracle's; with one node the minimum itself is saturated and the replication
    is refused (FOGNET_ERR_CAPACITY) instead of guessing the order."""
    MS = 10**9
    res = {}
    for N in (2, 1):
        mips = np.full(N, 1, np.int32)  # service = MIPSRequired seconds
        dl = np.full(N, MS, np.int64)
        ul = np.full(N, MS, np.int64)
        init = np.full(N, MS, np.int64)
        q = 2200  # queued tasks of 2,000,000 s each: 4.4e9 s > 2^32 s advertised
        arrive = np.concatenate([[50 * MS], 50 * MS + 1 + np.arange(q), [5 * TPS, 6 * TPS, 7 * TPS]]).astype(np.int64)
        req = np.concatenate([[1], np.full(q, 2_000_000), [1, 1, 1]]).astype(np.int32)
        down = np.full(N, np.iinfo(np.int64).max, np.int64)
        down[0] = 51 * MS + TPS + 1  # just after task 0 (1 s) completes and advertises
        tr = dict(arrive=arrive[None], req=req[None], mips=mips, dl=dl, ul=ul, init=init, down=down)
        dev = torch.device("cuda", ctx.device)
        out = fa.run_batch(ctx, fa.as_device_trace(tr, dev))
        torch.cuda.synchronize()
        st = out.rep_stats()[0]
        o = ol.run_batch(arrive[None], req[None], mips, dl, ul, init, down=down)
        res[N] = (st, out.node[0].cpu().numpy(), o)
    st, node, o = res[2]
    assert st["status"] == 0
    np.testing.assert_array_equal(node, o["node"][0])
    assert list(node[-3:]) == [1, 1, 1]  # node 0 advertised 4.4e9 s of work
    assert res[1][0]["status"] == _abi.FOGNET_ERR_CAPACITY


def test_compact_ring_bounds_hand_over(ctx):
    """The register kernel's 8-B ring entries (internal.h RingWord: arrival
    < 2^56 ticks, service < 256 s): a replication with a longer service time or
    a later arrival is handed to the wide kernel inside the same call; mixed
    with replications that stay, every record is bit-exact against the oracle."""
    tr = tg.make_batch(14, 5, 8, 800, rho=0.8)
    tr = {k: v.copy() for k, v in tr.items()}
    tr["req"][1, 30] = 300 * int(tr["mips"][1].max())  # >= 300 s on any node
    tr["req"][3, 100:140] = 256 * int(tr["mips"][3].max())  # 256 s: one past the entry's 8 bits
    tr["arrive"][2] += 1 << 57  # past the entry's tick range, within the kernel's 2^61
    g = run_gpu_full(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=4, hist=True)
    assert (g["stats"]["status"] == 0).all()
    assert_parity(tr, g, o)
    np.testing.assert_array_equal(g["hist"], o["hist"].sum(axis=0))


@pytest.mark.parametrize("N", [16, 300])  # register-resident and wide kernel
@pytest.mark.parametrize("bad",["unsorted", "neg_req", "mips0", "late_advert", "early_advert_send", "huge_service"])
def test_precondition_errors(ctx, bad, N):
    tr = tg.make_batch(5, 2, N, 300)
    tr = {k: v.copy() for k, v in tr.items()}
    if bad == "unsorted":
        tr["arrive"][1, 100] = tr["arrive"][1, 99] - 1
    elif bad == "neg_req":
        tr["req"][1, 5] = -1
    elif bad == "mips0":
        tr["mips"][1, 3] = 0
    elif bad == "late_advert":
        tr["init"][1, 7] = tr["arrive"][1, 0]
    elif bad == "early_advert_send":
        tr["init"][1, 7] = tr["ul"][1, 7] - 1
    elif bad == "huge_service":
        tr["mips"][1, :] = 1
        tr["req"][1, :] = 2**31 - 1
    g = run_gpu(ctx, tr)
    assert g["stats"]["status"][0] == 0
    assert g["stats"]["status"][1] == _abi.FOGNET_ERR_ARG


def test_unsupported_sizes(ctx):
    """The wide kernel's limits: N <= 2^20 for the flat policies (its active-group mask words),
    N <= 65,536 for EXT_HIER (64 regions of 1,024 nodes); refused loudly above."""
    tr = tg.make_batch(5, 1, (1 << 20) + 1, 4)
    with pytest.raises(fa.FognetError) as e:
        run_gpu(ctx, tr)
    assert e.value.code == _abi.FOGNET_ERR_UNSUPPORTED
    tr = tg.make_batch(5, 1, 65537, 10)
    tr["region"] = np.zeros((1, 10), np.int32)
    with pytest.raises(fa.FognetError) as e:
        run_gpu_full(ctx, tr, policy="EXT_HIER")
    assert e.value.code == _abi.FOGNET_ERR_UNSUPPORTED


# ------------------------------------------------------------------ generator + stats

def test_device_tracegen_matches_host_recipe(ctx):
    R, T, N = 12, 3000, 256
    mg, sc = fa.sweep_params(np.arange(R), N)
    d = fa.generate_trace(ctx, 0x5EED0003, R, T, N, mg, sc)
    torch.cuda.synchronize()
    for r in range(R):
        h = tg.make_replication(0x5EED0003, r, N, T, rho=(0.5, 0.8, 0.95)[r % 3], lat_scale=int(sc[r]),
                                mean_gap_ticks=float(mg[r]))
        for k in ("arrive", "req", "mips", "dl", "ul", "init"):
            np.testing.assert_array_equal(d[k][r].cpu().numpy(), h[k], err_msg=f"{k} r={r}")


def test_device_tracegen_sharding_offset(ctx):
    N, T = 64, 500
    mg, sc = fa.sweep_params(np.arange(8), N)
    full = fa.generate_trace(ctx, 9, 8, T, N, mg, sc)
    part = fa.generate_trace(ctx, 9, 3, T, N, mg[5:], sc[5:], r0=5)
    torch.cuda.synchronize()
    for k in ("arrive", "req", "dl"):
        assert torch.equal(full[k][5:], part[k])


def job_from_reps(st):
    """Exact host reduction of rep stats (test-side), for comparison with the device."""
    ok = st[st["status"] == 0]
    def u128(lo, hi, top=None):
        return sum(int(a) | (int(b) << 64) | ((int(top[i]) << 128) if top is not None else 0)
                   for i, (a, b) in enumerate(zip(lo, hi)))
    def s128(lo, hi):  # two's complement 128-bit values, summed as Python ints, returned mod 2^192
        v = sum((x - (1 << 128) if x >> 127 else x) for x in (int(a) | (int(b) << 64) for a, b in zip(lo, hi)))
        return v % (1 << 192)
    return dict(n_reps=len(st), n_failed=int((st["status"] != 0).sum()), n_tasks=int(ok["n_tasks"].sum()),
                n_queued=int(ok["n_queued"].sum()), queue_sum=s128(ok["queue_sum_lo"], ok["queue_sum_hi"]),
                queue_sq=u128(ok["queue_sq_lo"], ok["queue_sq_hi"], ok["queue_sq_top"]),
                resp_sq=u128(ok["resp_sq_lo"], ok["resp_sq_hi"]),
                resp_max=int(ok["resp_max_ticks"].max()), max_pending=int(ok["max_pending"].max()))


def test_reduce_stats_exact(ctx):
    tr = tg.make_batch(21, 20, 64, 2000, sweep=True)
    tr["mips"][3, 0] = 0  # one failed replication
    g = run_gpu(ctx, tr)
    job = fa.reduce_stats(ctx, g["raw"].stats, 20)
    ref = job_from_reps(g["stats"])
    u192 = lambda a: int(a[0]) | (int(a[1]) << 64) | (int(a[2]) << 128)
    assert int(job["n_reps"]) == 20 and int(job["n_failed"]) == 1 == ref["n_failed"]
    assert int(job["n_tasks"]) == ref["n_tasks"] and int(job["n_queued"]) == ref["n_queued"]
    assert u192(job["queue_sum"]) == ref["queue_sum"] and u192(job["queue_sq"]) == ref["queue_sq"]
    assert u192(job["resp_sq"]) == ref["resp_sq"]
    assert int(job["resp_max_ticks"]) == ref["resp_max"] and int(job["max_pending"]) == ref["max_pending"]
    halves = [fa.reduce_stats(ctx, g["raw"].stats[: 7 * _abi.REP_STATS_DTYPE.itemsize], 7),
              fa.reduce_stats(ctx, g["raw"].stats[7 * _abi.REP_STATS_DTYPE.itemsize:], 13)]
    assert fa.merge_job_stats(halves).tobytes() == job.tobytes()


def test_reduce_stats_multi_block(ctx):
    """Above 4,096 records the job reduction runs in blocks plus a merge
    (generated replays: C4's million-replication launches); the integer
    fields equal the exact host reduction."""
    R, T, N = 9000, 64, 8
    mg, sc = fa.sweep_params(np.arange(R), N)
    out = fa.run_generated(ctx, 7, R, T, N, mg, sc, hist=False)
    job = fa.reduce_stats(ctx, out.stats, R)
    st = out.rep_stats()
    ref = job_from_reps(st)
    u192 = lambda a: int(a[0]) | (int(a[1]) << 64) | (int(a[2]) << 128)
    assert int(job["n_reps"]) == R and int(job["n_failed"]) == 0 == ref["n_failed"]
    assert int(job["n_tasks"]) == ref["n_tasks"] == R * T and int(job["n_queued"]) == ref["n_queued"]
    assert u192(job["queue_sum"]) == ref["queue_sum"] and u192(job["queue_sq"]) == ref["queue_sq"]
    assert u192(job["resp_sq"]) == ref["resp_sq"]
    assert int(job["resp_max_ticks"]) == ref["resp_max"] and int(job["max_pending"]) == ref["max_pending"]
    assert int(job["n_qtime"]) == int(st["n_qtime"].sum())


def test_full_size_sweep_properties(ctx):
    """C3 shape at reduced R: R=256 x T=100k x N=256, checked through
    size-independent properties on the device (FIFO recurrence per node,
    service times, statuses) plus one replication against the oracle."""
    R, T, N = 256, 100_000, 256
    dev = torch.device("cuda", ctx.device)
    mg, sc = fa.sweep_params(np.arange(R), N)
    d = fa.generate_trace(ctx, 0x5EED0003, R, T, N, mg, sc)
    out = fa.run_batch(ctx, d)
    torch.cuda.synchronize()
    st = out.rep_stats()
    assert (st["status"] == 0).all() and (st["n_tasks"] == T).all()
    node = out.node.long()
    mips = torch.gather(d["mips"].long(), 1, node)
    dl = torch.gather(d["dl"], 1, node)
    S = d["req"].long() // mips
    a = d["arrive"] + dl
    assert torch.equal(out.done_tick - out.start_tick, S * TPS)
    assert bool((out.start_tick >= a).all())
    assert bool(((out.status == 5) <= (out.start_tick == a)).all())
    # per node FIFO: start = max(a, previous done on the same node)
    key = node * T + torch.arange(T, device=dev).unsqueeze(0)
    order = torch.argsort(key, dim=1)
    n_s, a_s = torch.gather(node, 1, order), torch.gather(a, 1, order)
    s_s, d_s = torch.gather(out.start_tick, 1, order), torch.gather(out.done_tick, 1, order)
    prev = torch.cat([torch.full((R, 1), -2**62, device=dev, dtype=torch.int64), d_s[:, :-1]], 1)
    same = torch.cat([torch.zeros((R, 1), device=dev, dtype=torch.bool), n_s[:, 1:] == n_s[:, :-1]], 1)
    prev = torch.where(same, prev, torch.full_like(prev, -2**62))
    assert torch.equal(s_s, torch.maximum(a_s, prev))
    # one full replication bit-exact against the oracle
    r = 1
    h = {k: d[k][r].cpu().numpy() for k in ("arrive", "req", "mips", "dl", "ul", "init")}
    o = ol.run_batch(h["arrive"], h["req"], h["mips"], h["dl"], h["ul"], h["init"])
    np.testing.assert_array_equal(out.node[r].cpu().numpy(), o["node"][0])
    np.testing.assert_array_equal(out.done_tick[r].cpu().numpy(), o["done"][0])
    assert st[r].tobytes() == o["stats"][0].tobytes()


@pytest.mark.parametrize("kernel", ["register", "wide", "inloop"])
@pytest.mark.parametrize("case", golden_io.qtime_cases(), ids=lambda c: c[0])
def test_qtime_known_answers_gpu(ctx, monkeypatch, case, kernel):
    """queueTime as the reference emits it (tests/golden/kat_qtime.json): the
    queueStartTime double round trip above 2^53 ticks, a negative value, the
    simtime_t overflow and the reference's abort point (the earliest
    overflowing emission, two_nodes: not the lowest index); both replay
    kernels and the in-loop statistics, fused statistics and histogram."""
    if kernel == "wide":
        monkeypatch.setenv("FOGNET_REPLAY_KERNEL", "wide")
    if kernel == "inloop":
        monkeypatch.setenv("FOGNET_REPLAY_STATS", "inloop")
    name, tr, exp = case
    dev = torch.device("cuda", ctx.device)
    out = fa.run_batch(ctx, fa.as_device_trace(tr, dev), hist=True)
    torch.cuda.synchronize()
    for k, g in (("node", out.node), ("status", out.status), ("start", out.start_tick), ("done", out.done_tick)):
        np.testing.assert_array_equal(g[0].cpu().numpy(), exp[k], err_msg=k)
    golden_io.check_qtime_record(out.rep_stats()[0], exp)
    assert int(out.hist[0].sum()) == exp["n_qtime"]


@pytest.mark.parametrize("kernel", ["register", "wide", "inloop", "separate", "generated"])
def test_reference_abort_point_and_prefix(ctx, monkeypatch, kernel):
    """The reference ends a run at its first overflowing queueTime emission
    (ComputeBrokerApp3.cc:238, no handler up to :84-86).  On C3-recipe
    replications (N = 256: the stale view herds the first publishes onto node 0
    and its queue passes ~9223 s within a few hundred tasks) the device reports
    the oracle's abort point, its outputs equal the stop-at-abort oracle (the
    reference) on every value that run defines, and FOGNET_FLAG_REF_ABORT turns
    those replications into FOGNET_REF_ABORTED (counted as failed by the job
    reduction); the N = 16 replication completes in the reference too."""
    if kernel == "wide":
        monkeypatch.setenv("FOGNET_REPLAY_KERNEL", "wide")
    if kernel == "inloop":
        monkeypatch.setenv("FOGNET_REPLAY_STATS", "inloop")
    T, N, R = 3000, 256, 6
    dev = torch.device("cuda", ctx.device)
    mg, sc = fa.sweep_params(np.arange(R), N)
    d = fa.generate_trace(ctx, 0x5EED0003, R, T, N, mg, sc)
    tr = {k: v for k, v in d.items() if not k.startswith("_")}
    h = {k: tr[k].cpu().numpy() for k in tr}
    big = np.iinfo(np.int64).max
    full = ol.run_batch(h["arrive"], h["req"], h["mips"], h["dl"], h["ul"], h["init"], threads=6)
    stop = ol.run_batch(h["arrive"], h["req"], h["mips"], h["dl"], h["ul"], h["init"], threads=6,
                        stop_at_ref_abort=True)
    assert (full["stats"]["abort_tick"] != big).all()
    if kernel == "generated":  # statistics-only, trace generated in the kernel: the records
        g = fa.run_generated(ctx, 0x5EED0003, R, T, N, mg, sc, hist=False)
        torch.cuda.synchronize()
        assert g.rep_stats().tobytes() == full["stats"].tobytes()
        return
    if kernel == "separate":  # fognet_replay_dev, then fognet_rep_stats_dev
        out = fa.run_batch(ctx, tr, stage="replay")
        fa.run_batch(ctx, tr, out=out, stage="stats")
    else:
        out = fa.run_batch(ctx, tr)
    torch.cuda.synchronize()
    st = out.rep_stats()
    assert st.tobytes() == full["stats"].tobytes()
    g = {k: getattr(out, a).cpu().numpy() for k, a in (("node", "node"), ("status", "status"),
                                                      ("start", "start_tick"), ("done", "done_tick"))}
    for r in range(R):
        ab = int(st[r]["abort_tick"])
        prefix = h["arrive"][r] <= ab
        np.testing.assert_array_equal(g["node"][r][prefix], stop["node"][r][prefix])
        reached = stop["status"][r] != 0
        np.testing.assert_array_equal(g["status"][r][reached], stop["status"][r][reached])
        for k in ("start", "done"):
            m = stop[k][r] >= 0
            np.testing.assert_array_equal(g[k][r][m], stop[k][r][m])
    # the reference mode: aborted replications fail, with outputs still written in full
    out2 = fa.run_batch(ctx, tr, ref_abort=True)
    torch.cuda.synchronize()
    st2 = out2.rep_stats()
    assert (st2["status"] == _abi.FOGNET_REF_ABORTED).all()
    assert torch.equal(out2.done_tick, out.done_tick) and torch.equal(out2.node, out.node)
    job = fa.reduce_stats(ctx, out2.stats, R)
    # failed records contribute nothing else, but the abort count includes them
    assert int(job["n_failed"]) == R and int(job["n_ref_aborted"]) == R
    job = fa.reduce_stats(ctx, out.stats, R)
    assert int(job["n_failed"]) == 0 and int(job["n_ref_aborted"]) == R
    # a replication the reference completes: no abort point, status OK under the flag
    one = tg.make_replication(0x5EED0003, 3, 16, T, rho=0.95)
    o16 = fa.run_batch(ctx, fa.as_device_trace({k: v[None] if k in ("arrive", "req") else v for k, v in one.items()},
                                               dev), ref_abort=True)
    torch.cuda.synchronize()
    s16 = o16.rep_stats()[0]
    assert s16["status"] == 0 and int(s16["abort_tick"]) == big and int(s16["abort_task"]) == -1


def _sharded_sample(ctx, seed, R_total, T, N, reps, ring, params):
    """Replications `reps` (global indices) of a device-generated sweep job,
    generated exactly as the bench's shards generate them (r0 = global index)."""
    dev = torch.device("cuda", ctx.device)
    outs = []
    for r in reps:
        mg, sc = params(np.array([r]), N)
        d = fa.generate_trace(ctx, seed, 1, T, N, mg, sc, r0=int(r))
        o = fa.run_batch(ctx, d, ring_capacity=ring, hist=False)
        outs.append((d, o))
    torch.cuda.synchronize()
    return outs


def test_c3_full_length_replications_bit_exact(ctx):
    """Config C3 at its full length (T = 100,000, N = 256, seed 0x5EED0003,
    ring 2048 as bench.py): 24 replications spread over the 4096-replication
    sweep (every rho x latency class), all outputs and records bit-exact
    against the oracle."""
    T, N = 100_000, 256
    reps = list(range(9)) + [1000, 1001, 1002, 2047, 2048, 2049, 3000, 3001, 3002, 4087, 4088, 4089, 4093, 4094, 4095]
    outs = _sharded_sample(ctx, 0x5EED0003, 4096, T, N, reps, 2048, fa.sweep_params)
    for r, (d, o) in zip(reps, outs):
        h = {k: d[k][0].cpu().numpy() for k in ("arrive", "req", "mips", "dl", "ul", "init")}
        ref = ol.run_batch(h["arrive"], h["req"], h["mips"], h["dl"], h["ul"], h["init"])
        for k_gpu, k_ref in (("node", "node"), ("status", "status"), ("start_tick", "start"), ("done_tick", "done")):
            np.testing.assert_array_equal(getattr(o, k_gpu)[0].cpu().numpy(), ref[k_ref][0], err_msg=f"{k_gpu} r={r}")
        assert o.rep_stats()[0].tobytes() == ref["stats"][0].tobytes(), f"stats r={r}"


def test_c4_workload_shape_matches_oracle(ctx):
    """Config C4 (BASELINE.json configs[3]): T = 10,000, N = 256, seed
    0x5EED0004, the sweep recipe, replications drawn from the whole
    1,000,000-replication job (as the 8 GPU shards generate them), in one
    batch of 256 like a bench block; every output and record against the oracle."""
    T, N = 10_000, 256
    rng = np.random.default_rng(4)
    reps = np.sort(np.concatenate([np.arange(128), rng.choice(np.arange(128, 1_000_000), 128, replace=False)]))
    dev = torch.device("cuda", ctx.device)
    d = fa.allocate_trace(len(reps), T, N, dev)
    for i, r in enumerate(reps):  # generate each at its global index, then replay them as one block
        mg, sc = fa.sweep_params(np.array([r]), N)
        one = fa.generate_trace(ctx, 0x5EED0004, 1, T, N, mg, sc, r0=int(r))
        for k in ("arrive", "req", "mips", "dl", "ul", "init"):
            d[k][i].copy_(one[k][0])
    tr = {k: v for k, v in d.items() if not k.startswith("_")}
    out = fa.run_batch(ctx, tr, ring_capacity=2048, hist=True)
    torch.cuda.synchronize()
    h = {k: tr[k].cpu().numpy() for k in tr}
    ref = ol.run_batch(h["arrive"], h["req"], h["mips"], h["dl"], h["ul"], h["init"], threads=8, hist=True)
    for k_gpu, k_ref in (("node", "node"), ("status", "status"), ("start_tick", "start"), ("done_tick", "done")):
        np.testing.assert_array_equal(getattr(out, k_gpu).cpu().numpy(), ref[k_ref], err_msg=k_gpu)
    assert out.rep_stats().tobytes() == ref["stats"].tobytes()
    np.testing.assert_array_equal(out.hist.cpu().numpy(), ref["hist"].sum(axis=0))


@pytest.mark.parametrize("kind", ["register", "wide", "handover", "ext_lat", "short"])
def test_stats_only_equals_full_outputs(ctx, monkeypatch, kind):
    """Statistics-only replays (no per-task arrays: the statistics are
    accumulated while the replay runs, C4's mode) give the same records and
    histogram as the replay with full outputs."""
    ring, policy = 0, "REF_V3"
    if kind == "wide":
        monkeypatch.setenv("FOGNET_REPLAY_KERNEL", "wide")
    tr = tg.make_batch(41, 6, 64, 5000, sweep=True)
    if kind == "handover":
        ring = 4
    if kind == "ext_lat":
        policy = "EXT_LAT"
    if kind == "short":  # T below one flush window and not a multiple of 64
        tr = tg.make_batch(42, 5, 17, 333, rho=0.9)
    pb, pi = fa.power_model(tr["mips"])
    tr = dict(tr, p_busy=pb, p_idle=pi)
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace(tr, dev)
    R, T = tr["arrive"].shape
    full = fa.run_batch(ctx, d, ring_capacity=ring, policy=policy, hist=True)
    so = fa.allocate_outputs(R, T, dev, hist=True, per_task=False)
    fa.run_batch(ctx, d, out=so, ring_capacity=ring, policy=policy)
    torch.cuda.synchronize()
    assert (full.rep_stats()["status"] == 0).all()
    assert so.rep_stats().tobytes() == full.rep_stats().tobytes()
    assert torch.equal(so.hist, full.hist)


@pytest.mark.parametrize("kind", ["c4_first", "c4_last", "n64", "n100", "ext_lat", "handover", "wide", "energy"])
def test_generated_equals_materialized(ctx, monkeypatch, kind):
    """Generated replays (fognet_run_generated_dev: trace chunks and node
    parameters computed inside the replay kernel, statistics only: C4's mode,
    SURVEY.md §8(d)) give the records, histograms and energy of
    fognet_gen_trace_dev + fognet_run_batch_dev on the same replications
    (which test_c4_workload_shape_matches_oracle checks against the oracle)."""
    seed, R, T, N, r0, ring, policy = 0x5EED0004, 64, 10_000, 256, 0, 0, "REF_V3"
    if kind == "c4_last":  # the last block of the 1,000,000-replication job
        r0 = 1_000_000 - R
    if kind == "n64":
        N, T = 64, 3000
    if kind == "n100":
        R, N, T = 16, 100, 4001
    if kind == "ext_lat":
        policy, T = "EXT_LAT", 3000
    if kind == "handover":  # every replication overflows a 4-entry ring: the wide kernel generates too
        ring, T = 4, 3000
    if kind == "wide":
        monkeypatch.setenv("FOGNET_REPLAY_KERNEL", "wide")
        T = 3000
    dev = torch.device("cuda", ctx.device)
    mg, sc = fa.sweep_params(np.arange(r0, r0 + R), N)
    d = {k: v for k, v in fa.generate_trace(ctx, seed, R, T, N, mg, sc, r0=r0).items() if not k.startswith("_")}
    power = None
    if kind == "energy":
        pb, pi = fa.power_model(1000 * (1 + np.arange(N) % 4))
        power = tuple(torch.from_numpy(np.tile(x, (R, 1))).to(dev) for x in (pb, pi))
        d = dict(d, p_busy=power[0], p_idle=power[1])
    full = fa.run_batch(ctx, d, ring_capacity=ring, policy=policy, hist=True)
    gen = fa.run_generated(ctx, seed, R, T, N, mg, sc, r0=r0, ring_capacity=ring, policy=policy, power=power,
                           hist=True, energy=power is not None)
    torch.cuda.synchronize()
    st = full.rep_stats()
    assert (st["status"] == 0).all() and (st["n_tasks"] == T).all()
    if kind == "handover":
        assert (st["max_pending"] > 4).all()
    assert gen.rep_stats().tobytes() == st.tobytes()
    assert torch.equal(gen.hist, full.hist)
    if power is not None:
        assert torch.equal(gen.node_energy, full.node_energy)


@pytest.mark.parametrize("N,T,ring", [(7, 1500, 0), (64, 3000, 0), (130, 2111, 0), (256, 3000, 0), (64, 3000, 4)])
def test_inloop_statistics_equal_epilogue(ctx, monkeypatch, N, T, ring):
    """FOGNET_REPLAY_STATS=inloop (replay_inl_kernel: statistics accumulated
    while the runs are pushed) writes the outputs, records, histograms and
    energy of the default fused epilogue, with per-task outputs and without."""
    tr = tg.make_batch(51 + N, 5, N, T, sweep=True)
    pb, pi = fa.power_model(tr["mips"])
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace(dict(tr, p_busy=pb, p_idle=pi), dev)
    R = tr["arrive"].shape[0]
    ref = fa.run_batch(ctx, d, ring_capacity=ring, hist=True)
    torch.cuda.synchronize()
    monkeypatch.setenv("FOGNET_REPLAY_STATS", "inloop")
    inl = fa.run_batch(ctx, d, ring_capacity=ring, hist=True)
    so = fa.allocate_outputs(R, T, dev, N=N, energy=True, hist=True, per_task=False)
    fa.run_batch(ctx, d, out=so, ring_capacity=ring)
    torch.cuda.synchronize()
    assert (ref.rep_stats()["status"] == 0).all()
    for k in ("node", "status", "start_tick", "done_tick"):
        assert torch.equal(getattr(inl, k), getattr(ref, k)), k
    for o in (inl, so):
        assert o.rep_stats().tobytes() == ref.rep_stats().tobytes()
        assert torch.equal(o.hist, ref.hist) and torch.equal(o.node_energy, ref.node_energy)


def test_generated_preconditions(ctx):
    """fognet_run_generated_dev refuses what it cannot replay exactly."""
    mg, sc = fa.sweep_params(np.arange(2), 8)
    with pytest.raises(fa.FognetError) as e:
        fa.run_generated(ctx, 1, 2, 100, 8, mg, sc, policy=7)
    assert e.value.code == _abi.FOGNET_ERR_UNSUPPORTED
    out = fa.run_generated(ctx, 1, 2, 0, 8, mg, sc)  # empty traces
    torch.cuda.synchronize()
    assert (out.rep_stats()["status"] == 0).all() and (out.rep_stats()["n_tasks"] == 0).all()


# ------------------------------------------------------------------ a10/a11 statistics and the EXT_LAT policy
# Builder-defined rows (include/fognet_hip.h): parity against the oracle's
# restatement of the same definitions (not pinned by the reference).

def run_gpu_full(ctx, tr, policy="REF_V3", ring_capacity=0):
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace(tr, dev)
    out = fa.run_batch(ctx, d, ring_capacity=ring_capacity, policy=policy, hist=True)
    torch.cuda.synchronize()
    return dict(node=out.node.cpu().numpy(), status=out.status.cpu().numpy(),
                start=out.start_tick.cpu().numpy(), done=out.done_tick.cpu().numpy(),
                stats=out.rep_stats(), raw=out,
                energy=out.node_energy.cpu().numpy() if out.node_energy is not None else None,
                hist=out.hist.cpu().numpy())


@pytest.mark.parametrize("shared", [False, True])
def test_energy_and_histograms_match_oracle(ctx, shared):
    tr = tg.make_batch(0x5EED0003, 12, 256, 3000, sweep=True)
    if shared:
        tr = dict(tr, mips=tr["mips"][0], dl=tr["dl"][0], ul=tr["ul"][0], init=tr["init"][0])
    pb, pi = fa.power_model(tr["mips"])
    tr = dict(tr, p_busy=pb, p_idle=pi)
    g = run_gpu_full(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8,
                     p_busy=pb, p_idle=pi, hist=True)
    assert_parity(tr, g, o)
    # same IEEE operation sequence on both sides: bit-identical (north star asks 1e-9 relative)
    np.testing.assert_array_equal(g["energy"], o["node_energy"])
    assert g["stats"].tobytes() == o["stats"].tobytes()
    np.testing.assert_array_equal(g["hist"], o["hist"].sum(axis=0))
    # queueTime: one count per emission the reference can make (the rest overflow simtime_t)
    assert g["hist"][0].sum() == o["stats"]["n_qtime"].sum() and g["hist"][1].sum() == 12 * 3000
    assert (o["stats"]["n_qtime"] + o["stats"]["n_qtime_overflow"] == o["stats"]["n_queued"]).all()
    job = fa.reduce_stats(ctx, g["raw"].stats, 12)
    assert int(job["busy_s"]) == int(o["stats"]["busy_s"].sum())
    np.testing.assert_allclose(float(job["energy_j"]), float(o["stats"]["energy_j"].sum()), rtol=1e-12)


@pytest.mark.parametrize("N,T", [(7, 1500), (64, 1000), (130, 2111), (256, 3000), (300, 1500), (1000, 1200)])
def test_fused_statistics_equal_separate_pass(ctx, N, T):
    """fognet_run_batch_dev runs the statistics pass as the replay kernel's
    epilogue; fognet_replay_dev + fognet_rep_stats_dev run it as its own
    kernel.  Same record, histogram and per-node energy, bit for bit."""
    tr = tg.make_batch(0x5EED0077 + N, 5, N, T, sweep=True)
    pb, pi = fa.power_model(tr["mips"])
    tr = dict(tr, p_busy=pb, p_idle=pi)
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace(tr, dev)
    fused = fa.run_batch(ctx, d, hist=True)
    sep = fa.allocate_outputs(5, T, dev, N=N, energy=True, hist=True)
    fa.run_batch(ctx, d, out=sep, stage="replay")
    fa.run_batch(ctx, d, out=sep, stage="stats")
    torch.cuda.synchronize()
    assert fused.stats.cpu().numpy().tobytes() == sep.stats.cpu().numpy().tobytes()
    np.testing.assert_array_equal(fused.hist.cpu().numpy(), sep.hist.cpu().numpy())
    np.testing.assert_array_equal(fused.node_energy.cpu().numpy(), sep.node_energy.cpu().numpy())
    assert int(fused.hist.cpu().numpy()[1].sum()) == 5 * T


@pytest.mark.parametrize("ring", [2, 8])
def test_fused_statistics_equal_separate_pass_with_hand_over(ctx, ring):
    """The same with rings so small that replications are handed over to the
    wide kernel inside the replay stage: its inline histogram and energy must
    not be added on top of the statistics stage's."""
    N, T, R = 64, 2000, 5
    tr = tg.make_batch(0x5EED0078, R, N, T, sweep=True)
    pb, pi = fa.power_model(tr["mips"])
    d = fa.as_device_trace(dict(tr, p_busy=pb, p_idle=pi), torch.device("cuda", ctx.device))
    fused = fa.run_batch(ctx, d, hist=True, ring_capacity=ring)
    sep = fa.allocate_outputs(R, T, d["arrive"].device, N=N, energy=True, hist=True)
    fa.run_batch(ctx, d, out=sep, stage="replay", ring_capacity=ring)
    fa.run_batch(ctx, d, out=sep, stage="stats", ring_capacity=ring)
    torch.cuda.synchronize()
    assert (fused.rep_stats()["max_pending"] > ring).any()  # the hand-over happened
    assert fused.stats.cpu().numpy().tobytes() == sep.stats.cpu().numpy().tobytes()
    np.testing.assert_array_equal(fused.hist.cpu().numpy(), sep.hist.cpu().numpy())
    np.testing.assert_array_equal(fused.node_energy.cpu().numpy(), sep.node_energy.cpu().numpy())
    assert int(sep.hist.cpu().numpy()[1].sum()) == R * T


def test_decide_batch_rejects_other_policies(ctx):
    """fognet_decide_batch_dev, like fognet_decide and fognet_decide_window,
    evaluates REF_V3 only."""
    import ctypes as C
    dev = torch.device("cuda", ctx.device)
    busy = torch.zeros((1, 4), dtype=torch.float64, device=dev)
    mips = torch.full((1, 4), 1000, dtype=torch.int32, device=dev)
    req = torch.full((1,), 5000, dtype=torch.int32, device=dev)
    node = torch.empty(1, dtype=torch.int32, device=dev)
    for pol in (_abi.FOGNET_POLICY_EXT_LAT, _abi.FOGNET_POLICY_EXT_HIER, 0):
        rc = ctx._lib.fognet_decide_batch_dev(ctx.handle, pol, 1, 4, C.c_void_p(busy.data_ptr()),
                                              C.c_void_p(mips.data_ptr()), C.c_void_p(req.data_ptr()),
                                              C.c_void_p(node.data_ptr()), None, None)
        assert rc == _abi.FOGNET_ERR_UNSUPPORTED


def test_histogram_accumulates_across_calls(ctx):
    tr = tg.make_batch(3, 4, 32, 1000)
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace(tr, dev)
    out = fa.run_batch(ctx, d, hist=True)
    fa.run_batch(ctx, d, out=out)
    torch.cuda.synchronize()
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], hist=True)
    np.testing.assert_array_equal(out.hist.cpu().numpy(), 2 * o["hist"].sum(axis=0))


@pytest.mark.parametrize("N,T,R,rho", [(1, 500, 2, 0.9), (5, 2000, 3, 0.8), (64, 3000, 4, 0.8), (100, 2000, 3, 0.95),
                                       (256, 2500, 6, None)])
def test_ext_lat_policy_matches_oracle(ctx, N, T, R, rho):
    tr = tg.make_batch(4242 + N, R, N, T, sweep=rho is None, rho=rho or 0.8)
    g = run_gpu_full(ctx, tr, policy="EXT_LAT")
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8,
                     policy=ol.POLICY_EXT_LAT, hist=True)
    assert (o["stats"]["status"] == 0).all()
    assert_parity(tr, g, o)
    np.testing.assert_array_equal(g["hist"], o["hist"].sum(axis=0))


@pytest.mark.parametrize("seed", range(3))
def test_ext_lat_tie_heavy(ctx, seed):
    tr = tie_heavy(100 + seed, 8, 3 + 40 * seed, 1500)
    g = run_gpu_full(ctx, tr, policy="EXT_LAT", ring_capacity=4096)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8,
                     policy=ol.POLICY_EXT_LAT, hist=True)
    assert_parity(tr, g, o)


def test_ext_lat_latency_bound(ctx):
    tr = tg.make_batch(9, 2, 8, 100)
    tr = {k: v.copy() for k, v in tr.items()}
    tr["dl"][1, 2] = 2**50
    g = run_gpu_full(ctx, tr, policy="EXT_LAT")
    assert g["stats"]["status"][0] == 0 and g["stats"]["status"][1] == _abi.FOGNET_ERR_ARG


# ------------------------------------------------------------------ wide replay kernel (N > 256, config C5)
# replay_wide.hip restates the same closed form for node sets that do not fit
# in registers; FOGNET_REPLAY_KERNEL=wide forces it for small N as well.

# REF_V3 herds every publish onto the least-advertised node until its first
# completion advert lands, so the C3 loads (rho 0.5..0.95) keep 10^3-10^4 nodes
# on node 0 for the whole trace; light loads spread decisions over many nodes.
@pytest.mark.parametrize("N,T,R,rho", [(257, 2000, 3, 0.8), (700, 3000, 3, 0.01), (4096, 4000, 2, 0.01),
                                       (12288, 3000, 1, 0.002), (20000, 1500, 1, 0.001),
                                       (65536, 1200, 1, 0.0005),  # the last N with the group minima in LDS
                                       (70000, 1200, 2, 0.0005), (262144, 400, 1, 0.0002)])  # in HBM (BIG)
def test_wide_matches_oracle(ctx, N, T, R, rho):
    tr = tg.make_batch(0x5EED0005 + N, R, N, T, rho=rho, lat_scale=10)
    pb, pi = fa.power_model(tr["mips"])
    tr = dict(tr, p_busy=pb, p_idle=pi)
    g = run_gpu_full(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8,
                     p_busy=pb, p_idle=pi, hist=True)
    assert (o["stats"]["status"] == 0).all()
    assert_parity(tr, g, o)
    np.testing.assert_array_equal(g["energy"], o["node_energy"])
    assert g["stats"].tobytes() == o["stats"].tobytes()
    np.testing.assert_array_equal(g["hist"], o["hist"].sum(axis=0))


@pytest.mark.parametrize("policy,N,down", [("REF_V3", 700, False), ("REF_V3", 10_000, False), ("EXT_LAT", 3000, False),
                                           ("REF_V3", 2000, True)])
def test_wide_big_layout_equals_lds_layout(ctx, monkeypatch, policy, N, down):
    """FOGNET_WIDE_BIG=1 keeps the wide kernel's group minima in HBM (the layout above N = 65,536)
    at any N: every output, record and histogram equals the LDS layout's, and the oracle's."""
    tr = tg.make_batch(0xB16 + N, 3, N, 2000, rho=0.01, lat_scale=10)
    if down:
        tr = with_crashes(tr, 5, 0.2)
    lds = run_gpu_full(ctx, tr, policy=policy)
    monkeypatch.setenv("FOGNET_WIDE_BIG", "1")
    big = run_gpu_full(ctx, tr, policy=policy)
    for k in ("node", "status", "start", "done", "hist"):
        np.testing.assert_array_equal(big[k], lds[k], err_msg=k)
    assert big["stats"].tobytes() == lds["stats"].tobytes()
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=3, hist=True,
                     policy=ol.POLICIES[policy], down=tr.get("down"))
    assert_parity(tr, big, o)


def test_wide_ext_lat_above_65536_nodes(ctx):
    """EXT_LAT (the north-star cost, every node's cost per publish) at N = 70,000: the group
    minima in HBM; equal to the oracle."""
    tr = tg.make_batch(0x7000, 1, 70_000, 300, sweep=True)
    g = run_gpu_full(ctx, tr, policy="EXT_LAT")
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], policy=ol.POLICY_EXT_LAT,
                     hist=True)
    assert (o["stats"]["status"] == 0).all()
    assert_parity(tr, g, o)


@pytest.mark.parametrize("N", [1, 5, 64, 100, 256])
def test_wide_kernel_forced_equals_register_kernel(ctx, monkeypatch, N):
    tr = tg.make_batch(1000 + N, 3, N, 1500, rho=0.9)
    narrow = run_gpu_full(ctx, tr, ring_capacity=4096)
    monkeypatch.setenv("FOGNET_REPLAY_KERNEL", "wide")
    wide = run_gpu_full(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=3, hist=True)
    assert_parity(tr, wide, o)
    assert wide["stats"].tobytes() == narrow["stats"].tobytes()
    np.testing.assert_array_equal(wide["hist"], narrow["hist"])


@pytest.mark.parametrize("policy", ["REF_V3", "EXT_LAT"])
def test_wide_head_next_paths(ctx, monkeypatch, policy):
    """The three paths that set a node record's hd_next (the
    root cause of round 2's wrong-decision experiment), each followed by the
    node's advert, which advances the head to hd_next: a push onto a node with
    one pending task, a push onto one with two, a multi-task run onto an idle
    node; on the wide kernel the chain invariant is checked at every advert
    (FOGNET_ERR_INTERNAL) and every output equals the oracle."""
    monkeypatch.setenv("FOGNET_REPLAY_KERNEL", "wide")
    MS = 10**9
    N = 3
    base = 50 * MS
    # bursts of 1, 2, 3 and 6 publishes one tick apart onto the argmin, spaced so adverts land in between
    ticks, reqs = [], []
    for b, (n, gap_s) in enumerate(((1, 3), (2, 5), (3, 7), (6, 11), (2, 2), (1, 1))):
        t0 = base + sum((3, 5, 7, 11, 2, 1)[:b]) * 10**12 + b * MS
        for q in range(n):
            ticks.append(t0 + q)
            reqs.append((1 + (q + b) % 3) * 1000)
    arrive = np.array(ticks, np.int64)[None]
    req = np.array(reqs, np.int32)[None]
    mips = np.full(N, 1000, np.int32)
    dl = np.array([MS, 2 * MS, 3 * MS], np.int64)
    ul = np.array([MS, MS, 2 * MS], np.int64)
    init = np.full(N, 2 * MS, np.int64)
    tr = dict(arrive=arrive, req=req, mips=mips, dl=dl, ul=ul, init=init)
    g = run_gpu_full(ctx, tr, policy=policy)
    o = ol.run_batch(arrive, req, mips, dl, ul, init, hist=True, policy=ol.POLICIES[policy])
    assert g["stats"]["status"][0] == 0
    assert_parity(tr, g, o)
    assert int(g["stats"]["max_pending"][0]) >= 3


@pytest.mark.parametrize("seed", range(4))
def test_wide_tie_heavy(ctx, monkeypatch, seed):
    tr = tie_heavy(seed, 8, 1 + 37 * seed, 2000)
    monkeypatch.setenv("FOGNET_REPLAY_KERNEL", "wide")
    g = run_gpu(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8)
    assert_parity(tr, g, o)


def test_wide_tie_heavy_many_nodes(ctx):
    tr = tie_heavy(77, 4, 600, 3000)
    g = run_gpu(ctx, tr)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=4)
    assert_parity(tr, g, o)


@pytest.mark.parametrize("N", [300, 2000])
def test_wide_ext_lat_matches_oracle(ctx, N):
    tr = tg.make_batch(4343 + N, 3, N, 1500, sweep=True)
    g = run_gpu_full(ctx, tr, policy="EXT_LAT")
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=3,
                     policy=ol.POLICY_EXT_LAT, hist=True)
    assert (o["stats"]["status"] == 0).all()
    assert_parity(tr, g, o)
    np.testing.assert_array_equal(g["hist"], o["hist"].sum(axis=0))


def test_wide_ext_lat_forced_tie_heavy(ctx, monkeypatch):
    tr = tie_heavy(123, 8, 41, 1500)
    monkeypatch.setenv("FOGNET_REPLAY_KERNEL", "wide")
    g = run_gpu_full(ctx, tr, policy="EXT_LAT")
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8,
                     policy=ol.POLICY_EXT_LAT, hist=True)
    assert_parity(tr, g, o)


def test_c5_large_topology_sample(ctx):
    """Config C5 shape (BASELINE.json configs[4]): N = 10,000 fog nodes,
    T = 10,000 tasks, device-generated traces; every replication against the oracle."""
    R, T, N = 4, 10_000, 10_000
    mg, sc = fa.c5_params(np.arange(R), N)
    d = fa.generate_trace(ctx, 0x5EED0005, R, T, N, mg, sc)
    out = fa.run_batch(ctx, d)
    torch.cuda.synchronize()
    st = out.rep_stats()
    assert (st["status"] == 0).all() and (st["n_tasks"] == T).all()
    for r in range(R):
        h = {k: d[k][r].cpu().numpy() for k in ("arrive", "req", "mips", "dl", "ul", "init")}
        o = ol.run_batch(h["arrive"], h["req"], h["mips"], h["dl"], h["ul"], h["init"])
        for k_gpu, k_ref in (("node", "node"), ("status", "status"), ("start_tick", "start"), ("done_tick", "done")):
            np.testing.assert_array_equal(getattr(out, k_gpu)[r].cpu().numpy(), o[k_ref][0], err_msg=k_gpu)
        assert st[r].tobytes() == o["stats"][0].tobytes()


# ------------------------------------------------------------------ user-side signals (ack relay)
# fognet_user_stats_dev (closed form over the replay outputs) against the
# oracle's event-level restatement (acks as FES events relayed by the broker).

def assert_user_parity(g_user, o_user):
    for n in ol.USER_SIGNALS:
        for f in ("count", "min_raw", "max_raw", "sum_lo", "sum_hi", "sq_lo", "sq_hi", "sq_top", "overflow"):
            np.testing.assert_array_equal(g_user[n][f], o_user[n][f], err_msg=f"{n}.{f}")


@pytest.mark.parametrize("kind", ["one_user", "per_task", "tie_heavy", "wide"])
def test_user_stats_match_oracle(ctx, kind):
    rng = np.random.default_rng(31)
    if kind == "tie_heavy":
        tr = tie_heavy(5, 6, 37, 1500)
    elif kind == "wide":
        tr = tg.make_batch(0x5EED0005, 3, 400, 2000, rho=0.01, lat_scale=10)
    else:
        tr = tg.make_batch(0x5EED0003, 6, 64, 2000, sweep=True)
    R, T = tr["arrive"].shape
    shape = (R, T) if kind == "per_task" else (R,)
    uu = rng.integers(0, 5 * 10**9, shape).astype(np.int64)
    ud = rng.integers(0, 5 * 10**9, shape).astype(np.int64)
    if kind == "tie_heavy":
        uu[:] = 0
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace(tr, dev)
    out = fa.run_batch(ctx, d, ring_capacity=4096)
    g = fa.user_stats(ctx, d, out, uu, ud)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=6, user_ul=uu,
                     user_dl=ud)
    assert (o["stats"]["status"] == 0).all()
    assert_user_parity(g, o["user"])


def test_user_stats_with_reference_task_source(ctx):
    """Several users publishing through mqttApp2's timer chain and glibc rand()
    stream (fognet_gen_trace_mqtt); per-task user links from the user index."""
    from fognetsimpp_amd import formats
    MS = 10**9
    U = 6
    up = np.array([2, 3, 5, 7, 11, 13], np.int64) * MS
    dn = np.array([1, 4, 6, 8, 9, 10], np.int64) * MS
    g = formats.gen_trace_mqtt(1, np.arange(U) * 7 * MS, np.full(U, 20_000 * MS), up, dn, 2000 * 10**12,
                               req_base=1000, req_span=30000)
    n = 8
    tr = dict(arrive=g["arrive"][None], req=g["req"][None], mips=(1000 * (1 + np.arange(n) % 4)).astype(np.int32),
              dl=np.full(n, 3 * MS, np.int64), ul=np.full(n, 4 * MS, np.int64), init=np.full(n, 4 * MS, np.int64))
    uu, ud = up[g["user"]][None], dn[g["user"]][None]
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace(tr, dev)
    out = fa.run_batch(ctx, d)
    gu = fa.user_stats(ctx, d, out, uu, ud)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], user_ul=uu, user_dl=ud)
    assert o["stats"]["status"][0] == 0 and int(o["stats"]["n_tasks"][0]) == g["arrive"].size
    np.testing.assert_array_equal(out.node.cpu().numpy(), o["node"])
    assert_user_parity(gu, o["user"])


# ------------------------------------------------------------------ v2 model replay
# replay_v2.hip (lane-parallel FES per replication) against the oracle's
# heap-ordered DES restatement (oracle/fognet_oracle_v2.c).

V2_FIELDS = ("n_tasks", "n_local", "n_forwarded", "n_accepted", "n_rejected", "n_dropped", "n_no_nodes",
             "n_released_broker", "n_inflated", "n_released_node", "n_relayed", "events", "node_mips_final_sum",
             "broker_mips_final", "status")


def run_v2_gpu(ctx, tr, broker_mips, stop, rt=0.01, qcap=0):
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace({k: tr[k] for k in ("arrive", "req", "mips", "dl", "ul", "first_adv")}, dev)
    out = fa.run_v2(ctx, d, broker_mips, stop, rt, queue_capacity=qcap)
    torch.cuda.synchronize()
    return dict(node=out.node.cpu().numpy(), status=out.status.cpu().numpy(), start=out.start_tick.cpu().numpy(),
                done=out.done_tick.cpu().numpy(), stats=out.rep_stats())


def assert_v2_parity(g, o):
    for k in ("node", "status", "start", "done"):
        np.testing.assert_array_equal(g[k], o[k], err_msg=k)
    for f in V2_FIELDS:
        np.testing.assert_array_equal(g["stats"][f], o["stats"][f], err_msg=f)


@pytest.mark.parametrize("case", golden_io.replay_v2_cases(), ids=lambda c: c[0])
def test_v2_replay_known_answers_gpu(ctx, case):
    name, tr, e = case
    g = run_v2_gpu(ctx, tr, tr["broker_mips"], tr["stop"])
    assert g["node"][0].tolist() == e["node"] and g["status"][0].tolist() == e["status"]
    assert g["start"][0].tolist() == e["start"] and g["done"][0].tolist() == e["done"]
    assert int(g["stats"]["status"][0]) == e.get("rep_status", 0)
    o = ol.run_v2(tr["arrive"], tr["req"], tr["broker_mips"], tr["mips"], tr["dl"], tr["ul"], tr["first_adv"],
                  tr["stop"])
    assert_v2_parity(g, o)


def v2_random(seed, R, N, T):
    """Coarse millisecond grids so arrivals, timer firings and messages share
    ticks often (the FES insertion-order rule decides), per-replication broker
    pools, requiredTime values and stop times; shared node parameters."""
    rng = np.random.default_rng(seed)
    MS = 10**9
    gaps = rng.choice([0, 1, 2, 5, 10, 50], size=(R, T)) * MS
    arrive = (rng.integers(0, 30, size=(R, 1)) * MS + np.cumsum(gaps, axis=1)).astype(np.int64)
    req = rng.integers(0, 1600, size=(R, T)).astype(np.int32)
    mips = rng.choice([500, 1000, 1500], size=(R, N)).astype(np.int32)
    dl = rng.choice([0, 1, 2, 10, 20], size=(R, N)).astype(np.int64) * MS
    ul = rng.choice([0, 1, 2, 10, 20], size=(R, N)).astype(np.int64) * MS
    first = rng.integers(0, 21, size=(R, N)).astype(np.int64) * MS
    broker = rng.choice([0, 300, 1000, 2500], size=R).astype(np.int32)
    rt = rng.choice([0.01, 0.005, 0.02], size=R)
    stop = arrive[:, -1] + rng.integers(0, 200, size=R) * MS
    return dict(arrive=arrive, req=req, mips=mips, dl=dl, ul=ul, first_adv=first), broker, stop, rt


@pytest.mark.parametrize("seed,N,R", [(0, 1, 16), (1, 2, 16), (2, 5, 16), (3, 13, 16), (4, 64, 16), (5, 5, 16),
                                      (6, 16, 7), (7, 17, 5), (8, 3, 1), (9, 5, 13), (10, 65, 5), (11, 200, 4),
                                      (12, 129, 3), (13, 300, 2), (14, 1024, 2), (15, 2048, 2), (16, 4096, 1),
                                      (17, 4097, 1), (18, 8192, 2), (19, 8193, 1), (20, 16384, 1)])
def test_v2_random_matches_oracle(ctx, seed, N, R):
    """N <= 16: replay_v2_rows_kernel<16> (four replications per wavefront, R not
    a multiple of four included); 17 <= N <= 32: replay_v2_rows_kernel<32> (two);
    N > 32: replay_v2_kernel<NPL> with node j on lane j % 64, slot j / 64 (NPL = 1,
    2, 4, 8, 16, 32, 64, 128, 256: N <= 16384, the batches cut at 4,096 firings above 8,192; the
    reference's loop takes any brokers.size(),
    BrokerBaseApp2.cc:241-248).  Every node's 10-ms timer fires throughout, so the
    wider node sets take shorter traces."""
    tr, broker, stop, rt = v2_random(seed, R, N, 3000 if N <= 256 else 1500 if N <= 1024 else 400 if N <= 2048 else
                                     200 if N <= 4096 else 120 if N <= 8192 else 60)
    g = run_v2_gpu(ctx, tr, broker, stop, rt, qcap=4096)
    o = ol.run_v2(tr["arrive"], tr["req"], broker, tr["mips"], tr["dl"], tr["ul"], tr["first_adv"], stop, rt,
                  threads=8)
    assert (o["stats"]["status"] == 0).all()
    assert_v2_parity(g, o)


@pytest.mark.parametrize("N,T", [(4096, 400), (8192, 200), (16384, 100)])
def test_v2_widest_node_set_reserves_on_high_slots(ctx, N, T):
    """N = 4096 (replay_v2_kernel<64>: 64 nodes per lane, per-node records in scratch) and N = 8192
    (replay_v2_kernel<128>: the slot masks take 128 bits) with R = 4 and traces long enough for
    reservations, rejections and releases on the high slots: node 0 advertises the smallest MIPS, so
    BrokerBaseApp2's "last node whose MIPS exceeds node 0's" (BrokerBaseApp2.cc:241-248) lands at
    j >= N / 2 (slots past 64 at N = 8192).  Equal to the oracle DES."""
    R = 4
    tr, broker, stop, rt = v2_random(61, R, N, T)
    tr["mips"][:, 0] = 500
    tr["mips"][:, -64:] = 1500  # the last few nodes beat node 0 in every replication
    tr["req"] = (tr["req"] % 400).astype(np.int32)  # small requirements: several reservations per node at once
    rt = np.array([0.01, 0.02, 0.05, 0.05])
    g = run_v2_gpu(ctx, tr, broker, stop, rt, qcap=256)
    o = ol.run_v2(tr["arrive"], tr["req"], broker, tr["mips"], tr["dl"], tr["ul"], tr["first_adv"], stop, rt,
                  threads=4)
    assert (o["stats"]["status"] == 0).all()
    assert_v2_parity(g, o)
    fwd = g["node"][np.isin(g["status"], [_abi.V2_ST_ACCEPTED, _abi.V2_ST_REJECTED])]
    assert fwd.size > 0 and fwd.min() >= N // 2
    assert (g["stats"]["n_accepted"] > 0).all() and (g["stats"]["n_released_node"] > 0).all()


def test_v2_widest_node_set_capacity_refused(ctx):
    """N = 4096 with a reservation list of capacity 16 and long requiredTimes: the replications whose
    node holds more than 16 reservations at once are refused (FOGNET_ERR_CAPACITY, the queues never
    wrap); a replication that stays within the capacity is still equal to the oracle DES."""
    R, N, T = 3, 4096, 300
    tr, broker, stop, rt = v2_random(62, R, N, T)
    tr["mips"][:, 0] = 500
    tr["mips"][:, -64:] = 1500
    tr["req"] = (tr["req"] % 20 + 1).astype(np.int32)
    rt = np.array([0.5, 0.5, 0.001])  # replication 2: each reservation released before the next arrives
    broker = np.zeros(R, np.int32)  # no broker pool: every publish is forwarded
    g = run_v2_gpu(ctx, tr, broker, stop, rt, qcap=16)
    st = g["stats"]["status"]
    assert (st[:2] == _abi.FOGNET_ERR_CAPACITY).all()
    o = ol.run_v2(tr["arrive"][2:], tr["req"][2:], broker[2:], tr["mips"][2:], tr["dl"][2:], tr["ul"][2:],
                  tr["first_adv"][2:], stop[2:], rt[2:], threads=1)
    assert st[2] == 0 and (o["stats"]["status"] == 0).all()
    assert_v2_parity({k: v[2:] for k, v in g.items()}, o)


@pytest.mark.parametrize("env", [("FOGNET_V2_ROW", "32"), ("FOGNET_V2_ACTIVE", "4")])
@pytest.mark.parametrize("N", [5, 16])
def test_v2_two_rows_per_wave_at_small_n(ctx, monkeypatch, N, env):
    """Where N <= 16 takes replay_v2_rows_kernel<16, 2> (16-lane rows, two of the
    four busy), FOGNET_V2_ROW=32 forces replay_v2_rows_kernel<32> (two 32-lane
    rows per wavefront) and FOGNET_V2_ACTIVE=4 all four 16-lane rows: same outputs
    (R = 7: a wavefront with a row past R in every variant)."""
    monkeypatch.setenv(*env)
    tr, broker, stop, rt = v2_random(40 + N, 7, N, 3000)
    g = run_v2_gpu(ctx, tr, broker, stop, rt, qcap=4096)
    o = ol.run_v2(tr["arrive"], tr["req"], broker, tr["mips"], tr["dl"], tr["ul"], tr["first_adv"], stop, rt,
                  threads=7)
    assert (o["stats"]["status"] == 0).all()
    assert_v2_parity(g, o)


@pytest.mark.parametrize("seed,N,R", [(21, 16, 8), (22, 5, 9), (23, 3, 4)])
def test_v2_deep_fifos_and_long_uplinks(ctx, seed, N, R):
    """Links longer than the 10-ms advert period (ul up to 45 ms, dl up to 60 ms):
    several adverts of one node in flight, so most cannot be left out of the queue
    and the FIFOs hold three or more entries (the entries past the two kept in
    registers live in HBM); N = 16 is the rows kernel's widest row.  Equal to the
    oracle DES, event counts included."""
    rng = np.random.default_rng(seed)
    MS = 10**9
    T = 1500
    gaps = rng.choice([0, 1, 3, 10, 20], size=(R, T)) * MS
    arrive = (rng.integers(0, 30, size=(R, 1)) * MS + np.cumsum(gaps, axis=1)).astype(np.int64)
    req = rng.integers(0, 900, size=(R, T)).astype(np.int32)
    tr = dict(arrive=arrive, req=req, mips=rng.choice([600, 1000, 1400], size=(R, N)).astype(np.int32),
              dl=rng.choice([1, 15, 35, 60], size=(R, N)).astype(np.int64) * MS,
              ul=rng.choice([1, 10, 25, 45], size=(R, N)).astype(np.int64) * MS,
              first_adv=rng.integers(0, 25, size=(R, N)).astype(np.int64) * MS)
    broker = rng.choice([0, 500, 2000], size=R).astype(np.int32)
    rt = rng.choice([0.01, 0.03, 0.05], size=R)
    stop = arrive[:, -1] + rng.integers(0, 300, size=R) * MS
    g = run_v2_gpu(ctx, tr, broker, stop, rt, qcap=4096)
    o = ol.run_v2(tr["arrive"], tr["req"], broker, tr["mips"], tr["dl"], tr["ul"], tr["first_adv"], stop, rt,
                  threads=8)
    assert (o["stats"]["status"] == 0).all()
    assert_v2_parity(g, o)


def test_v2_node_reproduces_general0_recording_gpu(ctx):
    """The device v2 replay on the General-0 recording fixture (see test_oracle)."""
    tr, d = golden_io.general0_v2_node()
    dev = torch.device("cuda", ctx.device)
    dt = fa.as_device_trace(dict(arrive=tr["arrive"], req=tr["req"], mips=tr["mips"], dl=tr["dl"], ul=tr["ul"],
                                 first_adv=tr["first_adv"]), dev)
    out = fa.run_v2(ctx, dt, tr["broker_mips"], tr["stop"], 0.01)
    torch.cuda.synchronize()
    assert (out.node[0].cpu().numpy() == 0).all()
    np.testing.assert_array_equal(out.start_tick[0].cpu().numpy(), d["task_arrival_ticks"])
    np.testing.assert_array_equal(out.done_tick[0].cpu().numpy(), d["release_ticks"])
    assert out.rep_stats()["n_released_node"][0] == 4


def test_v2_c1_as_shipped(ctx):
    """Config C1 (BASELINE.json configs[0]) with the modules its ini names:
    one user (mqttApp2's timer chain + glibc rand()), broker and 5 nodes at 1000
    MIPS, 1000 s.  Bit-exact with the oracle, including the rounding-stuck pool."""
    from fognetsimpp_amd import formats
    MS = 10**9
    g0 = formats.gen_trace_mqtt(1, [0], [50 * MS], [MS], [-1], 1000 * 10**12)
    n = 5
    tr = dict(arrive=g0["arrive"][None], req=g0["req"][None], mips=np.full(n, 1000, np.int32), dl=np.full(n, MS),
              ul=np.full(n, MS), first_adv=np.full(n, 20 * MS))
    g = run_v2_gpu(ctx, tr, 1000, 1000 * 10**12)
    o = ol.run_v2(tr["arrive"], tr["req"], 1000, tr["mips"], tr["dl"], tr["ul"], tr["first_adv"], 1000 * 10**12)
    assert_v2_parity(g, o)
    assert (int(g["stats"]["n_local"][0]), int(g["stats"]["n_forwarded"][0])) == (9, 19990)


def test_v2_errors(ctx):
    MS = 10**9
    tr = dict(arrive=np.array([[10 * MS, 12 * MS]]), req=np.array([[150, 150]], np.int32),
              mips=np.zeros(0, np.int32), dl=np.zeros(0, np.int64), ul=np.zeros(0, np.int64),
              first_adv=np.zeros(0, np.int64))
    g = run_v2_gpu(ctx, tr, 100, 100 * MS)
    assert int(g["stats"]["status"][0]) == _abi.FOGNET_ERR_STATE
    n = _abi.V2_MAX_NODES + 1  # (256 nodes per lane)
    big = dict(arrive=np.array([[10 * MS]]), req=np.array([[1]], np.int32), mips=np.full(n, 1000, np.int32),
               dl=np.ones(n, np.int64), ul=np.ones(n, np.int64), first_adv=np.ones(n, np.int64))
    with pytest.raises(fa.FognetError) as e:
        run_v2_gpu(ctx, big, 100, 100 * MS)
    assert e.value.code == _abi.FOGNET_ERR_UNSUPPORTED
    tr2, broker, stop, rt = v2_random(9, 2, 3, 500)
    g = run_v2_gpu(ctx, tr2, broker, np.full(2, 2**53 + 1), rt)
    assert (g["stats"]["status"] == _abi.FOGNET_ERR_ARG).all()


# ------------------------------------------------------------------ node-down extension

def with_crashes(tr, seed, frac=0.3, grid=None):
    """Crash ticks for a fraction of the nodes, between each node's first advert
    and the last publish (snapped to ``grid`` so crashes collide with events)."""
    rng = np.random.default_rng(seed)
    init = np.asarray(tr["init"])
    last = int(np.asarray(tr["arrive"]).max())
    down = np.full(init.shape, fa.NEVER, np.int64)
    pick = rng.random(init.shape) < frac
    pick[..., 0] = True  # the stale view favours low indices: make the crashes matter
    t = rng.integers(init, np.maximum(init + 1, last), dtype=np.int64)
    if grid:
        t = np.maximum(init, (t // grid) * grid)
    down[pick] = t[pick]
    return dict(tr, down=down)


def oracle_down(tr, **kw):
    return ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], down=tr["down"],
                        hist=True, **kw)


@pytest.mark.parametrize("case", golden_io.replay_down_cases(), ids=lambda c: c[0])
def test_down_known_answers_gpu(ctx, case):
    name, tr, exp = case
    tr = dict(tr, arrive=tr["arrive"][None], req=tr["req"][None])
    g = run_gpu_full(ctx, tr)
    np.testing.assert_array_equal(g["node"][0], exp["node"])
    np.testing.assert_array_equal(g["status"][0], exp["status"])
    np.testing.assert_array_equal(g["start"][0], exp["start"])
    np.testing.assert_array_equal(g["done"][0], exp["done"])
    o = oracle_down(tr)
    assert g["stats"].tobytes() == o["stats"].tobytes()
    np.testing.assert_array_equal(g["hist"], o["hist"].sum(axis=0))


@pytest.mark.parametrize("N,T,R,policy", [(5, 2000, 6, "REF_V3"), (64, 2000, 4, "REF_V3"), (300, 2000, 3, "REF_V3"),
                                          (1000, 1500, 2, "REF_V3"), (40, 1500, 4, "EXT_LAT"),
                                          (300, 1500, 3, "EXT_LAT")])
def test_down_matches_oracle(ctx, N, T, R, policy):
    tr = with_crashes(tg.make_batch(0xD0 + N, R, N, T, rho=0.9, lat_scale=10), seed=N)
    g = run_gpu_full(ctx, tr, policy=policy)
    o = oracle_down(tr, threads=R, policy=ol.POLICIES[policy])
    assert (o["stats"]["status"] == 0).all()
    assert ((o["status"] == 9) | (o["done"] == -1)).any()  # the crashes bite
    assert_parity(tr, g, o)
    assert g["stats"].tobytes() == o["stats"].tobytes()
    np.testing.assert_array_equal(g["hist"], o["hist"].sum(axis=0))


@pytest.mark.parametrize("seed", range(4))
def test_down_tie_heavy(ctx, seed):
    """Crash ticks on the same coarse grid as arrivals, completions and adverts."""
    tr = with_crashes(tie_heavy(300 + seed, 6, 1 + 23 * seed, 1500), seed=seed, frac=0.5, grid=10**11)
    g = run_gpu_full(ctx, tr)
    o = oracle_down(tr, threads=6)
    assert_parity(tr, g, o)
    assert g["stats"].tobytes() == o["stats"].tobytes()


def test_down_never_equals_plain_run(ctx):
    tr = tg.make_batch(0xD1, 3, 50, 1500, rho=0.9)
    plain = run_gpu_full(ctx, tr)
    g = run_gpu_full(ctx, dict(tr, down=np.full(np.shape(tr["mips"]), fa.NEVER, np.int64)))
    for k in ("node", "status", "start", "done", "hist"):
        np.testing.assert_array_equal(g[k], plain[k])
    assert g["stats"].tobytes() == plain["stats"].tobytes()


def test_down_user_stats(ctx):
    """Lost tasks send no node ack, never-completed tasks no status-6 ack."""
    tr = with_crashes(tg.make_batch(0xD2, 4, 30, 2000, rho=0.9), seed=2, frac=0.4)
    R = 4
    rng = np.random.default_rng(3)
    uu = rng.integers(0, 5 * 10**9, R).astype(np.int64)
    ud = rng.integers(0, 5 * 10**9, R).astype(np.int64)
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace(tr, dev)
    out = fa.run_batch(ctx, d)
    g = fa.user_stats(ctx, d, out, uu, ud)
    o = oracle_down(tr, threads=4, user_ul=uu, user_dl=ud)
    assert (o["stats"]["status"] == 0).all()
    assert_user_parity(g, o["user"])


def test_down_errors(ctx):
    tr = golden_io.replay_down_cases()[0][1]
    tr = dict(tr, arrive=tr["arrive"][None], req=tr["req"][None])
    bad = tr["down"].copy()
    bad[0] = tr["init"][0] - 1
    g = run_gpu(ctx, dict(tr, down=bad))
    assert g["stats"]["status"][0] == _abi.FOGNET_ERR_ARG
    pb, pi = fa.power_model(tr["mips"])
    dev = torch.device("cuda", ctx.device)
    with pytest.raises(fa.FognetError) as ei:
        fa.run_batch(ctx, fa.as_device_trace(dict(tr, p_busy=pb, p_idle=pi), dev))
    assert ei.value.code == _abi.FOGNET_ERR_UNSUPPORTED


# ------------------------------------------------------------------ hierarchical brokers + mobility (C5 extension)
# FOGNET_POLICY_EXT_HIER (not in the reference): parity against the oracle's
# restatement of the same definition (include/fognet_hip.h).

def test_hier_known_answer_gpu(ctx):
    tr, exp, kw = hier_kat()
    dev = torch.device("cuda", ctx.device)
    out = fa.run_batch(ctx, fa.as_device_trace(tr, dev), policy="EXT_HIER", **kw)
    torch.cuda.synchronize()
    assert out.rep_stats()["status"][0] == 0
    for k, g in (("node", out.node), ("status", out.status), ("start", out.start_tick), ("done", out.done_tick)):
        np.testing.assert_array_equal(g[0].cpu().numpy(), exp[k], err_msg=k)


@pytest.mark.parametrize("kind", ["sweep", "tie_heavy", "down", "light"])
def test_hier_matches_oracle(ctx, kind):
    """Hierarchical brokers with mobility handoff (fa.mobility_regions) against the
    oracle: escalations, same-tick arrivals of escalated tasks, node crashes."""
    thr, up = 5, 20 * 10**9
    if kind == "tie_heavy":
        tr = tie_heavy(17, 3, 2100, 1500)
        up = 10**11  # the tie-heavy tick base: escalated arrivals collide with completions
        thr = 1
    elif kind == "light":
        tr = tg.make_batch(18, 3, 3000, 3000, rho=0.01, lat_scale=10)
    else:
        tr = tg.make_batch(19, 3, 2500, 3000, rho=0.8)
    tr = dict(tr, region=fa.mobility_regions(tr["arrive"], tr["mips"].shape[-1], users=37))
    if kind == "down":
        rng = np.random.default_rng(3)
        dn = np.full(tr["mips"].shape, np.iinfo(np.int64).max, np.int64)
        pick = rng.random(dn.shape) < 0.02
        dn[pick] = (tr["init"].max() + rng.integers(1, 3000, size=dn.shape) * 10**11)[pick]
        tr["down"] = dn
    dev = torch.device("cuda", ctx.device)
    out = fa.run_batch(ctx, fa.as_device_trace(tr, dev), policy="EXT_HIER", hist=True, hier_threshold_s=thr,
                       hier_up_tick=up)
    torch.cuda.synchronize()
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8, hist=True,
                     policy=ol.POLICY_EXT_HIER, region=tr["region"], down=tr.get("down"), hier_threshold_s=thr,
                     hier_up_tick=up)
    g = dict(node=out.node.cpu().numpy(), status=out.status.cpu().numpy(), start=out.start_tick.cpu().numpy(),
             done=out.done_tick.cpu().numpy(), stats=out.rep_stats())
    assert (g["stats"]["status"] == 0).all()
    assert_parity(tr, g, o)
    np.testing.assert_array_equal(out.hist.cpu().numpy(), o["hist"].sum(axis=0))


def test_hier_region_pass_and_handover(ctx, monkeypatch):
    """EXT_HIER by region (replay_region.hip: one wavefront per regional broker
    while no region escalates) with the sequential hand-over: of six
    replications five never escalate (two regions, one of 6 nodes) and one does
    (297 escalated publishes in the oracle).  FOGNET_HIER_REGIONS=only shows the
    region pass finishing exactly the five; the default (region pass + the sixth
    continued by the sequential kernel from its first escalated publish), the
    restart (FOGNET_HIER_RESUME=0: the sixth replayed from the start) and
    FOGNET_HIER_REGIONS=0 (sequential only) all equal the oracle, records and job
    histogram included."""
    tr = tg.make_batch(21, 6, 1030, 4000, rho=0.9)
    reg = np.zeros_like(tr["req"])
    reg[1::2, 1::2] = 1
    reg[0, 5::7] = 1
    pb, pi = fa.power_model(tr["mips"])
    tr = dict(tr, region=reg, p_busy=pb, p_idle=pi)
    kw = dict(policy="EXT_HIER", hier_threshold_s=0, hier_up_tick=10**12, hist=True)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=6, hist=True,
                     policy=ol.POLICY_EXT_HIER, region=reg, hier_threshold_s=0, hier_up_tick=10**12,
                     p_busy=pb, p_idle=pi)
    esc = (o["node"] // _abi.HIER_REGION_NODES != reg).sum(axis=1)
    assert list(esc > 0) == [False] * 5 + [True]
    dev = torch.device("cuda", ctx.device)
    d = fa.as_device_trace(tr, dev)
    monkeypatch.setenv("FOGNET_HIER_REGIONS", "only")
    out = fa.run_batch(ctx, d, **kw)
    torch.cuda.synchronize()
    st = out.rep_stats()
    assert list(st["status"][:5]) == [0] * 5 and st["status"][5] not in (0, _abi.FOGNET_ERR_ARG)
    for k, gk in (("node", out.node), ("status", out.status), ("start", out.start_tick), ("done", out.done_tick)):
        np.testing.assert_array_equal(gk.cpu().numpy()[:5], o[k][:5], err_msg=k)
    assert st[:5].tobytes() == o["stats"][:5].tobytes()
    np.testing.assert_array_equal(out.node_energy.cpu().numpy()[:5], o["node_energy"][:5])
    np.testing.assert_array_equal(out.hist.cpu().numpy(), o["hist"][:5].sum(axis=0))
    for mode in ("1", "1-restart", "0"):  # (1: the sixth resumed at its first escalated publish)
        monkeypatch.setenv("FOGNET_HIER_REGIONS", mode.split("-")[0])
        monkeypatch.setenv("FOGNET_HIER_RESUME", "0" if mode == "1-restart" else "1")
        out = fa.run_batch(ctx, d, **kw)
        torch.cuda.synchronize()
        g = dict(node=out.node.cpu().numpy(), status=out.status.cpu().numpy(), start=out.start_tick.cpu().numpy(),
                 done=out.done_tick.cpu().numpy(), stats=out.rep_stats())
        assert (g["stats"]["status"] == 0).all()
        assert_parity(tr, g, o)
        assert out.rep_stats().tobytes() == o["stats"].tobytes()
        np.testing.assert_array_equal(out.node_energy.cpu().numpy(), o["node_energy"])
        np.testing.assert_array_equal(out.hist.cpu().numpy(), o["hist"].sum(axis=0))


@pytest.mark.parametrize("resume", ["1", "0"])
def test_hier_resume_at_first_escalation(ctx, monkeypatch, resume):
    """EXT_HIER resume (replay_region.hip): twelve replications whose 6-node second region
    takes most publishes from a replication-specific point on, so each escalates first at a
    different publish (116 .. 1,589 in the oracle: anywhere in a 64-publish chunk, early and
    late); the second region pass stops every region exactly before it and the sequential
    kernel continues from there.  Outputs, records, per-node energy and the job histogram
    equal the oracle's, as with FOGNET_HIER_RESUME=0 (restart from the first publish)."""
    R, N, T = 12, 1030, 3000
    tr = tg.make_batch(33, R, N, T, rho=0.01)
    reg = np.zeros_like(tr["req"])
    rng = np.random.default_rng(5)
    for r, s0 in enumerate([0, 0, 0, 0, 0, 0, 200, 400, 600, 800, 1000, 1500]):
        reg[r, s0:][rng.random(T - s0) < 0.5 + 0.04 * r] = 1
    pb, pi = fa.power_model(tr["mips"])
    tr = dict(tr, region=reg, p_busy=pb, p_idle=pi)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8, hist=True,
                     policy=ol.POLICY_EXT_HIER, region=reg, hier_threshold_s=0, hier_up_tick=10**11,
                     p_busy=pb, p_idle=pi)
    esc = o["node"] // _abi.HIER_REGION_NODES != reg
    first = np.where(esc.any(axis=1), esc.argmax(axis=1), -1)
    assert (first > 0).all() and first.min() < 200 and len(set((first % 64).tolist())) > 6
    monkeypatch.setenv("FOGNET_HIER_REGIONS", "1")
    monkeypatch.setenv("FOGNET_HIER_RESUME", resume)
    out = fa.run_batch(ctx, fa.as_device_trace(tr, torch.device("cuda", ctx.device)), policy="EXT_HIER",
                       hier_threshold_s=0, hier_up_tick=10**11, hist=True)
    torch.cuda.synchronize()
    st = out.rep_stats()
    g = dict(node=out.node.cpu().numpy(), status=out.status.cpu().numpy(), start=out.start_tick.cpu().numpy(),
             done=out.done_tick.cpu().numpy(), stats=st)
    assert (st["status"] == 0).all()
    assert_parity(tr, g, o)
    assert st.tobytes() == o["stats"].tobytes()
    np.testing.assert_array_equal(out.node_energy.cpu().numpy(), o["node_energy"])
    np.testing.assert_array_equal(out.hist.cpu().numpy(), o["hist"].sum(axis=0))


@pytest.mark.parametrize("thr,up_s", [(0, 1), (3, 2), (0, 40), (2, 300)])
def test_hier_overtaken_escalation_matches_oracle(ctx, thr, up_s):
    """EXT_HIER: publishes alternating between a saturated 6-node region and a
    1024-node one, so escalated tasks (+1 s / +2 s hop) to the global argmin are
    overtaken by the other region's direct tasks to the same node.  The node
    serves in arrival order; the device defers each escalated task until the
    tasks that reach its node first are pushed, and equals the oracle (a DES)
    bit for bit, statistics included."""
    tr = tg.make_batch(21, 6, 1030, 4000, rho=0.9)
    reg = np.zeros_like(tr["req"])
    reg[:, 1::2] = 1
    tr = dict(tr, region=reg)
    up = up_s * 10**12
    dev = torch.device("cuda", ctx.device)
    out = fa.run_batch(ctx, fa.as_device_trace(tr, dev), policy="EXT_HIER", hier_threshold_s=thr, hier_up_tick=up,
                       hist=True)
    torch.cuda.synchronize()
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=6, hist=True,
                     policy=ol.POLICY_EXT_HIER, region=reg, hier_threshold_s=thr, hier_up_tick=up)
    inverted = []
    for r in range(tr["req"].shape[0]):  # the oracle served a later-decided task first somewhere
        node, start = o["node"][r], o["start"][r]
        inverted.append(any((np.diff(start[node == k]) < 0).any() for k in np.unique(node)))
    assert any(inverted), "the trace no longer provokes an overtaken escalation"
    g = dict(node=out.node.cpu().numpy(), status=out.status.cpu().numpy(), start=out.start_tick.cpu().numpy(),
             done=out.done_tick.cpu().numpy(), stats=out.rep_stats())
    assert (g["stats"]["status"] == 0).all()
    assert_parity(tr, g, o)
    assert out.rep_stats().tobytes() == o["stats"].tobytes()
    np.testing.assert_array_equal(out.hist.cpu().numpy(), o["hist"].sum(axis=0))


def escalations_in_flight(tr, o, region, up):
    """Most escalated tasks in flight at once in the oracle's run: decided (publish
    tick t) and not yet arrived (t + dl + hop) at some publish tick."""
    most = 0
    for r in range(tr["req"].shape[0]):
        t = tr["arrive"][r]
        node = o["node"][r]
        esc = node // _abi.HIER_REGION_NODES != region[r]
        dl = np.asarray(tr["dl"])[r] if np.ndim(tr["dl"]) == 2 else np.asarray(tr["dl"])
        a_esc = np.sort(t[esc] + dl[node[esc]] + up)
        t_esc = t[esc]
        # at publish tick x: escalations decided at or before x whose arrival is after x
        for x in t_esc:
            most = max(most, int(np.searchsorted(t_esc, x, side="right") - np.searchsorted(a_esc, x, side="right")))
    return most


@pytest.mark.parametrize("up_s", [1000, 90])
def test_hier_pending_escalations_spill_to_hbm(ctx, up_s):
    """More than 64 escalated tasks in flight at once (every publish escalated,
    a 90-s / 1000-s hop): past the 64 LDS slots they wait in the HBM overflow
    list, and the replay equals the oracle (whose node FIFO takes any length,
    ComputeBrokerApp3.cc:305-309) bit for bit, statistics included."""
    tr = tg.make_batch(22, 3, 1030, 4000, rho=0.9)
    reg = np.ones_like(tr["req"])  # region 1: 6 nodes, soon all advertising busy > 0
    tr = dict(tr, region=reg)
    up = up_s * 10**12
    out = fa.run_batch(ctx, fa.as_device_trace(tr, torch.device("cuda", ctx.device)), policy="EXT_HIER",
                       hier_threshold_s=0, hier_up_tick=up, hist=True)
    torch.cuda.synchronize()
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=3, hist=True,
                     policy=ol.POLICY_EXT_HIER, region=reg, hier_threshold_s=0, hier_up_tick=up)
    assert escalations_in_flight(tr, o, reg, up) > 64, "the trace no longer spills past the LDS slots"
    g = dict(node=out.node.cpu().numpy(), status=out.status.cpu().numpy(), start=out.start_tick.cpu().numpy(),
             done=out.done_tick.cpu().numpy(), stats=out.rep_stats())
    assert (g["stats"]["status"] == 0).all()
    assert_parity(tr, g, o)
    assert out.rep_stats().tobytes() == o["stats"].tobytes()
    np.testing.assert_array_equal(out.hist.cpu().numpy(), o["hist"].sum(axis=0))


@pytest.mark.parametrize("mode", ["only", "0"])
def test_c5_ext_hier_as_named(ctx, monkeypatch, mode):
    """Config C5 as BASELINE.json configs[4] names it, in the bench's settings:
    N = 10,000 fog nodes in 10 regional brokers (every rotated-lane row of the
    wide kernel), fa.mobility_regions handoffs, T = 10,000 device-generated
    publishes (C5 recipe), 60-s escalation threshold, 20-ms hop; every output,
    record and histogram bin against the oracle.  At this size no publish is
    escalated -- in the oracle either: a regional broker escalates only when every
    node of its region (784-1,024) advertises more than the threshold, a node
    advertises only after a completion, and the stale view herds a region's
    publishes onto one node until that node's first advert, so ~1,000 publishes
    per region touch a few dozen nodes; escalations, overtaking and the overflow
    list are covered at smaller regions (test_hier_*).  mode "only": the region
    pass alone (one wavefront per regional broker, replay_region.hip, no
    sequential hand-over); "0": the sequential wide kernel alone."""
    monkeypatch.setenv("FOGNET_HIER_REGIONS", mode)
    R, T, N = 4, 10_000, 10_000
    mg, sc = fa.c5_params(np.arange(R), N)
    d = fa.generate_trace(ctx, 0x5EED0005, R, T, N, mg, sc)
    d["region"] = fa.mobility_regions(d["arrive"], N)
    thr, up = 60, 20 * 10**9
    out = fa.run_batch(ctx, d, policy="EXT_HIER", hier_threshold_s=thr, hier_up_tick=up, hist=True)
    torch.cuda.synchronize()
    h = {k: d[k].cpu().numpy() for k in ("arrive", "req", "mips", "dl", "ul", "init", "region")}
    assert len(np.unique(h["region"])) == 10
    o = ol.run_batch(h["arrive"], h["req"], h["mips"], h["dl"], h["ul"], h["init"], threads=4, hist=True,
                     policy=ol.POLICY_EXT_HIER, region=h["region"], hier_threshold_s=thr, hier_up_tick=up)
    g = dict(node=out.node.cpu().numpy(), status=out.status.cpu().numpy(), start=out.start_tick.cpu().numpy(),
             done=out.done_tick.cpu().numpy(), stats=out.rep_stats())
    assert (g["stats"]["status"] == 0).all() and (g["stats"]["n_tasks"] == T).all()
    assert_parity(h, g, o)
    assert out.rep_stats().tobytes() == o["stats"].tobytes()
    np.testing.assert_array_equal(out.hist.cpu().numpy(), o["hist"].sum(axis=0))
    assert (o["node"] // _abi.HIER_REGION_NODES == h["region"]).all()  # (no escalation, see above)
    # every region's broker placed tasks
    assert len(np.unique(o["node"] // _abi.HIER_REGION_NODES)) == 10


@pytest.fixture(scope="module")
def c5_saturated():
    """Eight C5-topology replications (N = 10,000 in 10 regions, mobility_regions,
    T = 32,768) of fa.saturating_trace: six saturate every region and escalate
    (~7,900 publishes each, from all ten regional brokers, to the parent's
    global argmin in rows 0 and 3-8 of the wide kernel), two stay below the
    threshold.  The oracle run (power model, histograms) is shared."""
    R, T, N = 8, 32_768, 10_000
    tr = fa.saturating_trace(11, R, T, N, escalate=[True] * 6 + [False] * 2)
    pb, pi = fa.power_model(tr["mips"])
    tr = dict(tr, p_busy=pb, p_idle=pi)
    o = ol.run_batch(tr["arrive"], tr["req"], tr["mips"], tr["dl"], tr["ul"], tr["init"], threads=8, hist=True,
                     policy=ol.POLICY_EXT_HIER, region=tr["region"], hier_threshold_s=60, hier_up_tick=20 * 10**9,
                     p_busy=pb, p_idle=pi)
    return tr, o


def test_c5_saturated_trace_escalates_everywhere(c5_saturated):
    """The oracle's side of the escalation tests below: escalations originate in
    every region (rows 0-9 of the wide kernel's rotated lanes), land in rows 0
    and 3..8 (the parent's smallest advertised giant, placed in region 3 + r %
    7), and the non-escalating replications none."""
    tr, o = c5_saturated
    reg, node = tr["region"], o["node"]
    esc = node // _abi.HIER_REGION_NODES != reg
    n_esc = esc.sum(axis=1)
    assert (n_esc[:6] > 5000).all() and (n_esc[6:] == 0).all()
    assert set(np.unique(reg[esc])) == set(range(10))
    dest = set(np.unique(node[esc] // _abi.HIER_REGION_NODES))
    assert {3, 4, 5, 6, 7, 8} <= dest
    for r in range(6):
        assert (3 + r % 7) in set(np.unique(node[r][esc[r]] // _abi.HIER_REGION_NODES))
    assert (o["stats"]["status"] == 0).all() and (o["stats"]["n_qtime_overflow"] == 0).all()


@pytest.mark.parametrize("mode", ["1", "1-restart", "0", "only"])
def test_c5_ext_hier_escalations(ctx, monkeypatch, c5_saturated, mode):
    """EXT_HIER at the C5 topology WITH escalations: every
    output, record (a11 energy included), per-node energy and histogram bin
    against the oracle.  mode "1" (default): the region pass finishes the two
    non-escalating replications; the six others are replayed again by a second
    region pass up to their first escalated publish (past publish 16,000 here),
    whose state the sequential wide kernel continues from (resume: regional argmin
    per region, BrokerBaseApp3.cc:267-281; node FIFO of any length,
    ComputeBrokerApp3.cc:305-309; escalated tasks of all ten rows); "1-restart"
    (FOGNET_HIER_RESUME=0): the sequential kernel replays the six from the start;
    "0": the sequential kernel for all eight; "only": the region pass alone -- the
    two finished replications equal the oracle, the six others report
    FOGNET_ERR_UNSUPPORTED."""
    tr, o = c5_saturated
    monkeypatch.setenv("FOGNET_HIER_REGIONS", mode.split("-")[0])
    if mode == "1-restart":
        monkeypatch.setenv("FOGNET_HIER_RESUME", "0")
    else:
        monkeypatch.delenv("FOGNET_HIER_RESUME", raising=False)
    dev = torch.device("cuda", ctx.device)
    out = fa.run_batch(ctx, fa.as_device_trace(tr, dev), policy="EXT_HIER", hier_threshold_s=60,
                       hier_up_tick=20 * 10**9, hist=True)
    torch.cuda.synchronize()
    st = out.rep_stats()
    g = dict(node=out.node.cpu().numpy(), status=out.status.cpu().numpy(), start=out.start_tick.cpu().numpy(),
             done=out.done_tick.cpu().numpy(), stats=st)
    energy = out.node_energy.cpu().numpy()
    if mode == "only":
        assert list(st["status"]) == [_abi.FOGNET_ERR_UNSUPPORTED] * 6 + [0, 0]
        keep = slice(6, 8)
        for k in ("node", "status", "start", "done"):
            np.testing.assert_array_equal(g[k][keep], o[k][keep], err_msg=k)
        assert st[keep].tobytes() == o["stats"][keep].tobytes()
        np.testing.assert_array_equal(energy[keep], o["node_energy"][keep])
        np.testing.assert_array_equal(out.hist.cpu().numpy(), o["hist"][keep].sum(axis=0))
        return
    assert (st["status"] == 0).all()
    assert_parity(tr, g, o)
    assert st.tobytes() == o["stats"].tobytes()
    np.testing.assert_array_equal(energy, o["node_energy"])
    np.testing.assert_array_equal(out.hist.cpu().numpy(), o["hist"].sum(axis=0))


@pytest.mark.parametrize("resume", [True, False])
def test_c5_ext_hier_automatic_path(monkeypatch, c5_saturated, resume):
    """FOGNET_HIER_REGIONS unset (the default).  With resume (the default) every
    launch takes the region pass: an escalated replication continues on the
    sequential kernel from its first escalated publish, so the pass is never
    wasted.  With FOGNET_HIER_RESUME=0 the first launch takes the region pass,
    which hands six of the eight replications over; once that count has reached
    the host, the next launch goes straight to the sequential replay
    (fognet_hier_path_stats).  Every output, record, per-node energy and histogram
    equals the oracle on both launches.  A light C5 trace (no escalation) keeps
    the region pass."""
    tr, o = c5_saturated
    monkeypatch.delenv("FOGNET_HIER_REGIONS", raising=False)
    if resume:
        monkeypatch.delenv("FOGNET_HIER_RESUME", raising=False)
    else:
        monkeypatch.setenv("FOGNET_HIER_RESUME", "0")
    c = fa.Context(0)  # (a fresh context: the measurement is per context)
    dev = torch.device("cuda", c.device)
    d = fa.as_device_trace(tr, dev)
    for launch in range(2):
        out = fa.run_batch(c, d, policy="EXT_HIER", hier_threshold_s=60, hier_up_tick=20 * 10**9, hist=True)
        torch.cuda.synchronize()
        assert c.hier_path_stats() == ((1, 0) if launch == 0 else (2, 0) if resume else (1, 1))
        st = out.rep_stats()
        g = dict(node=out.node.cpu().numpy(), status=out.status.cpu().numpy(), start=out.start_tick.cpu().numpy(),
                 done=out.done_tick.cpu().numpy(), stats=st)
        assert (st["status"] == 0).all()
        assert_parity(tr, g, o)
        assert st.tobytes() == o["stats"].tobytes()
        np.testing.assert_array_equal(out.node_energy.cpu().numpy(), o["node_energy"])
        np.testing.assert_array_equal(out.hist.cpu().numpy(), o["hist"].sum(axis=0))
    R, T, N = 4, 10_000, 10_000
    mg, sc = fa.c5_params(np.arange(R), N)
    light = fa.generate_trace(c, 0x5EED0005, R, T, N, mg, sc)
    light["region"] = fa.mobility_regions(light["arrive"], N)
    # another job (shape) on the same context is measured afresh, not sent to the sequential replay on the
    # strength of the saturated job's count (the decision is paired with the launch it measured)
    fa.run_batch(c, light, policy="EXT_HIER", hier_threshold_s=60, hier_up_tick=20 * 10**9)
    torch.cuda.synchronize()
    assert c.hier_path_stats() == ((3, 0) if resume else (2, 1))
    c2 = fa.Context(0)
    for _ in range(2):
        fa.run_batch(c2, light, policy="EXT_HIER", hier_threshold_s=60, hier_up_tick=20 * 10**9)
        torch.cuda.synchronize()
    assert c2.hier_path_stats() == (2, 0)
    c.close()
    c2.close()


@pytest.mark.parametrize("kind", ["ext_hier", "long"])
def test_generated_wide_paths_equal_materialized(ctx, kind):
    """Generated replays the register kernel does not take run on the wide
    kernel, with the trace still computed in the kernel: EXT_HIER (each
    publish's region from fa.mobility_regions' model, in the kernel; N = 1,030:
    a 6-node second region that saturates, threshold 0, so it escalates) and requirement ranges with
    T * req_hi / 1000 >= 2^32 (round 4 refused them: the register kernel's node
    totals are 32-bit; any task of more than 255 s leaves that kernel anyway, and
    at N = 16 such traces run past 2^61 ticks, so both paths report the same
    FOGNET_ERR_ARG record).  Records, histograms and per-node energy equal
    fognet_gen_trace_dev + the materialised replay bit for bit."""
    dev = torch.device("cuda", ctx.device)
    if kind == "ext_hier":
        R, T, N, seed, rq, kw = 6, 12000, 1030, 0x5EED0007, (1000, 64000), dict(hier_threshold_s=0, hier_up_tick=10**12)
        mg, sc = fa.sweep_params(np.arange(R), N, rho=0.9)
        pol = "EXT_HIER"
    else:
        R, T, N, seed, rq, kw = 2, 2100, 16, 0x5EED0008, (1000, 2_100_000_000), {}
        assert T * (rq[1] // 1000) >= 2**32
        mg, sc = fa.sweep_params(np.arange(R), N, req_lo=rq[0], req_hi=rq[1])
        pol = "REF_V3"
    tr = fa.generate_trace(ctx, seed, R, T, N, mg, sc, req_lo=rq[0], req_hi=rq[1])
    pb, pi = fa.power_model(tr["mips"].cpu().numpy())
    power = (torch.from_numpy(pb).to(dev), torch.from_numpy(pi).to(dev))
    tr = {k: v for k, v in tr.items() if not k.startswith("_")}
    tr["p_busy"], tr["p_idle"] = power
    if pol == "EXT_HIER":
        tr["region"] = fa.mobility_regions(tr["arrive"], N)
    ref = fa.run_batch(ctx, tr, policy=pol, hist=True, **kw)
    gen = fa.run_generated(ctx, seed, R, T, N, mg, sc, req_lo=rq[0], req_hi=rq[1], policy=pol, power=power,
                           hist=True, energy=True, **kw)
    torch.cuda.synchronize()
    st = ref.rep_stats()
    if pol == "EXT_HIER":  # the regional brokers escalate somewhere
        assert (st["status"] == 0).all()
        node, reg = ref.node.cpu().numpy(), tr["region"].cpu().numpy()
        assert (node // _abi.HIER_REGION_NODES != reg).any()
    else:
        assert (st["status"] == _abi.FOGNET_ERR_ARG).all()
    assert gen.rep_stats().tobytes() == st.tobytes()
    assert torch.equal(gen.hist, ref.hist) and torch.equal(gen.node_energy, ref.node_energy)
