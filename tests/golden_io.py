"""Loaders for the hand-traced fixtures in tests/golden/ (test infrastructure)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _f(x):
    return float(x) if not isinstance(x, str) else float(x.replace("inf", "inf"))


def decide_cases():
    d = json.load(open(os.path.join(GOLDEN, "kat_decide.json")))
    out = []
    for c in d["cases"]:
        busy = np.array([_f(x) for x in c["busy"]], dtype=np.float64)
        mips = np.array(c["mips"], dtype=np.int32)
        out.append((c["name"], busy, mips, int(c["req"]), c.get("node"), c.get("error")))
    return out


def replay_cases():
    d = json.load(open(os.path.join(GOLDEN, "kat_replay.json")))
    out = []
    for c in d["cases"]:
        tr = dict(arrive=np.array(c["arrive"], np.int64), req=np.array(c["req"], np.int32),
                  mips=np.array(c["mips"], np.int32), dl=np.array(c["dl"], np.int64),
                  ul=np.array(c["ul"], np.int64), init=np.array(c["init"], np.int64))
        out.append((c["name"], tr, c["expect"]))
    return out


def decide_v2_cases():
    d = json.load(open(os.path.join(GOLDEN, "kat_decide_v2.json")))
    return [(c["name"], np.array(c["mips"], dtype=np.int32), int(c["local"]), int(c["req"]), int(c["action"]),
             int(c["node"])) for c in d["cases"]]


def replay_v2_cases():
    d = json.load(open(os.path.join(GOLDEN, "kat_replay_v2.json")))
    ms = d["ms"]
    out = []
    for c in d["cases"]:
        tr = dict(arrive=np.array(c["arrive_ms"], np.int64)[None] * ms, req=np.array(c["req"], np.int32)[None],
                  broker_mips=int(c["broker_mips"]), mips=np.array(c["mips"], np.int32),
                  dl=np.array(c["dl_ms"], np.int64) * ms, ul=np.array(c["ul_ms"], np.int64) * ms,
                  first_adv=np.array(c["first_adv_ms"], np.int64) * ms, stop=int(c["stop_ms"]) * ms)
        e = dict(c["expect"])
        e["start"] = [x * ms if x >= 0 else -1 for x in e.pop("start_ms")]
        e["done"] = [x * ms if x >= 0 else -1 for x in e.pop("done_ms")]
        out.append((c["name"], tr, e))
    return out


def replay_down_cases():
    d = json.load(open(os.path.join(GOLDEN, "kat_replay_down.json")))
    ms = d["ms"]
    never = np.iinfo(np.int64).max
    out = []
    for c in d["cases"]:
        tr = dict(arrive=np.array(c["arrive_ms"], np.int64) * ms, req=np.array(c["req"], np.int32),
                  mips=np.array(c["mips"], np.int32), dl=np.array(c["dl_ms"], np.int64) * ms,
                  ul=np.array(c["ul_ms"], np.int64) * ms, init=np.array(c["init_ms"], np.int64) * ms,
                  down=np.array([never if x is None else x * ms for x in c["down_ms"]], np.int64))
        e = dict(c["expect"])
        e["start"] = [x * ms if x >= 0 else -1 for x in e.pop("start_ms")]
        e["done"] = [x * ms if x >= 0 else -1 for x in e.pop("done_ms")]
        out.append((c["name"], tr, e))
    return out


def qtime_cases():
    """tests/golden/kat_qtime.json (make_kat_qtime.py): the reference's queueTime value."""
    d = json.load(open(os.path.join(GOLDEN, "kat_qtime.json")))
    out = []
    for c in d["cases"]:
        tr = dict(arrive=np.array(c["arrive"], np.int64)[None], req=np.array(c["req"], np.int32)[None],
                  mips=np.array(c["mips"], np.int32), dl=np.array(c["dl"], np.int64),
                  ul=np.array(c["ul"], np.int64), init=np.array(c["init"], np.int64))
        out.append((c["name"], tr, c["expect"]))
    return out


def check_qtime_record(st, exp):
    """Compare a fognet_rep_stats / orc_rep_stats record with a kat_qtime expectation."""
    assert st["status"] == 0
    assert int(st["n_qtime"]) == exp["n_qtime"] and int(st["n_qtime_overflow"]) == exp["n_qtime_overflow"]
    s = int(st["queue_sum_lo"]) | (int(st["queue_sum_hi"]) << 64)
    s = s - (1 << 128) if s >> 127 else s
    q = int(st["queue_sq_lo"]) | (int(st["queue_sq_hi"]) << 64) | (int(st["queue_sq_top"]) << 128)
    assert s == exp["queue_sum"] and q == exp["queue_sq"]
    if exp["queue_min"] is not None:
        assert int(st["queue_min_raw"]) == exp["queue_min"] and int(st["queue_max_raw"]) == exp["queue_max"]
    else:
        assert int(st["queue_min_raw"]) == np.iinfo(np.int64).max
    # the reference's abort point (first overflowing emission; fognet_hip.h)
    ab = np.iinfo(np.int64).max if exp["abort_tick"] is None else exp["abort_tick"]
    assert int(st["abort_tick"]) == ab and int(st["abort_task"]) == exp["abort_task"]


def general0_v2_node():
    """tests/golden/general0_v2_node.json (make_general0_fixture.py): the fog node
    of the reference's recorded example run (ComputeBrokerApp2 timing)."""
    d = json.load(open(os.path.join(GOLDEN, "general0_v2_node.json")))
    ms = 10**9
    arr_node = np.array(d["task_arrival_ticks"], np.int64)
    n = d["ini"]["nodes"]
    # The recorded broker is older code: the fixture feeds the node the
    # same four tasks by forwarding every publish (a broker pool of 0 MIPS) over a
    # 1-ms link; MIPSRequired 100 (the v1 user of that run, mqttApp.cc:330).
    tr = dict(arrive=(arr_node - ms)[None], req=np.full((1, len(arr_node)), 100, np.int32),
              broker_mips=0, mips=np.full(n, d["ini"]["node_mips"], np.int32), dl=np.full(n, ms, np.int64),
              ul=np.full(n, ms, np.int64), first_adv=np.full(n, d["connack_tick"] + 10 * ms, np.int64),
              stop=3_360_000_000_000)
    return tr, d
