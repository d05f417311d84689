"""Generates tests/golden/kat_qtime.json: known answers for the queueTime value
the reference emits (ComputeBrokerApp3.cc:238, queueStartTime = simTime().dbl()
at :306, Request.cc:26).

The event traces (which task queues, when it starts) are hand-traced below;
the emitted value follows OMNeT++ 4.6's SimTime arithmetic at scale 1e-12,
restated here with Python floats (IEEE binary64, round to nearest), an
implementation independent of oracle/ and the kernels:
  dbl(t)          = float(t) * 1e-12
  SimTime(d)      = toInt64(1e12 * d)
  t * d           = toInt64(float(t) * d)
  toInt64(x)      = floor(x + 0.5), cRuntimeError when outside int64
  queueTime raw   = toInt64(float(now - SimTime(dbl(a))) * 1000.0)

Every case: one fog node of 1000 MIPS (int service time S = req / 1000 s),
dl = ul = 1 ms, the node's first advert lands before the first publish.

  round_trip  publishes at t0 (req 3000: S = 3 s) and t0 + 1 tick (req 1000),
              a1 = t0 + 1 + dl = 2^54 + 6.  Task 0 starts at its arrival a0
              (status 5), done d0 = a0 + 3e12; task 1 arrives at a1 < d0 and
              queues (status 4), starts at d0.  Exact wait d0 - a1 = 3e12 - 1
              ticks; float(a1) rounds to 2^54 + 8, so the reference's
              queueStartTime round trip gives a1 + 2 and the emitted value is
              1000 * (3e12 - 3).
  same_tick   publishes at t0 and t0 (req 500: S = 0, then req 2000), arrival
              a = 2^54 + 3.  Task 0 completes at its own arrival tick; task 1's
              arrival there was inserted first (dl >= S * 1e12 with S = 0) and
              queues; releaseResource pops it in the same tick: exact wait 0,
              the round trip gives a + 1, emitted raw -1000 (a negative queueTime).
  overflow    small ticks (the round trip is exact); task 0 req 9223000 (S =
              9223 s), tasks 1, 2 req 1000 one tick apart.  Task 1 waits
              9223 s - 1 tick: raw = toInt64(float(9223e12 - 1) * 1000) fits
              int64; task 2 waits 9224 s - 2 ticks: 9.224e18 > 2^63, the
              reference throws (cRuntimeError) and the emission is counted as
              an overflow, not recorded.
  late_ticks  the round_trip trace moved to ~2^60 ticks (13.3 days), where
              float(a) has an ulp of 256 ticks.
  two_nodes   the reference's abort point is the EARLIEST overflowing emission,
              not the lowest task index.  Two 1000-MIPS nodes; publishes at 50
              ms (req 1000: S = 1 s), 50 ms + 1 tick (req 9310000: 9310 s), 50 ms
              + 2 ticks (req 1000), all to node 0 (every advertised busy is 0,
              ties -> index 0).  Node 0 completes task 0 at a0 + 1 s and
              advertises busyTime 9311 (both queued tasks arrived), which reaches
              the broker 1 ms later; the publishes at 2 s (req 9300000: 9300 s)
              and 2 s + 1 tick (req 1000) go to node 1 (busy 0 < 9311).  Node 1's
              task 4 waits 9300 s - 1 tick and overflows at tick 2 s + 1 ms +
              9300 s, node 0's task 2 (waiting ~9311 s) only at 0.051 s + 1 s +
              9310 s: the abort is (node 1's tick, task 4).

Every case also records the abort point (abort_tick / abort_task: the first
RELEASERESOURCE whose queueTime emission throws, ComputeBrokerApp3.cc:238 with
no handler up to :84-86; null / -1 when the run completes) and the per-task
outputs of the reference-defined prefix (stop_start / stop_done: -1 for a
start or completion the aborted reference run never reaches; the aborting
completion itself is reached, its status-6 ack and busyTime update precede
the emit at :228-234).

Run: python tests/golden/make_kat_qtime.py  (rewrites the JSON next to it)
"""
import json
import math
import os

MS = 10**9
TPS = 10**12


def dbl(t):
    return float(t) * 1e-12


def to_int64(x):
    f = math.floor(x + 0.5)
    return int(f) if abs(f) < 2.0**63 else None


def qtime_raw(now, a):
    qs = to_int64(1e12 * dbl(a))
    return to_int64(float(now - qs) * 1000.0)


def case_round_trip(base):
    # t0 + 1 + dl = base + 6
    t0 = base + 5 - MS
    arrive = [t0, t0 + 1]
    req = [3000, 1000]
    a0, a1 = t0 + MS, t0 + 1 + MS
    d0 = a0 + 3 * TPS
    start = [a0, d0]
    done = [d0, d0 + 1 * TPS]
    return arrive, req, start, done, [5, 4], [qtime_raw(d0, a1)]


def case_same_tick():
    a = 2**54 + 3
    t0 = a - MS
    arrive = [t0, t0]
    req = [500, 2000]
    start = [a, a]
    done = [a, a + 2 * TPS]
    return arrive, req, start, done, [5, 4], [qtime_raw(a, a)]


def case_overflow():
    t0 = 50 * MS
    arrive = [t0, t0 + 1, t0 + 2]
    req = [9223000, 1000, 1000]
    a = [t + MS for t in arrive]
    d0 = a[0] + 9223 * TPS
    d1 = d0 + TPS
    start = [a[0], d0, d1]
    done = [d0, d1, d1 + TPS]
    return arrive, req, start, done, [5, 4, 4], [qtime_raw(d0, a[1]), qtime_raw(d1, a[2])]


def case_two_nodes():
    arrive = [50 * MS, 50 * MS + 1, 50 * MS + 2, 2 * TPS, 2 * TPS + 1]
    req = [1000, 9310000, 1000, 9300000, 1000]
    a = [t + MS for t in arrive]
    d0 = a[0] + TPS                  # task 0 (node 0, started at its arrival)
    d1 = d0 + 9310 * TPS             # task 1 starts at d0 (queued)
    d2 = d1 + TPS                    # task 2 starts at d1 (queued): waits ~9311 s
    d3 = a[3] + 9300 * TPS           # task 3 (node 1, idle)
    d4 = d3 + TPS                    # task 4 starts at d3 (queued): waits 9300 s - 1 tick
    start = [a[0], d0, d1, a[3], d3]
    done = [d0, d1, d2, d3, d4]
    # queueTime emissions in start order: task 1 at d0, task 4 at d3, task 2 at d1 (d3 < d1)
    return arrive, req, start, done, [5, 4, 4, 5, 4], [qtime_raw(d0, a[1]), qtime_raw(d3, a[4]), qtime_raw(d1, a[2])]


def main():
    cases = []
    for name, (arrive, req, start, done, status, raws) in (
            ("round_trip", case_round_trip(2**54)), ("same_tick", case_same_tick()),
            ("overflow", case_overflow()), ("late_ticks", case_round_trip(2**60 + 1000)),
            ("two_nodes", case_two_nodes())):
        rec = [r for r in raws if r is not None]
        n_nodes = 2 if name == "two_nodes" else 1
        node = [0, 0, 0, 1, 1] if name == "two_nodes" else [0] * len(arrive)
        # the abort point: the earliest queued task whose emission throws (start tick, then index)
        ovf = sorted((s_, i) for i, (s_, st) in enumerate(zip(start, status))
                     if st == 4 and qtime_raw(s_, arrive[i] + MS) is None)
        ab_tick, ab_task = ovf[0] if ovf else (None, -1)
        stop_start = [x if ab_tick is None or x < ab_tick else -1 for x in start]
        stop_done = [x if ab_tick is None or x <= ab_tick else -1 for x in done]
        if ab_tick is not None:  # the task the aborting emission belongs to never starts
            stop_start[ab_task] = -1
        cases.append(dict(
            name=name, arrive=arrive, req=req, mips=[1000] * n_nodes, dl=[MS] * n_nodes, ul=[MS] * n_nodes,
            init=[MS] * n_nodes,
            expect=dict(node=node, status=status, start=start, done=done,
                        abort_tick=ab_tick, abort_task=ab_task, stop_start=stop_start, stop_done=stop_done,
                        qtime_raw=raws,  # per queued task in start order; null = the reference throws
                        n_qtime=len(rec), n_qtime_overflow=len(raws) - len(rec),
                        queue_sum=sum(rec), queue_sq=sum(r * r for r in rec),
                        queue_min=min(rec) if rec else None, queue_max=max(rec) if rec else None,
                        exact_wait_ticks=[s - (t + MS) for s, t, st in zip(start, arrive, status) if st == 4])))
    out = dict(source="tests/golden/make_kat_qtime.py (hand-traced events; OMNeT++ 4.6 SimTime ops restated "
                      "with Python floats)", cases=cases)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "kat_qtime.json"), "w") as f:
        json.dump(out, f, indent=1)
        f.write("\n")


if __name__ == "__main__":
    main()
