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


def main():
    cases = []
    for name, (arrive, req, start, done, status, raws) in (
            ("round_trip", case_round_trip(2**54)), ("same_tick", case_same_tick()),
            ("overflow", case_overflow()), ("late_ticks", case_round_trip(2**60 + 1000))):
        rec = [r for r in raws if r is not None]
        cases.append(dict(
            name=name, arrive=arrive, req=req, mips=[1000], dl=[MS], ul=[MS], init=[MS],
            expect=dict(node=[0] * len(arrive), status=status, start=start, done=done,
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
