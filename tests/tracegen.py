"""Synthetic trace generator, numpy restatement (test infrastructure).

This is the CPU twin of the device generator in
``fognetsimpp_amd/csrc/tracegen.hip``: both implement the same integer-exact
recipe (Philox4x32-10 counters, a fixed IEEE-only ``-ln(u)``), so a trace made
on the GPU can be checked element-for-element against this file.

Recipe:
  * replication ``r`` uses Philox key ``(seed, r)``;
  * node ``j``: counter ``(j, 1, 0, 0)``; ``dl = (1e6 + x0 % (1e9 - 1e6 + 1)) * lat_scale``,
    ``ul`` likewise from ``x1``; ``mips = 1000 * (1 + j % 4)``
    (the simulations/testing/wireless5.ini:116-119 pattern); the initial
    advertisement reaches the broker at ``init = ul`` (sent at t = 0);
  * task ``i``: counter ``(i, 0, 0, 0)``; ``req = req_lo + x0 % (req_hi - req_lo + 1)``;
    ``u = ((x1 << 21) | (x2 >> 11)) + 1) * 2**-53`` in (0, 1];
    ``gap = trunc(mean_gap_ticks * -ln(u))``;
    ``arrive[0] = max(init) + 1 + gap[0]``, ``arrive[i] = arrive[i-1] + gap[i]``.
"""
from __future__ import annotations

import numpy as np

TICKS_PER_SECOND = 10**12

M0 = np.uint64(0xD2511F53)
M1 = np.uint64(0xCD9E8D57)
W0 = np.uint32(0x9E3779B9)
W1 = np.uint32(0xBB67AE85)
MASK32 = np.uint64(0xFFFFFFFF)

LN2 = 0.6931471805599453


def philox4x32_10(c0, c1, c2, c3, k0, k1):
    """Vectorised Philox4x32-10 on uint32 arrays (broadcasting)."""
    c0, c1, c2, c3 = (np.asarray(x, dtype=np.uint32) for x in (c0, c1, c2, c3))
    k0 = np.asarray(k0, dtype=np.uint32)
    k1 = np.asarray(k1, dtype=np.uint32)
    c0, c1, c2, c3, k0, k1 = np.broadcast_arrays(c0, c1, c2, c3, k0, k1)
    c0, c1, c2, c3, k0, k1 = (x.copy() for x in (c0, c1, c2, c3, k0, k1))
    with np.errstate(over="ignore"):
        for _ in range(10):
            p0 = M0 * c0.astype(np.uint64)
            p1 = M1 * c2.astype(np.uint64)
            hi0 = (p0 >> np.uint64(32)).astype(np.uint32)
            lo0 = (p0 & MASK32).astype(np.uint32)
            hi1 = (p1 >> np.uint64(32)).astype(np.uint32)
            lo1 = (p1 & MASK32).astype(np.uint32)
            c0, c1, c2, c3 = hi1 ^ c1 ^ k0, lo1, hi0 ^ c3 ^ k1, lo0
            k0 = k0 + W0
            k1 = k1 + W1
    return c0, c1, c2, c3


def neg_log_unit(u):
    """-ln(u) for u in (0, 1] using only IEEE +,-,*,/ (bit-reproducible on the GPU)."""
    u = np.asarray(u, dtype=np.float64)
    bits = u.view(np.uint64)
    e = ((bits >> np.uint64(52)) & np.uint64(0x7FF)).astype(np.int64) - 1023
    m = ((bits & np.uint64(0x000FFFFFFFFFFFFF)) | np.uint64(0x3FF0000000000000)).view(np.float64)
    big = m > 1.4142135623730951
    m = np.where(big, m * 0.5, m)
    e = np.where(big, e + 1, e)
    f = (m - 1.0) / (m + 1.0)
    f2 = f * f
    # atanh series: ln(m) = 2 (f + f^3/3 + ... + f^21/21), Horner in f2
    acc = np.full_like(f, 1.0 / 21.0)
    for k in (19, 17, 15, 13, 11, 9, 7, 5, 3):
        acc = acc * f2 + (1.0 / k)
    acc = acc * f2 + 1.0
    ln_m = 2.0 * f * acc
    ln_u = e.astype(np.float64) * LN2 + ln_m
    return -ln_u


def gen_nodes(seed: int, r: int, n: int, lat_scale: int = 1):
    j = np.arange(n, dtype=np.uint64)
    x0, x1, _, _ = philox4x32_10(j.astype(np.uint32), 1, 0, 0, seed & 0xFFFFFFFF, r & 0xFFFFFFFF)
    span = np.uint64(10**9 - 10**6 + 1)
    dl = (np.uint64(10**6) + x0.astype(np.uint64) % span).astype(np.int64) * lat_scale
    ul = (np.uint64(10**6) + x1.astype(np.uint64) % span).astype(np.int64) * lat_scale
    mips = (1000 * (1 + (np.arange(n) % 4))).astype(np.int32)
    init = ul.copy()
    return mips, dl, ul, init


def gen_tasks(seed: int, r: int, t: int, mean_gap_ticks: float, start_tick: int,
              req_lo: int = 1000, req_hi: int = 64000):
    i = np.arange(t, dtype=np.uint64)
    x0, x1, x2, _ = philox4x32_10(i.astype(np.uint32), 0, 0, 0, seed & 0xFFFFFFFF, r & 0xFFFFFFFF)
    req = (np.uint64(req_lo) + x0.astype(np.uint64) % np.uint64(req_hi - req_lo + 1)).astype(np.int32)
    k53 = (x1.astype(np.uint64) << np.uint64(21)) | (x2.astype(np.uint64) >> np.uint64(11))
    u = (k53 + np.uint64(1)).astype(np.float64) * (2.0 ** -53)
    gap = (float(mean_gap_ticks) * neg_log_unit(u)).astype(np.int64)
    arrive = np.int64(start_tick) + np.cumsum(gap, dtype=np.int64)
    return arrive, req


def mean_service_seconds(mips, req_lo=1000, req_hi=64000):
    return 0.5 * (req_lo + req_hi) * float(np.mean(1.0 / np.asarray(mips, dtype=np.float64)))


def make_replication(seed: int, r: int, n: int, t: int, rho: float = 0.8, lat_scale: int = 1,
                     req_lo: int = 1000, req_hi: int = 64000, mean_gap_ticks: float | None = None):
    mips, dl, ul, init = gen_nodes(seed, r, n, lat_scale)
    if mean_gap_ticks is None:
        mean_gap_ticks = mean_service_seconds(mips, req_lo, req_hi) / (n * rho) * TICKS_PER_SECOND
    start = int(init.max()) + 1
    arrive, req = gen_tasks(seed, r, t, mean_gap_ticks, start, req_lo, req_hi)
    return dict(arrive=arrive, req=req, mips=mips, dl=dl, ul=ul, init=init)


def make_batch(seed: int, R: int, n: int, t: int, rho=0.8, lat_scale=1, sweep=False, **kw):
    """R replications stacked SoA: arrive[R,T], req[R,T], node params [R,N]."""
    reps = []
    for r in range(R):
        if sweep:
            rho_r = (0.5, 0.8, 0.95)[r % 3]
            sc = (1, 10, 100)[(r // 3) % 3]
        else:
            rho_r, sc = rho, lat_scale
        reps.append(make_replication(seed, r, n, t, rho_r, sc, **kw))
    return {k: np.stack([rp[k] for rp in reps]) for k in reps[0]}
