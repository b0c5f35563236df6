"""Exact MultiSURF row means for the mean-correction tests.

mu_i = sum_j D_ij / (n - 1) with D_ij = sum_f |x_if - x_jf| * recip_f
(continuous) + [x_if != x_jf] (discrete) -- MultiSURF.py:177-193 -- from
per-column sorts and float64 prefix sums, O(p n log n) instead of O(n^2 p):
for a column sorted ascending, sample at position k with value v has
sum_j |v - v_j| = v (2k - n + 1) - 2 P_k + (T - v), P_k the sum of the values
before it (equal values contribute nothing either way, so tie order does not
matter).  This is the real-number mean the library's corrected quantised row
sums approximate (fs_colsort.hip); the reference's own float32 products move
it by ~1e-8 / sqrt(n p) relative.
"""
import numpy as np


def exact_row_means(X, recip, is_discrete):
    x = np.asarray(X, dtype=np.float32).astype(np.float64)
    n, p = x.shape
    s = np.zeros(n, dtype=np.float64)
    cont = np.flatnonzero(~np.asarray(is_discrete, dtype=bool))
    disc = np.flatnonzero(np.asarray(is_discrete, dtype=bool))
    k = np.arange(n, dtype=np.float64)[:, None]
    for c0 in range(0, cont.size, 256):
        cols = cont[c0:c0 + 256]
        xc = x[:, cols]
        order = np.argsort(xc, axis=0, kind="stable")
        v = np.take_along_axis(xc, order, axis=0)
        P = np.cumsum(v, axis=0) - v                     # exclusive prefix
        T = P[-1] + v[-1]
        sums = v * (2.0 * k - n + 1.0) - 2.0 * P + (T - v)
        out = np.empty_like(sums)
        np.put_along_axis(out, order, sums, axis=0)
        s += out @ np.asarray(recip, dtype=np.float32)[cols].astype(np.float64)
    for f in disc:
        _, inv, cnt = np.unique(x[:, f], return_inverse=True, return_counts=True)
        s += (n - cnt[inv]).astype(np.float64)
    return s / (n - 1)


def plan_row_means(job):
    """mu_i of a MultiSURF job after step(): (sum D_q - correction) / (n - 1) / SC."""
    rs = job.rowstats.cpu().numpy().reshape(-1, 3)
    sc = job.plan.calibration()["SC"]
    return (rs[:, 0] - rs[:, 2]) / (job.n - 1) / sc


def assert_means_exact(mu, exact, sc, *info):
    """Row means within 1e-2 of a quantum (sc integer units per scaled-diff
    unit) of the exact ones.  The binned round-3 correction was off by up to
    ~p / 3 quanta on heavy-tailed columns (every sample of a column in one
    bin).  The exact order leaves the float32 rounding of the terms and the
    order of samples whose 32-bit keys tie -- same q and eps within 2^-8 of a
    quantum on 32-bit operands, each such pair off by < 2^-7 quanta: measured
    <= 1e-4 quanta on ordinary data, 2.7e-3 on the crowded lognormal
    (a = 4) case, where thousands of samples share a handful of quanta."""
    err = np.max(np.abs(np.asarray(mu) - np.asarray(exact))) * sc
    assert err <= 1e-2, (err, *info)
