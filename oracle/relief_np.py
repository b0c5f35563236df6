"""Independent vectorised numpy restatement -- TEST INFRASTRUCTURE ONLY.

A second, differently structured restatement of the reference's CPU kernels
(row-at-a-time numpy broadcasting instead of scalar loops) used to cross-check
``relief_oracle.c`` on small inputs.  Same sources as the C oracle:
MultiSURF.py:165-253, ReliefF.py:137-220, SURF.py:131-195.  ReliefF ordering
uses the C oracle's numba-quicksort port only when ``numba_order`` is given;
otherwise a stable argsort (identical whenever the distance row has no ties).

Arrays are expected already preprocessed exactly as the reference ``fit`` does
(see ``oracle.py``): x in the kernel dtype, float32 recip, bool is_discrete.
"""
from __future__ import annotations

import numpy as np


def _diff_rows(x, i, recip, is_disc):
    """All diffs of focal sample i against every j, in the kernel's arithmetic."""
    if x.dtype == np.float32:
        cont = (np.abs(x[i][None, :] - x) * recip[None, :]).astype(np.float64)
    else:
        cont = np.abs(x[i][None, :] - x) * recip.astype(np.float64)[None, :]
    disc = (x[i][None, :] != x).astype(np.float64)
    return np.where(is_disc[None, :], disc, cont)


def multisurf(x32, y, recip, is_disc, use_star):
    n, p = x32.shape
    temp = np.zeros((n, p), dtype=np.float32)
    for i in range(n):
        d = _diff_rows(x32, i, recip, is_disc)           # (n, p) float64
        dist = d.sum(axis=1)
        others = np.arange(n) != i
        mu = dist[others].sum() / (n - 1)
        var = max(0.0, (dist[others] ** 2).sum() / (n - 1) - mu * mu)
        thr = mu - 0.5 * np.sqrt(var)
        hit = (y == y[i]) & others
        miss = (y != y[i]) & others
        near = dist < thr
        nh, nm = near & hit, near & miss
        hit_sum = d[nh].sum(axis=0)
        miss_sum = d[nm].sum(axis=0)
        if use_star:
            miss_sum = miss_sum - d[(~near) & miss].sum(axis=0)
        if nh.sum() > 0:
            hit_sum = hit_sum / nh.sum()
        if nm.sum() > 0:
            miss_sum = miss_sum / nm.sum()
        temp[i] = (miss_sum - hit_sum).astype(np.float32)
    return (temp.astype(np.float64).sum(axis=0) / n).astype(np.float32)


def relieff(x32, y_enc, recip, is_disc, k, class_probs, numba_order=None):
    n, p = x32.shape
    n_classes = class_probs.size
    temp = np.zeros((n, p), dtype=np.float32)
    for i in range(n):
        d = _diff_rows(x32, i, recip, is_disc)
        dists = d.sum(axis=1).astype(np.float32)
        dists[i] = np.inf
        order = numba_order(dists) if numba_order is not None else np.argsort(dists, kind="stable")
        lbl_i = y_enc[i]
        hits = [j for j in order if y_enc[j] == lbl_i][:k]
        denom = 1.0 - float(class_probs[lbl_i])
        if denom == 0:
            denom = 1.0
        upd = np.zeros(p)
        if hits:
            upd -= d[hits].sum(axis=0) / len(hits)
        for c in range(n_classes):
            if c == lbl_i:
                continue
            mc = [j for j in order if y_enc[j] == c][:k]
            if mc:
                upd += (float(class_probs[c]) / denom) * d[mc].sum(axis=0) / k
        temp[i] = upd.astype(np.float32)
    return (temp.astype(np.float64).sum(axis=0) / n).astype(np.float32)


def surf(x64, y_int, recip, is_disc, use_star):
    n, p = x64.shape
    temp = np.zeros((n, p), dtype=np.float64)
    for i in range(n):
        d = _diff_rows(x64, i, recip, is_disc).astype(np.float32).astype(np.float64)
        dist = _diff_rows(x64, i, recip, is_disc).sum(axis=1).astype(np.float32)
        dist[i] = 0.0
        s = np.float32(0.0)
        for v in dist:            # float32 sequential sum (SURF.py:162)
            s = np.float32(s + v)
        avg = float(s) / (n - 1)
        others = np.arange(n) != i
        hit = (y_int == y_int[i]) & others
        miss = (y_int != y_int[i]) & others
        near = dist.astype(np.float64) < avg
        upd = d[near & miss].sum(axis=0) - d[near & hit].sum(axis=0)
        if use_star:
            upd += d[(~near) & hit].sum(axis=0) - d[(~near) & miss].sum(axis=0)
        temp[i] = upd
    return (temp.sum(axis=0) / n).astype(np.float32)
