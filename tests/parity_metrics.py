"""Parity metrics of SURVEY.md §8(d), shared by the tests (conftest) and
tools/parity_report.py.

* scale-relative error: max_f |s_f - r_f| / max_f |r_f| -- the bar (1e-5);
* per-element relative error |s_f - r_f| / |r_f| on the features whose
  reference score is not small: |r_f| >= 1e-3 * max|r| (the band §8(d)
  names) and >= 1e-2 * max|r| -- reported beside the bar: the count of
  such features, the fraction over 1e-5 and the maximum;
* top-k index-set agreement.
"""
from __future__ import annotations

import numpy as np


def scale_rel_err(a, ref) -> float:
    a = np.asarray(a, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    den = np.abs(ref).max() if ref.size else 0.0
    if den == 0.0:
        return float(np.abs(a).max()) if a.size else 0.0
    return float(np.abs(a - ref).max() / den)


def per_element(a, ref, floor: float, rtol: float = 1e-5) -> dict:
    """Per-element relative error on the features with |ref| >= floor *
    max|ref|: n (how many), over (fraction above rtol), max."""
    a = np.asarray(a, dtype=np.float64)
    ref = np.asarray(ref, dtype=np.float64)
    top = np.abs(ref).max() if ref.size else 0.0
    sel = np.abs(ref) >= floor * top if top > 0 else np.zeros(ref.shape, bool)
    if not sel.any():
        return {"n": 0, "over": 0.0, "max": 0.0}
    r = np.abs(a[sel] - ref[sel]) / np.abs(ref[sel])
    return {"n": int(sel.sum()), "over": float((r > rtol).mean()), "max": float(r.max())}


def topk_same(a, ref, k: int) -> bool:
    ta = set(np.argsort(np.asarray(a))[::-1][:k].tolist())
    tr = set(np.argsort(np.asarray(ref))[::-1][:k].tolist())
    return ta == tr


def summary(a, ref, rtol: float = 1e-5) -> str:
    """One line: scale-relative error and the per-element figures."""
    e3, e2 = per_element(a, ref, 1e-3, rtol), per_element(a, ref, 1e-2, rtol)
    return (f"scale-rel {scale_rel_err(a, ref):.2e} | per-element (|r|>=1e-3 max: n={e3['n']}, "
            f">1e-5 {100 * e3['over']:.1f}%, max {e3['max']:.2e}) (|r|>=1e-2 max: n={e2['n']}, "
            f">1e-5 {100 * e2['over']:.1f}%, max {e2['max']:.2e})")
