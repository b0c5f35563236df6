"""SURF / SURF* on integer pass-1 distances (fs_surfint.hip, VERDICT r5
next #3): the float32 distances of SURF.py:146-160 recovered from 32-bit
quantised ones -- ambiguous pairs recomputed exactly where a row's float32
running sum (:162-163) or a near / far decision (:176) depends on them.

Both routes end with the same float32 distance for every pair, so every later
stage is the same computation: the integer route must give scores
BIT-IDENTICAL to the float64 route (the surf_f64 test hook) on ordinary and
adversarial data -- heavy tails, value grids, duplicated columns, near-equal
rows (distances near 0, where the band spans several float32 values), mixed
discrete columns -- in both accumulation modes, and to the oracle in
reference order (the surf_f64 hook forces each route).  On ordinary data
with enough features the automatic choice must be the integer route (plan
calibration [5] == 0), with pairs actually refined.
"""
import warnings

import numpy as np
import pytest
from sklearn.datasets import make_classification

from test_refacc import assert_bitexact

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    import fastselect_amd
    from fastselect_amd import _lib
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    return fastselect_amd


def _data(kind, n=1200, p=300, seed=5):
    rng = np.random.default_rng(seed)
    if kind == "classif":
        X, y = make_classification(n_samples=n, n_features=p, n_informative=12,
                                   n_redundant=20, random_state=seed)
        return X, y
    y = rng.integers(0, 2, n)
    if kind == "lognormal":
        X = np.exp(2.0 * rng.standard_normal((n, p)))
    elif kind == "grid":  # 41 levels: continuous for discrete_limit = 10, rounding coherent
        X = rng.integers(0, 41, (n, p)).astype(np.float64)
    elif kind == "dup":  # every column twice: errors add up in pairs
        h = rng.standard_normal((n, p // 2))
        X = np.concatenate([h, h], axis=1)
    elif kind == "neardup":  # rows 1e-12 apart: distances near 0
        X = rng.standard_normal((n, p))
        X[1::2] = X[0::2] + 1e-12 * rng.standard_normal((n // 2, p))
    elif kind == "mixed":
        X = rng.standard_normal((n, p))
        X[:, : p // 4] = rng.integers(0, 4, (n, p // 4))
    elif kind == "outlier":
        X = rng.standard_normal((n, p))
        X[rng.integers(0, n, p), np.arange(p)] = 1e7
    else:
        raise ValueError(kind)
    return X, y


def _fit(F, X, y, star, accumulation="fast"):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)
        est = F.SURF(backend="gpu", use_star=star, accumulation=accumulation)
        return np.asarray(est.fit(X, y).feature_importances_)


@pytest.mark.parametrize("kind", ["classif", "lognormal", "grid", "dup", "neardup", "mixed",
                                  "outlier"])
@pytest.mark.parametrize("star", [False, True])
def test_integer_route_is_the_float64_route(F, hooks, kind, star):
    X, y = _data(kind)
    hooks("surf_f64", 0)
    a = _fit(F, X, y, star)
    hooks("surf_f64", 1)
    b = _fit(F, X, y, star)
    assert_bitexact(a, b)


@pytest.mark.parametrize("kind", ["classif", "lognormal", "neardup", "mixed"])
def test_integer_route_reference_order_is_the_oracle(F, oracle, hooks, kind):
    hooks("surf_f64", 0)
    X, y = _data(kind, n=900, p=200, seed=11)
    for star in (False, True):
        assert_bitexact(_fit(F, X, y, star, "reference"),
                        oracle.surf_scores(X, y, use_star=star))


def test_ordinary_data_takes_the_integer_route(F, hooks):
    from fastselect_amd import _lib
    from fastselect_amd.SURF import surf_inputs
    X, y = _data("classif", n=2000, p=4000)
    isd, recip = surf_inputs(X, 10, "gpu")
    plans = {}
    for f64 in (-1, 1):  # automatic, then forced float64
        hooks("surf_f64", f64)
        plan = _lib.RowsPlan("gpu", "surf", np.ascontiguousarray(X), y.astype(np.int32), recip,
                             isd, use_star=True)
        import torch
        sums = torch.zeros(X.shape[1], dtype=torch.float64, device="cuda")
        torch.cuda.synchronize()
        plan.score(sums.data_ptr())
        plans[f64] = (plan.calibration(), plan.info()[2], sums.cpu().numpy())
        plan.close()
    cal, refined, s_int = plans[-1]
    assert not cal["surf_f64"] and cal["band_vs_model"] < 2.0, cal
    assert refined > 0  # some row sums depended on an ambiguous pair
    assert plans[1][0]["surf_f64"]
    assert_bitexact(s_int, plans[1][2])


def test_rows_slices_and_panels(F, hooks):
    from fastselect_amd import _lib
    from fastselect_amd.SURF import surf_inputs
    X, y = _data("classif", n=1500, p=250, seed=9)
    isd, recip = surf_inputs(X, 10, "gpu")
    yi = y.astype(np.int32)

    def run():
        out = [_lib.surf_score("gpu", X, yi, recip, True, isd, rows=(200, 1100))]
        hooks("row_panel", 256)
        out.append(_lib.surf_score("gpu", X, yi, recip, False, isd))
        hooks("row_panel", 0)
        return out

    hooks("surf_f64", 0)
    a = run()
    hooks("surf_f64", 1)
    b = run()
    for u, v in zip(a, b):
        assert_bitexact(u, v)


@pytest.mark.parametrize("parts", [2, 5])
def test_integer_route_k_split(F, hooks, parts):
    """SURF's integer route splits k_dist's tiles like MultiSURF's (the
    partial distance blocks merged by k_dist_merge, exact integers): forced
    K-splits give the float64 route's scores bit for bit, whole fit and a
    rows slice."""
    from fastselect_amd import _lib
    from fastselect_amd.SURF import surf_inputs
    X, y = _data("classif", n=1100, p=420, seed=13)
    isd, recip = surf_inputs(X, 10, "gpu")
    hooks("surf_f64", 1)
    ref = (_fit(F, X, y, True),
           _lib.surf_score("gpu", X, y.astype(np.int32), recip, True, isd, rows=(300, 700)))
    hooks("surf_f64", 0)
    hooks("ksplit", parts)
    got = (_fit(F, X, y, True),
           _lib.surf_score("gpu", X, y.astype(np.int32), recip, True, isd, rows=(300, 700)))
    for u, v in zip(got, ref):
        assert_bitexact(u, v)


@pytest.mark.parametrize("case", ["n2", "constant", "discrete", "single_class", "n129"])
def test_integer_route_edge_cases(F, hooks, case):
    """Edge inputs on the forced integer route against the float64 route:
    two samples, constant columns, an all-discrete layout (distances are
    mismatch counts, exact on both routes), one class, n = 129 (a
    one-sample second block)."""
    rng = np.random.default_rng(17)
    n, p = {"n2": (2, 6), "n129": (129, 40)}.get(case, (300, 50))
    X = rng.standard_normal((n, p))
    y = rng.integers(0, 2, n)
    if case == "constant":
        X[:, ::3] = 1.5
    elif case == "discrete":
        X = rng.integers(0, 3, (n, p)).astype(np.float64)
    elif case == "single_class":
        y = np.zeros(n, dtype=int)
    if case == "n2":
        y = np.array([0, 1])
    out = []
    for route in (0, 1):
        hooks("surf_f64", route)
        out.append([_fit(F, X, y, star) for star in (False, True)])
    for u, v in zip(*out):
        assert_bitexact(u, v)
