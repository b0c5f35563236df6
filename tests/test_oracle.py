"""Pin the parity oracle (oracle/) before trusting it.

1. The reference's own known-answer tests, re-run against the oracle on the
   reference's fixtures (tests/golden/reference_fixtures.npz):
   test_multisurf.py:36-45,96-110,193-205; test_relieff.py:36-63,98-111,195-207;
   test_surf.py:37-52,101-113,184-195.
2. The reference's MultiSURF output on the README dataset recorded in
   SURVEY.md §8c (top-15 set, max|score|).
3. Agreement with the independent numpy restatement (oracle/relief_np.py).
4. numba-quicksort argsort port properties (ReliefF.py:157).
"""
import json
import os

import numpy as np
import pytest
from conftest import scale_rel_err

GOLD = os.path.join(os.path.dirname(__file__), "golden")


@pytest.fixture(scope="module")
def fx():
    return dict(np.load(os.path.join(GOLD, "reference_fixtures.npz")))


def test_multisurf_kat_ranking(oracle, fx):
    s = oracle.multisurf_scores(fx["ms_x"], fx["ms_y"], discrete_limit=4)
    assert set(oracle.top_features(s, 1)) == {0}
    np.testing.assert_allclose(s[3], 0.0, atol=1e-7)


@pytest.mark.parametrize("star", [False, True])
def test_multisurf_kat_single_class(oracle, fx, star):
    s = oracle.multisurf_scores(fx["ms_x"], np.zeros(10), use_star=star)
    assert np.all(s <= 1e-7)


def test_relieff_kat_ranking(oracle, fx):
    s = oracle.relieff_scores(fx["rs_x"], fx["rs_y"], n_neighbors=1, discrete_limit=4)
    assert s[0] > s[1] and s[2] > s[1]
    np.testing.assert_allclose(s[3], 0.0)
    assert set(oracle.top_features(s, 2)) == {0, 2}
    s2 = oracle.relieff_scores(fx["rs_x"], fx["rs_y"], n_neighbors=1)
    np.testing.assert_allclose(s2[3], 0.0)


def test_relieff_kat_single_class(oracle, fx):
    s = oracle.relieff_scores(fx["rs_x"], np.zeros(6), n_neighbors=2)
    assert np.all(np.isfinite(s)) and np.all(s <= 0)


def test_surf_kat_ranking(oracle, fx):
    s = oracle.surf_scores(fx["rs_x"], fx["rs_y"], discrete_limit=3)
    assert s[0] > s[1] and s[2] > s[1]
    np.testing.assert_allclose(s[3], 0.0, atol=1e-7)
    assert set(oracle.top_features(s, 2)) == {0, 2}


def test_surf_kat_single_class(oracle, fx):
    s = oracle.surf_scores(fx["rs_x"], np.zeros(6))
    assert np.all(s <= 1e-7)


def test_discrete_limit_kat(oracle, fx):
    x = fx["dl_x"]
    np.testing.assert_array_equal(oracle.is_discrete_mask(x, 10), [False, True])
    np.testing.assert_array_equal(oracle.is_discrete_mask(x, 12), [True, True])


def test_cfg1_reference_output(oracle):
    """README quickstart data: reference top-15 and max|s| from SURVEY.md §8c."""
    import hashlib

    from sklearn.datasets import make_classification
    with open(os.path.join(GOLD, "cfg1_reference.json")) as f:
        ref = json.load(f)
    X, y = make_classification(n_samples=500, n_features=1000, n_informative=20,
                               n_redundant=100, random_state=42)
    assert hashlib.sha256(X.tobytes()).hexdigest()[:16] == ref["X_sha256_prefix"]
    assert int(y.sum()) == ref["y_sum"]
    s = oracle.multisurf_scores(X, y)
    assert sorted(oracle.top_features(s, 15).tolist()) == ref["top15"]
    assert abs(np.abs(s).max() - ref["max_abs_score"]) < 5e-4


def _prep(X, dtype, discrete_limit=10, force_disc_one=True):
    from oracle.oracle import is_discrete_mask
    x = X.astype(dtype)
    isd = is_discrete_mask(x, discrete_limit)
    r = x.max(0) - x.min(0)
    if force_disc_one:
        r[isd] = 1
    r[r == 0] = 1
    return x, isd, (1.0 / r).astype(np.float32)


@pytest.mark.parametrize("seed", [0, 1])
def test_oracle_matches_numpy_restatement(oracle, seed):
    from sklearn.datasets import make_classification

    from oracle import relief_np as N
    X, y = make_classification(n_samples=70, n_features=15, n_informative=5, n_redundant=2,
                               n_classes=2 + seed, n_clusters_per_class=1, random_state=seed)
    X[:, 0] = np.random.default_rng(seed).integers(0, 3, X.shape[0])
    X[:, 1] = 4.0
    for star in (False, True):
        x32, isd, rec = _prep(X, np.float32, force_disc_one=False)
        r32 = (x32.max(0) - x32.min(0)).astype(np.float32)
        r32[r32 == 0] = 1
        rec = (1 / r32).astype(np.float32)
        a = oracle.multisurf_scores(X, y, use_star=star)
        b = N.multisurf(x32, y.astype(float), rec, isd, star)
        assert scale_rel_err(a, b) < 1e-6
        x64, isd, rec = _prep(X, np.float64)
        a = oracle.surf_scores(X, y, use_star=star)
        b = N.surf(x64, y.astype(np.int32), rec, isd, star)
        assert scale_rel_err(a, b) < 1e-6
    x64, isd, rec = _prep(X, np.float64)
    cl, cc = np.unique(y, return_counts=True)
    for k in (1, 4):
        a = oracle.relieff_scores(X, y, n_neighbors=k)
        b = N.relieff(x64.astype(np.float32), np.searchsorted(cl, y), rec, isd, k,
                      (cc / len(y)).astype(np.float32), numba_order=oracle.numba_argsort)
        assert scale_rel_err(a, b) < 1e-6


def test_numba_argsort_port(oracle):
    rng = np.random.default_rng(3)
    v = rng.standard_normal(5000).astype(np.float32)
    np.testing.assert_array_equal(v[oracle.numba_argsort(v)], np.sort(v))
    # small arrays use insertion sort: stable, ties keep index order
    t = np.array([2, 1, 2, 1, 0, 2], dtype=np.float32)
    np.testing.assert_array_equal(oracle.numba_argsort(t), [4, 1, 3, 0, 2, 5])
    # NaN sorts last (lt_floats)
    w = np.array([3, np.nan, 1, 2], dtype=np.float32)
    assert oracle.numba_argsort(w)[-1] == 1


def test_bounded_sample_consistent(oracle):
    """The i-range used for the bench CPU baseline sums to the full result."""
    from sklearn.datasets import make_classification
    X, y = make_classification(n_samples=90, n_features=20, random_state=5)
    full = oracle.multisurf_scores(X, y)
    parts = oracle.multisurf_scores(X, y, i_range=(0, 40)) + \
        oracle.multisurf_scores(X, y, i_range=(40, 90))
    assert scale_rel_err(parts, full) < 1e-6
