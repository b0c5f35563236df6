"""Pass 1 on packed 16-bit operands (Prepared::q16, v_sad_u16): the default
for ReliefF from n = 4096, for MultiSURF from n = 16384 and for MultiSURF*
from n = 10000 samples.  Same bar
as every parity test: 1e-5 scale-relative and identical top-k.

ReliefF is exact with them (the band of exactly recomputed keys widens), so
it is forced on (the q16 test hook) at sizes the oracle runs in seconds.  MultiSURF's
thresholds carry a quantisation error whose score effect falls as ~n^-1.25
(DESIGN.md §2): it is checked against the oracle at n = 16384 (its default
size) and against the 32-bit path at n = 20000.
"""
import numpy as np
import pytest
from conftest import assert_parity, scale_rel_err
from sklearn.datasets import make_classification

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _fit(cls, X, y, **kw):
    est = cls(backend="gpu", n_features_to_select=1, **kw).fit(X, y)
    assert est.effective_backend_ == "gpu"
    return est.feature_importances_


def test_q16_mixed_blocks_relieff(oracle, hooks):
    from fastselect_amd import ReliefF
    hooks("q16", 1)
    rng = np.random.default_rng(5)
    n = 2000
    Xc = rng.standard_normal((n, 300)) * rng.uniform(0.1, 10, 300)
    Xd = rng.integers(0, 4, size=(n, 70)).astype(np.float64)
    X = np.concatenate([Xc, Xd], axis=1)[:, rng.permutation(370)]
    y = (X[:, 0] + X[:, 5] > 0).astype(int)
    assert_parity(_fit(ReliefF, X, y, n_neighbors=5), oracle.relieff_scores(X, y, n_neighbors=5),
                  TOL, k=10)


@pytest.mark.parametrize("k,ncls", [(10, 2), (3, 3)])
def test_q16_relieff_parity(oracle, k, ncls, hooks):
    from fastselect_amd import ReliefF
    hooks("q16", 1)
    X, y = make_classification(n_samples=3000, n_features=500, n_informative=20,
                               n_redundant=20, n_classes=ncls, random_state=k)
    assert_parity(_fit(ReliefF, X, y, n_neighbors=k),
                  oracle.relieff_scores(X, y, n_neighbors=k), TOL, k=10)


@pytest.mark.slow
def test_q16_multisurf_default_at_16384(oracle):
    """n = 16384 takes the 16-bit path by default (oracle: ~2e10 PFE)."""
    from fastselect_amd import MultiSURF
    X, y = make_classification(n_samples=16384, n_features=128, n_informative=20,
                               n_redundant=30, random_state=42)
    assert_parity(_fit(MultiSURF, X, y), oracle.multisurf_scores(X, y), TOL, k=10)


def test_q16_agrees_with_u32_path(hooks):
    from fastselect_amd import MultiSURF, ReliefF
    X, y = make_classification(n_samples=20000, n_features=2000, n_informative=20,
                               n_redundant=50, random_state=42)
    out = {}
    for flag in ("0", "1"):
        hooks("q16", int(flag))
        out[flag] = (_fit(MultiSURF, X, y), _fit(ReliefF, X, y, n_neighbors=10))
    for a, b in zip(out["0"], out["1"]):
        assert scale_rel_err(b, a) < 5e-6
        assert set(np.argsort(a)[::-1][:10]) == set(np.argsort(b)[::-1][:10])


@pytest.mark.slow
def test_q16_multisurf_mixed_default_at_16384(oracle):
    """The default 16-bit MultiSURF path with discrete and constant columns
    mixed in (u32 discrete rows after the packed continuous ones)."""
    from fastselect_amd import MultiSURF
    rng = np.random.default_rng(11)
    n = 16384
    Xc, y = make_classification(n_samples=n, n_features=70, n_informative=10, n_redundant=10,
                                random_state=3)
    Xd = rng.integers(0, 3, size=(n, 20)).astype(np.float64)
    Xk = np.full((n, 2), 4.0)
    X = np.concatenate([Xc, Xd, Xk], axis=1)[:, rng.permutation(92)]
    for star in (False, True):
        assert_parity(_fit(MultiSURF, X, y, use_star=star),
                      oracle.multisurf_scores(X, y, use_star=star), TOL, k=10)


def test_q16_multisurf_star_default_at_10000(oracle, hooks):
    """MultiSURF* takes the 16-bit pass from n = 10000: against the oracle
    (p = 96) and against the 32-bit path (p = 3000)."""
    from fastselect_amd import MultiSURF
    X, y = make_classification(n_samples=10000, n_features=96, n_informative=20,
                               n_redundant=30, random_state=7)
    assert_parity(_fit(MultiSURF, X, y, use_star=True),
                  oracle.multisurf_scores(X, y, use_star=True), TOL, k=10)
    X, y = make_classification(n_samples=10000, n_features=3000, n_informative=20,
                               n_redundant=100, random_state=42)
    out = {}
    for flag in ("0", "1"):
        hooks("q16", int(flag))
        out[flag] = _fit(MultiSURF, X, y, use_star=True)
    assert scale_rel_err(out["1"], out["0"]) < 5e-6
    assert set(np.argsort(out["0"])[::-1][:10]) == set(np.argsort(out["1"])[::-1][:10])
