"""scikit-learn surface of the estimators, mirroring the reference's own
behaviour tests (tests/test_multisurf.py, test_relieff.py, test_surf.py,
test_turf.py) on this package.  CPU backend (the container has no GPU); the
same checks run on the GPU backend in tests/test_gpu.py.
"""
import numpy as np
import pytest
from numpy.testing import assert_allclose, assert_array_equal
from sklearn.base import BaseEstimator, TransformerMixin
from sklearn.datasets import make_classification
from sklearn.exceptions import NotFittedError
from sklearn.utils.estimator_checks import check_estimator

from fastselect_amd import SURF, MultiSURF, ReliefF, TuRF, _lib


@pytest.fixture
def ms_data():
    """test_multisurf.py:10-34"""
    X = np.array([
        [1.1, 5.0, 10, 3.0], [1.2, 4.0, 10, 3.0], [2.3, 6.0, 10, 3.0], [2.5, 5.5, 10, 3.0],
        [1.5, 4.5, 20, 3.0], [8.8, 5.0, 20, 3.0], [8.9, 4.0, 20, 3.0], [9.5, 6.0, 20, 3.0],
        [10.5, 4.5, 20, 3.0], [10.5, 4.5, 10, 3.0]], dtype=np.float32)
    return X, np.array([0, 0, 0, 0, 0, 1, 1, 1, 1, 1], dtype=np.int32)


@pytest.fixture
def rs_data():
    """test_relieff.py:10-32 / test_surf.py:11-33"""
    X = np.array([
        [0.1, 5.0, 10, 3.0], [0.2, 4.0, 10, 3.0], [0.3, 6.0, 10, 3.0],
        [10.8, 5.0, 20, 3.0], [10.9, 4.0, 20, 3.0], [11.0, 6.0, 20, 3.0]], dtype=np.float32)
    return X, np.array([0, 0, 0, 1, 1, 1], dtype=np.int32)


NO_GPU = _lib.device_count() == 0

# ---------------------------------------------------------------- MultiSURF


def test_ms_feature_importance_ranking(ms_data):
    X, y = ms_data
    m = MultiSURF(n_features_to_select=1, backend="cpu", discrete_limit=4).fit(X, y)
    assert set(m.top_features_) == {0}
    assert_allclose(m.feature_importances_[3], 0.0, atol=1e-7)


def test_ms_sklearn_api_compliance():
    check_estimator(MultiSURF())


def test_ms_fit_transform_shape(ms_data):
    X, y = ms_data
    assert MultiSURF(n_features_to_select=3, backend="cpu").fit_transform(X, y).shape == (10, 3)


@pytest.mark.parametrize("est", [MultiSURF, SURF])
def test_discrete_limit(est):
    X = np.array([[i, i % 3] for i in range(11)] * 2, dtype=np.float32)
    y = np.array([0] * 11 + [1] * 11, dtype=np.int32)
    assert_array_equal(est(discrete_limit=10, backend="cpu", n_features_to_select=2)
                       .fit(X, y).is_discrete_, [False, True])
    assert_array_equal(est(discrete_limit=12, backend="cpu", n_features_to_select=2)
                       .fit(X, y).is_discrete_, [True, True])


@pytest.mark.parametrize("est", [MultiSURF, SURF, ReliefF])
def test_not_fitted(est, ms_data):
    with pytest.raises(NotFittedError):
        est().transform(ms_data[0])


@pytest.mark.parametrize("est", [MultiSURF, SURF, ReliefF])
@pytest.mark.parametrize("bad", [-1, 0, 100])
def test_invalid_n_features_to_select(est, rs_data, bad):
    X, y = rs_data
    with pytest.raises(ValueError):
        est(n_features_to_select=bad).fit(X, y)
    with pytest.raises(ValueError):
        est(n_features_to_select=1.1).fit(X, y)
    with pytest.raises(TypeError):
        est(n_features_to_select="hi").fit(X, y)


def test_ms_verbose(ms_data, capsys):
    X, y = ms_data
    for kw, text in (({}, "Running MultiSURF"), ({"use_star": True}, "Running MultiSURF*"),
                     ({"backend": "cpu"}, "Running MultiSURF"),
                     ({"backend": "cpu", "use_star": True}, "Running MultiSURF*")):
        MultiSURF(verbose=True, **kw).fit(X, y)
        assert text in capsys.readouterr().out


@pytest.mark.parametrize("est", [MultiSURF, SURF, ReliefF])
def test_bad_backend(est, rs_data):
    with pytest.raises(ValueError):
        est(n_features_to_select=4, backend="tpu").fit(*rs_data)


@pytest.mark.skipif(not NO_GPU, reason="a GPU is visible")
def test_gpu_backend_without_gpu(ms_data, rs_data):
    """test_multisurf.py:170-178, test_surf.py:124-132: RuntimeError, never a
    silent CPU fallback (also for ReliefF, which the reference left unchecked)."""
    with pytest.raises(RuntimeError, match="no compatible GPU"):
        MultiSURF(backend="gpu", n_features_to_select=2).fit(*ms_data)
    with pytest.raises(RuntimeError, match="no HIP-enabled GPU is available"):
        SURF(backend="gpu").fit(*rs_data)
    with pytest.raises(RuntimeError, match="no compatible GPU"):
        ReliefF(backend="gpu", n_neighbors=1).fit(*rs_data)
    # the reference tests' own patterns still match (drop-in callers)
    with pytest.raises(RuntimeError, match="no compatible NVIDIA GPU"):
        MultiSURF(backend="gpu", n_features_to_select=2).fit(*ms_data)
    with pytest.raises(RuntimeError, match="no CUDA-enabled GPU is available"):
        SURF(backend="gpu").fit(*rs_data)


@pytest.mark.parametrize("est", [MultiSURF, SURF])
def test_nan_input(est, ms_data):
    X, y = ms_data
    X = X.copy()
    X[0, 0] = np.nan
    with pytest.raises(ValueError, match="Input X contains NaN"):
        est(backend="cpu", n_features_to_select=2).fit(X, y)


@pytest.mark.parametrize("est", [MultiSURF, SURF])
def test_single_class(est, ms_data):
    X, _ = ms_data
    m = est(backend="cpu", n_features_to_select=4).fit(X, np.zeros(X.shape[0]))
    assert np.all(m.feature_importances_ <= 1e-7)


def test_auto_backend_resolution(ms_data):
    m = MultiSURF(n_features_to_select=2).fit(*ms_data)
    assert m.effective_backend_ == ("cpu" if NO_GPU else "gpu")

# ------------------------------------------------------------------ ReliefF


def test_rf_feature_importance_ranking(rs_data):
    X, y = rs_data
    t = ReliefF(n_neighbors=1, n_features_to_select=2, discrete_limit=4, backend="cpu").fit(X, y)
    s = t.feature_importances_
    assert s[0] > s[1] and s[2] > s[1]
    assert_allclose(s[3], 0.0)
    assert set(t.top_features_) == {0, 2}


def test_rf_zero_range_feature(rs_data):
    t = ReliefF(n_neighbors=1, n_features_to_select=4, backend="cpu").fit(*rs_data)
    assert_allclose(t.feature_importances_[3], 0.0)


def test_rf_sklearn_api_compliance():
    check_estimator(ReliefF())


def test_rf_fit_transform_shape(rs_data):
    Xt = ReliefF(n_features_to_select=2, n_neighbors=2).fit_transform(*rs_data)
    assert Xt.shape == (6, 2)


def test_rf_discrete_limit():
    X = np.array([[i, i % 3] for i in range(11)] * 2)
    y = np.array([0] * 11 + [1] * 11)
    assert_array_equal(ReliefF(discrete_limit=10, n_features_to_select=2, n_neighbors=1)
                       .fit(X, y).is_discrete_, [False, True])
    assert_array_equal(ReliefF(discrete_limit=12, n_features_to_select=2, n_neighbors=1)
                       .fit(X, y).is_discrete_, [True, True])


@pytest.mark.parametrize("bad_k", [-1, 0])
def test_rf_invalid_n_neighbors(rs_data, bad_k):
    with pytest.raises(ValueError):
        ReliefF(n_neighbors=bad_k).fit(*rs_data)


def test_rf_transform_wrong_width(rs_data):
    X, y = rs_data
    t = ReliefF(n_features_to_select=4, n_neighbors=2).fit(X, y)
    with pytest.raises(ValueError):
        t.transform(X[:, :-1])


def test_rf_verbose(rs_data, capsys):
    ReliefF(verbose=True).fit(*rs_data)
    assert "Running ReliefF" in capsys.readouterr().out
    ReliefF(verbose=True, backend="cpu").fit(*rs_data)
    assert "Running ReliefF" in capsys.readouterr().out


def test_rf_insufficient_neighbors_warning(rs_data):
    with pytest.warns(UserWarning, match="is greater than or equal to the smallest class size"):
        ReliefF(n_neighbors=5).fit(*rs_data)


def test_rf_single_class(rs_data):
    X, _ = rs_data
    m = ReliefF(backend="cpu", n_neighbors=2).fit(X, np.zeros(6))
    assert np.all(np.isfinite(m.feature_importances_))
    assert np.all(m.feature_importances_ <= 0)

# --------------------------------------------------------------------- SURF


def test_surf_feature_importance_ranking(rs_data):
    m = SURF(n_features_to_select=2, backend="cpu", discrete_limit=3).fit(*rs_data)
    s = m.feature_importances_
    assert s[0] > s[1] and s[2] > s[1]
    assert_allclose(s[3], 0.0, atol=1e-7)
    assert set(m.top_features_) == {0, 2}


def test_surf_sklearn_api_compliance():
    check_estimator(SURF())


def test_surf_fit_transform_shape(rs_data):
    assert SURF(n_features_to_select=2, backend="cpu").fit_transform(*rs_data).shape == (6, 2)


def test_surf_verbose(rs_data, capsys):
    SURF(verbose=True).fit(*rs_data)
    assert "Running SURF" in capsys.readouterr().out
    SURF(verbose=True, backend="cpu", use_star=True).fit(*rs_data)
    assert "Running SURF*" in capsys.readouterr().out

# --------------------------------------------------------------------- TuRF


class MockReliefEstimator(BaseEstimator, TransformerMixin):
    """test_turf.py:8-16"""

    def fit(self, X, y=None):
        self.feature_importances_ = np.linspace(1, 0, X.shape[1])
        return self

    def transform(self, X):
        return X


@pytest.fixture
def turf_data():
    rng = np.random.default_rng(0)
    return rng.random((100, 20)), rng.integers(0, 2, 100)


def test_turf_sklearn_compatibility():
    check_estimator(TuRF(estimator=MockReliefEstimator(), n_features_to_select=2))


def test_turf_basic(turf_data):
    X, y = turf_data
    t = TuRF(estimator=MockReliefEstimator(), n_features_to_select=5).fit(X, y)
    Xt = t.transform(X)
    assert t.n_features_in_ == 20 and len(t.top_features_) == 5 and Xt.shape == (100, 5)
    np.testing.assert_array_equal(Xt, t.fit_transform(X, y))


def test_turf_attributes(turf_data):
    X, y = turf_data
    t = TuRF(estimator=MockReliefEstimator(), n_features_to_select=7).fit(X, y)
    assert t.feature_importances_.shape == (20,)
    assert t.feature_importances_[0] > t.feature_importances_[-1]
    np.testing.assert_array_equal(t.top_features_, np.arange(7))


def test_turf_n_iterations(turf_data):
    t = TuRF(estimator=MockReliefEstimator(), n_features_to_select=10, n_iterations=1,
             pct_remove=0.1).fit(*turf_data)
    assert len(t.top_features_) == 18


def test_turf_removes_at_least_one(turf_data):
    t = TuRF(estimator=MockReliefEstimator(), n_features_to_select=1, pct_remove=0.001)
    assert len(t.fit(*turf_data).top_features_) == 1


def test_turf_no_overshoot():
    rng = np.random.default_rng(1)
    t = TuRF(estimator=MockReliefEstimator(), n_features_to_select=10, pct_remove=0.2)
    assert len(t.fit(rng.random((50, 11)), rng.integers(0, 2, 50)).top_features_) == 10


def test_turf_verbose(turf_data, capsys):
    TuRF(estimator=MockReliefEstimator(), n_features_to_select=15, verbose=True).fit(*turf_data)
    out = capsys.readouterr().out
    assert "Iteration" in out and "features remaining" in out


def test_turf_errors(turf_data):
    for bad in (0, 1, 1.1):
        with pytest.raises(ValueError, match="pct_remove must be between 0 and 1"):
            TuRF(estimator=MockReliefEstimator(), pct_remove=bad).fit(*turf_data)
    with pytest.raises(NotFittedError):
        TuRF(estimator=MockReliefEstimator()).transform(turf_data[0])
    t = TuRF(estimator=MockReliefEstimator(), n_features_to_select=5).fit(*turf_data)
    with pytest.raises(ValueError, match="X has 21 features, but TuRF is expecting 20"):
        t.transform(np.random.default_rng(2).random((10, 21)))


def test_turf_over_multisurf():
    """TuRF driving the native MultiSURF (TuRF.py:87,111)."""
    from sklearn.datasets import make_classification
    X, y = make_classification(n_samples=120, n_features=30, n_informative=4, n_redundant=0,
                               shuffle=False, random_state=0)
    t = TuRF(estimator=MultiSURF(backend="cpu"), n_features_to_select=4, pct_remove=0.3).fit(X, y)
    assert len(t.top_features_) == 4
    assert len(set(t.top_features_.tolist()) & {0, 1, 2, 3}) >= 3


# ---- SURFstar / MultiSURFstar (scikit-rebate names) ----

@pytest.mark.parametrize("names", [("SURFstar", "SURF"), ("MultiSURFstar", "MultiSURF")])
def test_star_aliases_equal_use_star(names):
    import fastselect_amd as F
    from sklearn.base import clone
    X, y = make_classification(n_samples=120, n_features=25, random_state=2)
    star_cls, base_cls = (getattr(F, n) for n in names)
    a = star_cls(backend="cpu", n_features_to_select=5).fit(X, y)
    b = base_cls(backend="cpu", use_star=True, n_features_to_select=5).fit(X, y)
    np.testing.assert_array_equal(a.feature_importances_, b.feature_importances_)
    np.testing.assert_array_equal(a.top_features_, b.top_features_)
    assert "use_star" not in a.get_params()
    assert clone(a).use_star is True


@pytest.mark.parametrize("name", ["SURFstar", "MultiSURFstar"])
def test_star_aliases_sklearn_api(name):
    import fastselect_amd as F
    from sklearn.utils.estimator_checks import check_estimator
    check_estimator(getattr(F, name)(backend="cpu"))


# ---- TuRF over a resident MultiSURF plan -------------

class _RefitMultiSURF(MultiSURF):
    """MultiSURF without the resident fast path: TuRF refits on X[:, active]."""
    _resident_scorer = None


@pytest.mark.parametrize("star", [False, True])
def test_turf_resident_plan_equals_refits(star):
    X, y = make_classification(n_samples=150, n_features=60, n_informative=6,
                               random_state=3)
    X[:, 5] = np.round(X[:, 5])  # a discrete column in the mix
    kw = dict(n_features_to_select=8, pct_remove=0.2)
    fast = TuRF(MultiSURF(backend="cpu", use_star=star, discrete_limit=12), **kw).fit(X, y)
    slow = TuRF(_RefitMultiSURF(backend="cpu", use_star=star, discrete_limit=12), **kw).fit(X, y)
    assert_array_equal(fast.top_features_, slow.top_features_)
    assert_allclose(fast.feature_importances_, slow.feature_importances_, rtol=0, atol=1e-7)


def test_turf_resident_plan_validates_like_refit():
    """An int n_features_to_select larger than a later subset raises the
    base estimator's ValueError in both paths."""
    X, y = make_classification(n_samples=80, n_features=30, random_state=1)
    for est in (MultiSURF(backend="cpu", n_features_to_select=25),
                _RefitMultiSURF(backend="cpu", n_features_to_select=25)):
        with pytest.raises(ValueError, match="n_features"):
            TuRF(est, n_features_to_select=5, pct_remove=0.3).fit(X, y)


# ---- TuRF over resident ReliefF / SURF plans (fs_plan_create_relieff/_surf) --

class _RefitReliefF(ReliefF):
    _resident_scorer = None


class _RefitSURF(SURF):
    _resident_scorer = None


@pytest.mark.parametrize("make", [
    lambda cls: cls(backend="cpu", n_neighbors=5, discrete_limit=12),
    lambda cls: cls(backend="cpu", n_neighbors=2, discrete_limit=3),
])
def test_turf_resident_relieff_equals_refits(make):
    X, y = make_classification(n_samples=140, n_features=50, n_informative=6, n_classes=3,
                               random_state=4)
    X[:, 7] = np.round(X[:, 7])
    kw = dict(n_features_to_select=8, pct_remove=0.2)
    fast = TuRF(make(ReliefF), **kw).fit(X, y)
    slow = TuRF(make(_RefitReliefF), **kw).fit(X, y)
    assert_array_equal(fast.top_features_, slow.top_features_)
    assert_allclose(fast.feature_importances_, slow.feature_importances_, rtol=0, atol=1e-7)


@pytest.mark.parametrize("star", [False, True])
def test_turf_resident_surf_equals_refits(star):
    X, y = make_classification(n_samples=130, n_features=45, n_informative=6, random_state=5)
    X[:, 2] = np.round(X[:, 2])
    kw = dict(n_features_to_select=7, pct_remove=0.25)
    fast = TuRF(SURF(backend="cpu", use_star=star, discrete_limit=12), **kw).fit(X, y)
    slow = TuRF(_RefitSURF(backend="cpu", use_star=star, discrete_limit=12), **kw).fit(X, y)
    assert_array_equal(fast.top_features_, slow.top_features_)
    assert_allclose(fast.feature_importances_, slow.feature_importances_, rtol=0, atol=1e-7)


def test_turf_resident_relieff_single_class_falls_back():
    X, _ = make_classification(n_samples=40, n_features=12, random_state=0)
    y = np.zeros(40, dtype=int)
    t = TuRF(ReliefF(backend="cpu"), n_features_to_select=3).fit(X, y)
    assert t.top_features_.size == 3


def test_devices_parameter_resolution(monkeypatch):
    """``devices=`` (single-process multi-GPU, SURVEY.md §5 "Config"):
    resolution rules on a pretend 4-GPU host, and a get_params round trip."""
    from fastselect_amd import _base, _lib
    monkeypatch.setattr(_lib, "device_count", lambda: 4)
    assert _base.fit_devices(None, "cpu", 10 ** 6) is None
    assert _base.fit_devices([7], "cpu", 10) is None           # ignored by the CPU backend
    assert _base.fit_devices(None, "gpu", 10 ** 6) == [0]      # default: one device
    assert _base.fit_devices("all", "gpu", 100) == [0]         # small job: one device
    assert _base.fit_devices("all", "gpu", 9000) == [0, 1]     # one per 4096 samples
    assert _base.fit_devices("all", "gpu", 10 ** 6) == [0, 1, 2, 3]
    assert _base.stage_device("gpu", None, 10 ** 6) in (0, None)
    assert _base.fit_devices(2, "gpu", 10) == [2]
    assert _base.fit_devices(np.int64(3), "gpu", 10) == [3]
    assert _base.fit_devices((0, 0, 1), "gpu", 10) == [0, 0, 1]
    for bad in ([], [4], [-1], "0", "ALL", 1.5, True, [0, None]):
        with pytest.raises(ValueError, match="devices"):
            _base.fit_devices(bad, "gpu", 10)
    est = MultiSURF(devices=[0, 1])
    assert est.get_params()["devices"] == [0, 1]
    assert ReliefF(devices=2).get_params()["devices"] == 2
    assert SURF().get_params()["devices"] is None
