"""fs_stage_x_cast: MultiSURF.fit's float64 -> float32 cast (float32 X: a
copy into pinned memory) fused with the finiteness scan and the upload of X
(row blocks uploaded while later ones are cast).  The cast must equal numpy's astype bit for bit, the scan must flag
exactly what scikit-learn's check would, and a fit through the staged copy
must score exactly as a fit of the float32 array."""
import numpy as np
import pytest
from sklearn.datasets import make_classification

pytestmark = pytest.mark.gpu


def _x64(n=3000, p=700, seed=3):
    rng = np.random.default_rng(seed)
    x = rng.standard_normal((n, p)) * 10.0 ** rng.integers(-30, 30, size=(1, p))
    x[0, :5] = [1e-45, -1e-46, 3.4028234663852886e38, 1.0 + 2.0 ** -24, 1.0 + 3 * 2.0 ** -25]
    return x


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_cast_matches_numpy_and_stages(dtype):
    from fastselect_amd import _lib
    x = _x64().astype(dtype)
    for n_jobs in (1, 3, -1):
        out, finite, h = _lib.stage_x_cast(x, n_jobs)
        try:
            assert finite and h != 0
            assert out.ctypes.data != x.ctypes.data
            np.testing.assert_array_equal(out.view(np.uint32), x.astype(np.float32).view(np.uint32))
        finally:
            with _lib.unstaged(h):
                pass


@pytest.mark.parametrize("bad", [np.nan, np.inf, -np.inf, 1e39])
def test_non_finite_is_flagged_and_not_staged(bad):
    from fastselect_amd import _lib
    x = _x64(n=2000, p=600)
    x[1777, 555] = bad  # in the last row block
    out, finite, h = _lib.stage_x_cast(x, -1)
    assert not finite and h == 0
    with np.errstate(over="ignore"):
        ref = x.astype(np.float32)
    np.testing.assert_array_equal(out.view(np.uint32), ref.view(np.uint32))


def test_fit_from_float64_equals_fit_from_float32():
    from fastselect_amd import MultiSURF
    X, y = make_classification(n_samples=1200, n_features=1000, n_informative=20,
                               n_redundant=40, random_state=8)
    assert X.size >= 1 << 20  # takes the staged cast
    a = MultiSURF(n_features_to_select=10, backend="gpu").fit(X, y)
    b = MultiSURF(n_features_to_select=10, backend="gpu").fit(X.astype(np.float32), y)
    # not staged at fit time (Fortran order takes validate_xy): same scores
    d = MultiSURF(n_features_to_select=10, backend="gpu").fit(np.asfortranarray(X), y)
    np.testing.assert_array_equal(a.feature_importances_, d.feature_importances_)
    np.testing.assert_array_equal(a.feature_importances_, b.feature_importances_)
    np.testing.assert_array_equal(a.top_features_, b.top_features_)
    # ... and again with the same array (the staged copy was released)
    c = MultiSURF(n_features_to_select=10, backend="gpu").fit(X, y)
    np.testing.assert_array_equal(a.feature_importances_, c.feature_importances_)


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_fit_with_nan_raises_scikit_learn_error(dtype):
    from fastselect_amd import MultiSURF
    X, y = make_classification(n_samples=1100, n_features=1000, random_state=2)
    X = X.astype(dtype)
    X[1050, 10] = np.nan
    with pytest.raises(ValueError, match="Input X contains NaN"):
        MultiSURF(backend="gpu").fit(X, y)
    X[1050, 10] = 0.0
    MultiSURF(backend="gpu").fit(X, y)  # no staged copy left behind


def test_fit_with_bad_parameter_releases_staged_copy():
    from fastselect_amd import MultiSURF
    X, y = make_classification(n_samples=1100, n_features=1000, random_state=4)
    with pytest.raises(ValueError):
        MultiSURF(n_features_to_select=5000, backend="gpu").fit(X, y)
    MultiSURF(n_features_to_select=5, backend="gpu").fit(X, y)
