"""Single-process multi-GPU fits (the estimators' ``devices=``; VERDICT r2
next #3, SURVEY.md §5 "Config / flags", §8(b) "one host thread per device").

On the one-GPU test box the device list repeats ordinal 0: every entry is its
own host thread with its own plan and stream, exactly the multi-GPU code path
(the tile / row partition and the host-side rank-order sums of the exchange
vectors), sharing one card.  Each case must equal the one-device fit within
1e-6 scale-relative with identical top-k, and the oracle within the 1e-5 bar.
"""
import numpy as np
import pytest
from sklearn.datasets import make_classification

from conftest import assert_parity, scale_rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    import fastselect_amd
    from fastselect_amd import _lib
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    return fastselect_amd


def _data(n=2500, p=700, seed=0, classes=2):
    return make_classification(n_samples=n, n_features=p, n_informative=15, n_redundant=30,
                               n_classes=classes, random_state=seed)


@pytest.mark.parametrize("star", [False, True])
@pytest.mark.parametrize("devs", [[0, 0], [0, 0, 0]])
def test_multisurf_devices_equal_one_device(F, oracle, star, devs):
    X, y = _data(2345, 700, 1)
    one = F.MultiSURF(backend="gpu", use_star=star, devices=[0], n_features_to_select=10).fit(X, y)
    many = F.MultiSURF(backend="gpu", use_star=star, devices=devs, n_features_to_select=10).fit(X, y)
    assert many.devices_ == devs and one.devices_ == [0]
    assert scale_rel_err(many.feature_importances_, one.feature_importances_) <= 1e-6
    assert set(many.top_features_) == set(one.top_features_)
    assert_parity(many.feature_importances_, oracle.multisurf_scores(X, y, use_star=star),
                  1e-5, 10)


def test_multisurf_devices_with_tile_shards(F, hooks):
    """V = 2 tile shards per device (n beyond HBM) under two device threads:
    tile t belongs to thread / shard t % 4."""
    X, y = _data(1800, 400, 2)
    one = F.MultiSURF(backend="gpu", devices=[0]).fit(X, y).feature_importances_
    hooks("shards", 2)
    many = F.MultiSURF(backend="gpu", devices=[0, 0]).fit(X, y).feature_importances_
    assert scale_rel_err(many, one) <= 1e-6


def test_relieff_devices_equal_one_device(F, oracle):
    X, y = _data(2100, 500, 3, classes=3)
    one = F.ReliefF(backend="gpu", n_neighbors=10, devices=0).fit(X, y)
    many = F.ReliefF(backend="gpu", n_neighbors=10, devices=[0, 0, 0]).fit(X, y)
    assert scale_rel_err(many.feature_importances_, one.feature_importances_) <= 1e-6
    assert set(many.top_features_) == set(one.top_features_)
    assert_parity(many.feature_importances_, oracle.relieff_scores(X, y, n_neighbors=10), 1e-5)


@pytest.mark.parametrize("star", [False, True])
def test_surf_devices_equal_one_device(F, oracle, star):
    X, y = _data(1500, 600, 4)
    one = F.SURF(backend="gpu", use_star=star, devices=[0]).fit(X, y)
    many = F.SURF(backend="gpu", use_star=star, devices=[0, 0]).fit(X, y)
    assert scale_rel_err(many.feature_importances_, one.feature_importances_) <= 1e-6
    assert_parity(many.feature_importances_, oracle.surf_scores(X, y, use_star=star), 1e-5)


def test_surf_devices_integer_route(F, hooks):
    """Two device threads on SURF's integer distance route (forced; this size
    would take the float64 route by itself): each thread's row plan resolves
    its rows' float32 distances, and the scores are the float64 route's."""
    X, y = _data(1500, 600, 4)
    hooks("surf_f64", 1)
    ref = F.SURF(backend="gpu", use_star=True, devices=[0, 0]).fit(X, y).feature_importances_
    hooks("surf_f64", 0)
    got = F.SURF(backend="gpu", use_star=True, devices=[0, 0]).fit(X, y).feature_importances_
    assert np.array_equal(np.asarray(got), np.asarray(ref))


def test_devices_bad_ordinal_is_a_value_error(F):
    from fastselect_amd import _lib
    X, y = _data(300, 80, 5)
    with pytest.raises(ValueError, match="devices"):
        F.MultiSURF(backend="gpu", devices=[0, _lib.device_count()]).fit(X, y)
    with pytest.raises(ValueError, match="devices"):
        F.ReliefF(backend="gpu", devices=[]).fit(X, y)


def test_devices_default_is_one_device(F):
    """devices=None: device 0, as the reference; devices='all':
    every visible device the job has work for (one per 4096 samples)."""
    from fastselect_amd import _base, _lib
    X, y = _data(500, 80, 6)
    est = F.MultiSURF(backend="gpu").fit(X, y)
    assert est.devices_ == [0]
    assert _base.fit_devices(None, "gpu", 10 ** 6) == [0]
    assert _base.fit_devices("all", "gpu", 10 ** 6) == list(range(_lib.device_count()))
    assert F.MultiSURF(backend="gpu", devices="all").fit(X, y).devices_ == [0]
