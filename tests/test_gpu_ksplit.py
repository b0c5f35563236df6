"""Pass-1 K-split (k_dist + k_dist_merge): tiles are split over their
feature range and the integer partial blocks added afterwards.  Distances are
exact integers, so every split gives bit-identical scores; forced here
(the ksplit test hook: s splits every tile into s parts, 1 disables it) against the
unsplit job, for the tiled layout (MultiSURF, MultiSURF*) and the full layout
(ReliefF, MultiSURF's focal-row slices), with continuous and discrete chunks
in one split range.  (The stream-K variant, measured no faster, was retired
in round 4.)
"""
import numpy as np
import pytest
from sklearn.datasets import make_classification

pytestmark = pytest.mark.gpu


def _data(n=1500, p=400, n_disc=40, seed=5):
    X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=30,
                               random_state=seed)
    rng = np.random.default_rng(seed)
    X[:, :n_disc] = rng.integers(0, 4, size=(n, n_disc))  # discrete chunks after the continuous
    return X, y


def _scores(monkeypatch, split, fn):
    """split: None (automatic) or an int (the ksplit test hook)."""
    from fastselect_amd import _lib
    with _lib.test_hooks(ksplit=0 if split is None else split):
        return fn()


@pytest.mark.parametrize("use_star", [False, True])
def test_multisurf_split_is_bit_identical(monkeypatch, use_star):
    from fastselect_amd import _lib
    from fastselect_amd.parallel import prepare_inputs
    X, y = _data()
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
    fn = lambda: _lib.multisurf_score("gpu", x, yv, recip, None, use_star, isd)
    ref = _scores(monkeypatch, 1, fn)
    # None: the automatic choice (the K-split model: every tile split here)
    for split in (None, 2, 5, 16):
        np.testing.assert_array_equal(_scores(monkeypatch, split, fn), ref)


def test_multisurf_rows_split_is_bit_identical(monkeypatch):
    from fastselect_amd import _lib
    from fastselect_amd.parallel import prepare_inputs
    X, y = _data(n=1100, p=300)
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
    fn = lambda: _lib.multisurf_score("gpu", x, yv, recip, None, False, isd, rows=(100, 700))
    ref = _scores(monkeypatch, 1, fn)
    for split in (None, 3):
        np.testing.assert_array_equal(_scores(monkeypatch, split, fn), ref)


def test_relieff_split_is_bit_identical(monkeypatch):
    from fastselect_amd import _lib
    from fastselect_amd.ReliefF import relieff_inputs
    X, y = _data(n=1300, p=350)
    x, ye, recip, isd, priors = relieff_inputs(X, y, 10, "gpu")
    fn = lambda: _lib.relieff_score("gpu", x, ye, recip, isd, 10, priors)
    ref = _scores(monkeypatch, 1, fn)
    for split in (None, 4):
        np.testing.assert_array_equal(_scores(monkeypatch, split, fn), ref)


def test_ksplit_many_tiles_is_bit_identical(monkeypatch):
    """More tiles than one round of workgroups (872 tiles; MultiSURF, 32-bit
    pass 1), split and unsplit."""
    from fastselect_amd import _lib
    from fastselect_amd.parallel import prepare_inputs
    X, y = _data(n=5300, p=150, n_disc=20)
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
    fn = lambda: _lib.multisurf_score("gpu", x, yv, recip, None, False, isd)
    ref = _scores(monkeypatch, 1, fn)
    for split in (None, 3, 8):
        np.testing.assert_array_equal(_scores(monkeypatch, split, fn), ref)
