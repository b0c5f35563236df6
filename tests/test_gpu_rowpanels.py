"""ReliefF / SURF plans that store only their focal rows of D, and focal
ranges scored in row panels.

A ReliefF / SURF plan keeps the distance rows of its own 128-sample blocks
(fs_gpu_internal.h d_row_in: a row-sharded rank holds 1/N of D instead of all of
it), and a one-shot call whose rows exceed the device is scored in panels of
whole blocks (row_panel_rows; the row_panel test hook forces the height here) -- the
reference streams each focal sample's distance row (ReliefF.py:143-157,
SURF.py:139-163).  Panels and slices must reproduce the one-panel scores
(ReliefF: float64 sums in another order, <= 1e-9 scale-relative; SURF:
the sparse pass 2 of a slice against the dense one of a whole fit, <= 1e-6)
and the oracle.
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


@pytest.mark.parametrize("panel", ["128", "384", "1000"])
def test_relieff_row_panels(F, oracle, hooks, panel):
    X, y = make_classification(n_samples=1100, n_features=300, n_informative=10, n_redundant=20,
                               n_classes=3, random_state=21)
    one = F.ReliefF(backend="gpu", n_neighbors=5).fit(X, y).feature_importances_
    hooks("row_panel", int(panel))
    s = F.ReliefF(backend="gpu", n_neighbors=5).fit(X, y).feature_importances_
    assert scale_rel_err(s, one) <= 1e-9
    assert_parity(s, oracle.relieff_scores(X, y, n_neighbors=5), 1e-5)


@pytest.mark.parametrize("star", [False, True])
def test_surf_row_panels(F, oracle, hooks, star):
    X, y = make_classification(n_samples=900, n_features=400, n_informative=10, n_redundant=20,
                               random_state=22)
    one = F.SURF(backend="gpu", use_star=star).fit(X, y).feature_importances_
    hooks("row_panel", 256)
    s = F.SURF(backend="gpu", use_star=star).fit(X, y).feature_importances_
    # a panel is a row slice, which takes the sparse pass 2 where the whole
    # fit takes the dense one (choose_sparse): float32 partials in another
    # order, a few ulps apart
    assert scale_rel_err(s, one) <= 1e-6
    assert_parity(s, oracle.surf_scores(X, y, use_star=star), 1e-5)


@pytest.mark.parametrize("algo", ["relieff", "surf"])
def test_row_slices_store_only_their_rows(F, oracle, algo):
    """Slices that do not start on a block boundary: the plan's window is
    their blocks; the slice sums partition the whole fit and match the
    oracle's focal-sample slice."""
    from fastselect_amd import _lib
    from fastselect_amd.ReliefF import relieff_inputs
    from fastselect_amd.SURF import surf_inputs
    X, y = make_classification(n_samples=1000, n_features=250, n_informative=10, n_redundant=20,
                               random_state=23)
    n = X.shape[0]
    parts = [(0, 77), (77, 500), (500, 1000)]
    if algo == "relieff":
        x32, ye, recip, isd, pri = relieff_inputs(np.asarray(X, np.float64), y, 10, "gpu")
        sums = [_lib.relieff_score("gpu", x32, ye, recip, isd, 4, pri, rows=r) for r in parts]
        ref_slice = oracle.relieff_scores(X, y, n_neighbors=4, i_range=parts[1])
        whole = oracle.relieff_scores(X, y, n_neighbors=4)
    else:
        x = np.ascontiguousarray(X, dtype=np.float64)
        isd, recip = surf_inputs(x, 10, "gpu")
        sums = [_lib.surf_score("gpu", x, y.astype(np.int32), recip, True, isd, rows=r)
                for r in parts]
        ref_slice = oracle.surf_scores(X, y, use_star=True, i_range=parts[1])
        whole = oracle.surf_scores(X, y, use_star=True)
    assert_parity((sums[1] / n).astype(np.float32), ref_slice, 1e-5)
    assert_parity((sum(sums) / n).astype(np.float32), whole, 1e-5)
