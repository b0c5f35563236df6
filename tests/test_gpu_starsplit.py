"""MultiSURF* / SURF* with the star split (fs_starterm.hip): pass 2 weighs the
near pairs only and every far pair's weight comes from an all-pairs term per
column, computed from the column's sorted values (MultiSURF.py:217-251,
SURF.py:180-193 weigh every miss / every pair).

The split is an exact rearrangement of the same sum, so against the dense
star weights (the star_split hook off) the scores may differ only by float
summation order: the dense pass sums float32 |a - b| terms in float32
partials, the split sums the far part in float64.  Bar: 2e-6 scale-relative
between the two forms (the dense form's own float32 error is ~1e-7 to 1e-6
at these sizes), and the oracle's 1e-5 for the split.  Cases: continuous,
discrete and mixed columns, value grids (ties), three classes, one class,
row slices of SURF, MultiSURF tile shards (the per-column terms split over
the shards), the dense near-only form (sparse hook off).
"""
import warnings

import numpy as np
import pytest
from sklearn.datasets import make_classification

from conftest import assert_parity
from parity_metrics import scale_rel_err

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def F():
    import fastselect_amd
    from fastselect_amd import _lib
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    return fastselect_amd


def _data(kind, n=1500, p=300, seed=3):
    rng = np.random.default_rng(seed)
    if kind == "classif":
        return make_classification(n_samples=n, n_features=p, n_informative=12, n_redundant=20,
                                   random_state=seed)
    if kind == "three":
        return make_classification(n_samples=n, n_features=p, n_informative=12, n_redundant=10,
                                   n_classes=3, n_clusters_per_class=1, random_state=seed)
    y = rng.integers(0, 2, n)
    if kind == "grid":  # 41 levels: continuous, many exact ties
        X = rng.integers(0, 41, (n, p)).astype(np.float64)
    elif kind == "mixed":
        X = rng.standard_normal((n, p))
        X[:, : p // 3] = rng.integers(0, 4, (n, p // 3))
    elif kind == "discrete":
        X = rng.integers(0, 3, (n, p)).astype(np.float64)
    elif kind == "single_class":
        X = rng.standard_normal((n, p))
        y = np.zeros(n, dtype=int)
    elif kind == "lognormal":
        X = np.exp(2.0 * rng.standard_normal((n, p)))
    else:
        raise ValueError(kind)
    return X, y


def _fit(F, algo, X, y):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)
        est = (F.MultiSURF if algo == "multisurf" else F.SURF)(backend="gpu", use_star=True)
        return np.asarray(est.fit(X, y).feature_importances_, dtype=np.float64)


def _oracle(oracle, algo, X, y):
    if algo == "multisurf":
        return oracle.multisurf_scores(X, y, use_star=True)
    return oracle.surf_scores(X, y, use_star=True)


@pytest.mark.parametrize("kind", ["classif", "three", "grid", "mixed", "discrete",
                                  "single_class", "lognormal"])
@pytest.mark.parametrize("algo", ["multisurf", "surf"])
def test_split_is_the_dense_star_sum(F, oracle, hooks, algo, kind):
    X, y = _data(kind)
    hooks("star_split", 0)
    dense = _fit(F, algo, X, y)
    hooks("star_split", 1)
    split = _fit(F, algo, X, y)
    err = scale_rel_err(split, dense)
    assert err <= 2e-6, f"{algo}* {kind}: split vs dense {err:.3e}"
    assert_parity(split, _oracle(oracle, algo, X, y), 1e-5)


@pytest.mark.parametrize("algo", ["multisurf", "surf"])
def test_split_dense_near_only_form(F, hooks, algo):
    """The split with the dense pass 2 (sparse hook off): near-only weights
    in k_weights / k_score, the same per-column terms."""
    X, y = _data("mixed", n=1100, p=200, seed=8)
    hooks("star_split", 0)
    dense = _fit(F, algo, X, y)
    hooks("star_split", 1)
    hooks("sparse", 0)
    split = _fit(F, algo, X, y)
    assert scale_rel_err(split, dense) <= 2e-6


def test_split_surf_row_slices(F, hooks):
    """A SURF* row slice scores its focal rows only: the column terms weigh
    those rows alone (alpha = 0 elsewhere)."""
    from fastselect_amd import _lib
    from fastselect_amd.SURF import surf_inputs
    X, y = _data("mixed", n=1400, p=260, seed=9)
    isd, recip = surf_inputs(X, 10, "gpu")
    yi = y.astype(np.int32)
    out = {}
    for split in (0, 1):
        hooks("star_split", split)
        out[split] = [_lib.surf_score("gpu", X, yi, recip, True, isd, rows=r)
                      for r in ((0, 1400), (200, 1100), (1300, 1400))]
    for a, b in zip(out[1], out[0]):
        assert scale_rel_err(a, b) <= 2e-6


@pytest.mark.parametrize("shards", [2, 3])
def test_split_multisurf_tile_shards(F, hooks, shards):
    """MultiSURF* over tile shards on one device: each shard adds the column
    terms of its share of the columns, the shards' sums add up to the
    whole's."""
    X, y = _data("mixed", n=1300, p=330, seed=12)
    hooks("star_split", 1)
    whole = _fit(F, "multisurf", X, y)
    hooks("shards", shards)
    sharded = _fit(F, "multisurf", X, y)
    assert scale_rel_err(sharded, whole) <= 1e-9


def test_split_is_the_default(F):
    """MultiSURF* and SURF* take the split on their own (n <= 24576, up to 8
    classes): pass 2 goes sparse, over the near pairs only."""
    from fastselect_amd import _lib
    from fastselect_amd.SURF import surf_inputs
    import torch
    X, y = _data("classif", n=4200, p=128, seed=21)  # SURF goes sparse from 4096 samples
    isd, recip = surf_inputs(X, 10, "gpu")
    nonstar = {}
    for star in (False, True):
        plan = _lib.RowsPlan("gpu", "surf", np.ascontiguousarray(X), y.astype(np.int32), recip,
                             isd, use_star=star)
        sums = torch.zeros(X.shape[1], dtype=torch.float64, device="cuda")
        plan.score(sums.data_ptr())
        torch.cuda.synchronize()
        nonstar[star] = plan.weighted_pairs()
        plan.close()
    # both sparse over the same near pairs: SURF weighs them, SURF* with the
    # split weighs them too (its far pairs are in the column terms)
    assert nonstar[False] > 0
    assert nonstar[True] == nonstar[False]
