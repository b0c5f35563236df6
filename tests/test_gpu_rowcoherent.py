"""Row-localised coherent rounding on the default 16-bit MultiSURF path
(VERDICT r2 weak #2 / next #1c).

tests/golden/make_rowcoherent.py builds n = 16384 inputs in which a few rows
round every feature the same way (values 0.6 of a 16-bit quantum above a grid
point; at each column's minimum the pair-error signs agree as well), so their
pairs' quantised distances are off by ~0.4 pc integer units -- about 4x the
refinement band of independent rounding -- while the whole-matrix sampled
calibration meets those rows only by chance (minrow4: ~2 sampled pairs).  The
default GPU path (16-bit pass 1 for MultiSURF at n >= 16384, MultiSURF* from
10000) must still match the oracle within the 1e-5 bar with identical top-10,
which the per-row guard provides (fs_pass1.hip row_guard: rows whose mean pass-1 error,
from the mean correction, is coherent get a band that covers it).
"""
import hashlib
import importlib.util
import os

import numpy as np
import pytest

from conftest import assert_parity

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
_spec = importlib.util.spec_from_file_location("mk_rowcoherent",
                                               os.path.join(GOLD, "make_rowcoherent.py"))
mk = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mk)


@pytest.fixture(scope="module")
def F():
    import fastselect_amd
    from fastselect_amd import _lib
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    return fastselect_amd


@pytest.mark.parametrize("star", [False, True])
@pytest.mark.parametrize("name", sorted(mk.CASES))
def test_row_coherent_rounding_default_path(F, name, star):
    path = os.path.join(GOLD, f"rowcoherent_{name}.npz")
    if not os.path.exists(path):
        pytest.fail(f"missing fixture {path} (tests/golden/make_rowcoherent.py)")
    fx = np.load(path, allow_pickle=False)
    X, y = mk.make(name)
    assert hashlib.sha256(X.tobytes()).hexdigest() == str(fx["x_sha256"])
    s = F.MultiSURF(backend="gpu", use_star=star, n_features_to_select=10).fit(X, y)
    assert_parity(s.feature_importances_, fx["scores_star" if star else "scores"], 1e-5, 10)


@pytest.mark.parametrize("name", ["minrows_16k", "minrow4_16k"])
def test_row_guard_takes_32bit_operands(F, name):
    """The per-row guard sees the coherent rows whether or not the sampled
    calibration did, and turns the 16-bit operands off; ordinary data of the
    same shape keeps them (no false trip)."""
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    X, y = mk.make(name)
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
    job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", shard=False)
    cal = job.plan.calibration()
    job.close()
    assert not cal["q16"] and cal["guard"]
    from sklearn.datasets import make_classification
    X0, y0 = make_classification(n_samples=mk.N, n_features=mk.P, n_informative=20,
                                 n_redundant=50, random_state=7)
    x, yv, recip, isd = prepare_inputs(X0, y0, backend="gpu")
    job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", shard=False)
    cal = job.plan.calibration()
    job.close()
    assert cal["q16"] and not cal["guard"]


@pytest.mark.parametrize("name", ["minrows_16k", "make_classification"])
def test_one_shot_guard_after_pass1_matches_plan(F, name):
    """The one-shot call decides the row guard after its first pass 1 (from
    the correction computed beside k_dist; fs_pass1.hip plan_pass1), a plan
    object before it: the operand width, and so the scores, are the same
    bit for bit -- the coherent case switched to 32-bit operands by the
    deferred guard, ordinary data kept on 16-bit ones."""
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    if name == "make_classification":
        from sklearn.datasets import make_classification
        X, y = make_classification(n_samples=mk.N, n_features=mk.P, n_informative=20,
                                   n_redundant=50, random_state=7)
    else:
        X, y = mk.make(name)
    one_shot = F.MultiSURF(backend="gpu", n_features_to_select=10).fit(X, y).feature_importances_
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
    job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", shard=False)
    try:
        q16 = job.plan.calibration()["q16"]
        stepped = job.step().cpu().numpy()
    finally:
        job.close()
    assert bool(q16) == (name == "make_classification")
    np.testing.assert_array_equal(one_shot, stepped)
