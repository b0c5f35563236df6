"""Other data families on the default MultiSURF / MultiSURF* path (VERDICT
r2 weak #2: the 16-bit pass-1 band and cut-offs were tuned on
make_classification).

tests/golden/make_families.py builds n = 16384 inputs, where 16-bit pass-1
operands are the default: iid uniform noise with unrelated labels, lognormal
columns whose ranges are set by a few extreme values, and mixed integer-level
/ coarse-grid / continuous columns.

What they showed (profiles/r03/families.txt): on signal-free data the
MultiSURF scores sit at the level of single near/far decisions, and the
quantised thresholds of the 16-bit path moved enough of them to give 1.6e-4
of max |s| against the oracle.  Every MultiSURF path now estimates that risk
after scoring (fs_plan_decision_guard; fs_plan.hip q16_decision_risk) and
scores again on 32-bit operands above 5e-6.  Since round 4 the row means are
exact (fs_colsort.hip), and the uniform and lognormal cases are checked
decision by decision against the oracle's counts (family_*_decisions.npz);
where the reference's own float32 sums are further than 5e-6 of max |s|
from the float64 sums of the same decisions, the residual must be
accumulation (conftest.assert_parity_attributed).
"""
import hashlib
import importlib.util
import os

import numpy as np
import pytest

from conftest import assert_parity, assert_parity_attributed

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
_spec = importlib.util.spec_from_file_location("mk_families",
                                               os.path.join(GOLD, "make_families.py"))
mk = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mk)


@pytest.fixture(scope="module")
def F():
    import fastselect_amd
    from fastselect_amd import _lib
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    return fastselect_amd


def _fit(F, name, star):
    from fastselect_amd import _lib
    path = os.path.join(GOLD, f"family_{name}.npz")
    if not os.path.exists(path):
        pytest.fail(f"missing fixture {path} (tests/golden/make_families.py)")
    fx = np.load(path, allow_pickle=False)
    X, y = mk.make(name)
    assert hashlib.sha256(X.tobytes()).hexdigest() == str(fx["x_sha256"])
    s = F.MultiSURF(backend="gpu", use_star=star, n_features_to_select=10).fit(X, y)
    return s.feature_importances_, fx["scores_star" if star else "scores"], _lib.multisurf_last_guard()


@pytest.mark.parametrize("star", [False, True])
def test_mixed_columns_default_path(F, star):
    """make_classification columns beside integer-level and coarse-grid ones:
    the 1e-5 bar against the oracle, and no 32-bit re-run (signal present)."""
    s, ref, (risk, rerun) = _fit(F, "mixed_16k", star)
    assert_parity(s, ref, 1e-5, 10)
    if not star:
        assert 0.0 <= risk < 5e-6 and not rerun


def test_uniform_noise_multisurf_star(F):
    s, ref, _ = _fit(F, "uniform_16k", True)
    assert_parity(s, ref, 1e-5, 10)


def _decided(name):
    """(plan-path scores, per-row near hit / miss counts) through
    ShardedMultiSURF (decision check included) and the oracle's counts and
    float64-sum scores (tests/golden/make_families.py --decisions / --f64)."""
    from fastselect_amd import parallel
    X, y = mk.make(name)
    x, yv, recip, isd = parallel.prepare_inputs(X, y, backend="gpu")
    job = parallel.ShardedMultiSURF(x, yv, recip, isd, backend="gpu", shard=False)
    try:
        s = job.step().cpu().numpy()
        counts = job.counts.cpu().numpy()
    finally:
        job.close()
    dec = np.load(os.path.join(GOLD, f"family_{name}_decisions.npz"), allow_pickle=False)
    exact = np.load(os.path.join(GOLD, f"family_{name}_f64.npz"), allow_pickle=False)["scores"]
    return s, counts, dec["counts"], exact


def test_uniform_noise_multisurf_reruns_on_32bit(F):
    """Signal-free data: the decision check trips and the call re-scores on
    32-bit operands.  Every row's near hit / miss count then equals the
    reference's; the reference's own float32 sums are 2.6e-5 of max |s| from
    the float64 sums of those decisions, so the bar is the attributed one
    (conftest.assert_parity_attributed): at least 5x closer to the float64
    sums, and within the reference's own error + 1e-5 of the reference."""
    s, ref, (risk, rerun) = _fit(F, "uniform_16k", False)
    assert risk > 5e-6 and rerun
    sp, counts, ref_counts, exact = _decided("uniform_16k")
    np.testing.assert_array_equal(sp, s)
    assert_parity_attributed(s, ref, exact, counts, ref_counts, 1e-5, 10)


def test_lognormal_multisurf_star(F):
    s, ref, _ = _fit(F, "lognormal_16k", True)
    assert_parity(s, ref, 1e-5, 10)


def test_lognormal_multisurf(F):
    """Columns whose ranges are set by a few values ~1e5 x the median: open in
    round 3 (2.7e-4 of max |s|; the binned ranks of the old mean correction
    moved the thresholds), closed by the exact per-column order
    (fs_colsort.hip): no decision differs from the reference's."""
    s, ref, _ = _fit(F, "lognormal_16k", False)
    sp, counts, ref_counts, exact = _decided("lognormal_16k")
    np.testing.assert_array_equal(sp, s)
    assert_parity_attributed(s, ref, exact, counts, ref_counts, 1e-5, 10)
