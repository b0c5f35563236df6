"""Parity at BASELINE.json's full sizes (north-star target).

Each case regenerates one BASELINE configuration on the GPU box, checks that
the input is bit-identical to the one the oracle scored (sha256 of X), runs
the default GPU path through the C ABI and compares with the committed oracle
scores of ``tests/golden/fullsize_*.npz`` (made in the container by
``tests/golden/make_fullsize.py`` with the C restatement of the reference's
backend='cpu' kernels, oracle/relief_oracle.c).

Bar (BASELINE north_star): max_f |s_f - s_ref_f| <= 1e-5 *
max_f |s_ref_f| and identical top-10 index sets (the reference ranks with
np.argsort(scores)[::-1][:k], MultiSURF.py:443).  Slices compare the sums of
the same focal samples (the reference's per-sample rows summed over
i_range, / n).

Attribution (VERDICT r2 next #1b): where a float64-accumulation fixture
exists (fullsize_*_f64.npz: the oracle with the same diffs and near/far
decisions but every later sum in float64), the GPU's scores must be at least
as close to those float64 sums as the reference arithmetic is -- in the
maximum and in the rms over all features -- i.e. the residual against the
reference is the reference's own float32 accumulation.  Where the GPU takes
every near/far decision as the reference does (32-bit pass 1: cfg2, ReliefF,
SURF's float64 pass) it must also meet the per-element rtol 1e-5 against
those sums on every feature with |s| >= 1e-2 max|s| (the 1e-3 band's
figures are reported, not asserted: see _attribute).
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import assert_parity
from parity_metrics import per_element, summary

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
TOL = 1e-5
TOPK = 10

_DATA = {}


def _fixture(name):
    path = os.path.join(GOLD, f"fullsize_{name}.npz")
    if not os.path.exists(path):
        pytest.fail(f"missing fixture {path} (tests/golden/make_fullsize.py)")
    return np.load(path, allow_pickle=False)


def _attribute(name, s, ref, per_element_bar, rms=True):
    """The attribution check above, when fullsize_{name}_f64.npz exists.
    rms=False (16-bit pass 1): only the max is compared -- pairs between the
    quantised and the reference threshold are decided differently there, an
    error of its own beside the accumulation's (Numerics)."""
    path = os.path.join(GOLD, f"fullsize_{name}_f64.npz")
    if not os.path.exists(path):
        return
    exact = np.load(path, allow_pickle=False)["scores"].astype(np.float64)
    s, ref = np.asarray(s, np.float64), np.asarray(ref, np.float64)
    dg, do = np.abs(s - exact), np.abs(ref - exact)
    msg = (f"GPU vs f64 sums: {summary(s, exact)}; reference arithmetic vs f64 sums: "
           f"{summary(ref, exact)}")
    print(msg)
    assert dg.max() <= do.max(), msg
    if rms:
        assert np.sqrt((dg ** 2).mean()) <= np.sqrt((do ** 2).mean()), msg
    if per_element_bar:
        # every feature with |s| >= 1e-2 max|s| within rtol 1e-5 of the
        # float64 sums; the 1e-3 band is reported (profiles/r03/
        # parity_report.txt): there the GPU's float32 pass-2 partials (one per
        # 64-row half tile and 8 columns) leave absolute errors of a few 1e-8
        # of max|s|, which exceed 1e-5 of the smallest scores of the band
        assert per_element(s, exact, 1e-2, TOL)["over"] == 0.0, msg


def _data(n, p, red, n_classes=2):
    key = (n, p, red, n_classes)
    if key not in _DATA:
        from sklearn.datasets import make_classification
        _DATA.clear()  # one configuration resident at a time (cfg5 X is 4 GB)
        _DATA[key] = make_classification(n_samples=n, n_features=p, n_informative=20,
                                         n_redundant=red, n_classes=n_classes, random_state=42)
    return _DATA[key]


def _inputs(fx):
    n, p, red = int(fx["n"]), int(fx["p"]), int(fx["n_redundant"])
    ncls = int(fx["n_classes"]) if "n_classes" in fx else 2
    X, y = _data(n, p, red, ncls)
    algo = str(fx["algo"])
    x = X if algo == "surf" else X.astype(np.float32)
    dig = hashlib.sha256(np.ascontiguousarray(x).tobytes()).hexdigest()
    assert dig == str(fx["x_sha256"]), "regenerated X differs from the one the oracle scored"
    assert int(np.asarray(y).sum()) == int(fx["y_sum"])
    return X, y


@pytest.fixture(scope="module")
def lib():
    import fastselect_amd
    from fastselect_amd import _lib
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    return fastselect_amd


def test_cfg2_multisurf_whole_fit(lib):
    fx = _fixture("cfg2_multisurf")
    X, y = _inputs(fx)
    est = lib.MultiSURF(backend="gpu", n_features_to_select=TOPK).fit(X, y)
    assert est.effective_backend_ == "gpu"
    assert_parity(est.feature_importances_, fx["scores"], TOL, TOPK)
    _attribute("cfg2_multisurf", est.feature_importances_, fx["scores"], True)


def test_cfg3_relieff_k10_whole_fit(lib):
    fx = _fixture("cfg3_relieff_k10")
    X, y = _inputs(fx)
    est = lib.ReliefF(backend="gpu", n_neighbors=10, n_features_to_select=TOPK).fit(X, y)
    assert est.effective_backend_ == "gpu"
    assert_parity(est.feature_importances_, fx["scores"], TOL, TOPK)
    _attribute("cfg3_relieff_k10", est.feature_importances_, fx["scores"], True)


def test_cfg3_relieff_k10_three_classes(lib):
    """SURVEY.md §8d's 3-class cfg3 variant: prior-weighted misses of two
    other classes per focal sample (ReliefF.py:177-216)."""
    fx = _fixture("cfg3_relieff_k10_3class")
    X, y = _inputs(fx)
    est = lib.ReliefF(backend="gpu", n_neighbors=10, n_features_to_select=TOPK).fit(X, y)
    assert est.effective_backend_ == "gpu"
    assert_parity(est.feature_importances_, fx["scores"], TOL, TOPK)
    _attribute("cfg3_relieff_k10_3class", est.feature_importances_, fx["scores"], True)


def test_cfg4_multisurf_north_star(lib):
    """BASELINE north_star: MultiSURF on 20000 x 20000 fp32, default GPU
    path (16-bit pass-1 operands), scores within 1e-5 and identical top-k."""
    fx = _fixture("cfg4_multisurf")
    X, y = _inputs(fx)
    est = lib.MultiSURF(backend="gpu", n_features_to_select=TOPK).fit(X, y)
    assert_parity(est.feature_importances_, fx["scores"], TOL, TOPK)
    # 16-bit pass 1 decides pairs between the quantised and the reference
    # threshold differently (Numerics): no per-element or rms claim
    # (measured: max 1.9e-6 vs the reference arithmetic's 2.9e-6 of max|s|,
    # rms 4.0e-7 vs 7.5e-8; profiles/r03/parity_report.txt)
    _attribute("cfg4_multisurf", est.feature_importances_, fx["scores"], False, rms=False)
    assert set(est.top_features_.tolist()) == set(np.argsort(fx["scores"])[::-1][:TOPK].tolist())


def test_cfg4_multisurf_q32_attribution(lib, hooks):
    """The north-star data on 32-bit pass-1 operands (q16 hook 0: every
    near/far decision the reference's): the whole residual is then
    accumulation, and the GPU is at least as close to the float64 sums as
    the reference's float32 arithmetic, max and rms."""
    hooks("q16", 0)
    fx = _fixture("cfg4_multisurf")
    X, y = _inputs(fx)
    est = lib.MultiSURF(backend="gpu", n_features_to_select=TOPK).fit(X, y)
    assert_parity(est.feature_importances_, fx["scores"], TOL, TOPK)
    _attribute("cfg4_multisurf", est.feature_importances_, fx["scores"], False)


def test_cfg4_multisurf_focal_slices_partition(lib):
    """fs_multisurf_score_rows on a partition of the focal samples sums to
    the whole fit's scores (the reference's prange rows are independent)."""
    from fastselect_amd import _lib
    from fastselect_amd.parallel import prepare_inputs
    fx = _fixture("cfg4_multisurf")
    X, y = _inputs(fx)
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
    n = x.shape[0]
    parts = [(0, 6400), (6400, 13001), (13001, n)]
    sums = sum(_lib.multisurf_score("gpu", x, yv, recip, None, False, isd, rows=r)
               for r in parts)
    assert_parity((sums / n).astype(np.float32), fx["scores"], TOL, TOPK)


def test_cfg5_multisurfstar_whole_fit(lib):
    fx = _fixture("cfg5_multisurfstar")
    X, y = _inputs(fx)
    est = lib.MultiSURF(backend="gpu", use_star=True, n_features_to_select=TOPK).fit(X, y)
    assert_parity(est.feature_importances_, fx["scores"], TOL, TOPK)
    _attribute("cfg5_multisurfstar", est.feature_importances_, fx["scores"], False)


@pytest.mark.parametrize("name,star", [("cfg5_surf", False), ("cfg5_surfstar", True)])
def test_cfg5_surf_whole_fit(lib, name, star):
    """SURF / SURF* at BASELINE configs[4] (10000 x 50000, float64 X) as one
    whole fit against the oracle's whole-fit vector (VERDICT r5 missing #2:
    k_surf_avg over every row and the whole column sum, not only the 384-row
    slices below)."""
    fx = _fixture(name)
    assert bool(fx["use_star"]) == star
    X, y = _inputs(fx)
    est = lib.SURF(backend="gpu", use_star=star, n_features_to_select=TOPK).fit(X, y)
    assert est.effective_backend_ == "gpu"
    assert_parity(est.feature_importances_, fx["scores"], TOL, TOPK)


@pytest.mark.parametrize("sparse", ["default", "0"])
@pytest.mark.parametrize("name", ["cfg5_surfstar_slice", "cfg5_surf_slice"])
def test_cfg5_surf_focal_slice(lib, name, sparse, hooks):
    """SURF / SURF* at 10000 x 50000: the oracle's focal-sample slice
    (SURF.py:131-195 over i_range) against fs_surf_score_rows.  A row slice
    takes the sparse pass 2; the sparse hook at 0 forces the dense k_weights ->
    k_score pass 2 that the whole single-device SURF / SURF* fit
    (BASELINE configs[4]) takes, so that path is compared with the oracle at
    size too."""
    from fastselect_amd import _lib
    if sparse != "default":
        hooks("sparse", int(sparse))
    from fastselect_amd.SURF import surf_inputs
    fx = _fixture(name)
    X, y = _inputs(fx)
    x = np.ascontiguousarray(X, dtype=np.float64)
    isd, recip = surf_inputs(x, 10, "gpu")
    lo, hi = (int(v) for v in fx["i_range"])
    sums = _lib.surf_score("gpu", x, np.asarray(y).astype(np.int32), recip,
                           bool(fx["use_star"]), isd, rows=(lo, hi))
    s = (sums / x.shape[0]).astype(np.float32)
    assert_parity(s, fx["scores"], TOL)
    _attribute(name, s, fx["scores"], True)
