"""Test configuration.

Markers: ``gpu`` -- needs a visible HIP device (MI355X); run with
``pytest -m gpu`` on the GPU box.  Everything else runs on CPU in a few
minutes (``pytest -m "not gpu"``).
"""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a visible HIP GPU (MI355X)")
    config.addinivalue_line("markers", "slow: long-running parity case")


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as O
    O.build()
    return O


from parity_metrics import scale_rel_err, summary, topk_same  # noqa: E402  (tests/ on sys.path)


def assert_parity(a, ref, tol=1e-5, k=None):
    """Scores within `tol` scale-relative, and identical
    top-k index sets.  A failure reports the per-element figures of §8d too."""
    err = scale_rel_err(a, ref)
    assert err <= tol, f"scale-relative error {err:.3e} > {tol:.1e} ({summary(a, ref)})"
    if k is not None:
        ta = set(np.argsort(np.asarray(a))[::-1][:k].tolist())
        tr = set(np.argsort(np.asarray(ref))[::-1][:k].tolist())
        assert ta == tr, f"top-{k} differ: {sorted(ta ^ tr)} ({summary(a, ref)})"


def assert_parity_attributed(a, ref, exact, counts=None, ref_counts=None, tol=1e-5, k=10):
    """The parity bar where the reference's own float32 sums may not allow
    it.  Decisions first: with ``counts`` (our near hit / miss count per row)
    and ``ref_counts`` (oracle_multisurf_decisions) no row may differ.  Then,
    when the reference's float32 arithmetic (``ref``) is within tol / 2 of the
    float64 sums of the same decisions (``exact``, the oracle's accum='f64'),
    the plain bar: ``a`` within ``tol`` of ``ref`` (scale-relative); otherwise
    the residual must be accumulation: ``a`` at least 5x closer to ``exact``
    than ``ref`` is (our terms keep the reference's float32 products, only the
    sums are float64; on the lognormal 3000 x 2000 case those products alone
    leave ~1e-6 against the reference's ~1e-5).  Top-k identical to ``ref``'s."""
    a, ref, exact = (np.asarray(v, dtype=np.float64) for v in (a, ref, exact))
    if counts is not None:
        c = np.asarray(counts).reshape(-1, 2).astype(np.int64)
        rc = np.asarray(ref_counts).reshape(-1, 2).astype(np.int64)
        flipped = int(np.sum(np.any(c != rc, axis=1)))
        assert flipped == 0, f"{flipped} rows decide differently from the reference"
    scale = np.max(np.abs(exact))
    ref_err = np.max(np.abs(ref - exact)) / scale
    if ref_err < 0.5 * tol:
        assert_parity(a, ref, tol, k)
        return
    acc_err = np.max(np.abs(a - exact)) / scale
    assert acc_err <= 0.2 * ref_err, (
        f"{acc_err:.3e} from the float64 sums, reference arithmetic {ref_err:.3e} "
        f"({summary(a, ref)})")
    # an absolute ceiling against the reference too: a regression
    # that moved the scores away from both the reference and the exact sums
    # would fail here even where the 5x bar above held
    ref_dist = np.max(np.abs(a - ref)) / scale
    assert ref_dist <= ref_err + tol, (
        f"{ref_dist:.3e} from the reference, above its own {ref_err:.3e} + {tol:.0e} "
        f"({summary(a, ref)})")
    ta = set(np.argsort(a)[::-1][:k].tolist())
    tr = set(np.argsort(ref)[::-1][:k].tolist())
    assert ta == tr, f"top-{k} differ: {sorted(ta ^ tr)} ({summary(a, ref)})"


@pytest.fixture
def hooks():
    """fs_test_hook overrides for one test (``hooks("ksplit", 4)``), reset
    afterwards (the library reads no environment variable for these)."""
    from fastselect_amd import _lib
    _lib.set_test_hook("reset")
    yield _lib.set_test_hook
    _lib.set_test_hook("reset")
