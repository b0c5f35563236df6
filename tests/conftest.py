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
