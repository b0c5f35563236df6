"""The committed full-size decision fixtures (tests/golden/make_fullsize.py
--decisions: oracle_multisurf_decisions, the reference's near hit / near
miss counts per row at cfg2 and cfg4) describe the same inputs as the score
fixtures the GPU tests compare against: same X (sha256 of the float32
matrix), same labels, one (hits, misses) pair per sample.  The GPU tests
(tests/test_gpu_refacc.py::test_decisions_row_by_row) and bench.py's
decisions_vs_reference read them."""
import os

import numpy as np
import pytest

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.mark.parametrize("name", ["cfg2_multisurf", "cfg4_multisurf"])
def test_decision_fixture_matches_score_fixture(name):
    dec = np.load(os.path.join(GOLD, f"fullsize_{name}_decisions.npz"), allow_pickle=False)
    fx = np.load(os.path.join(GOLD, f"fullsize_{name}.npz"), allow_pickle=False)
    assert str(dec["x_sha256"]) == str(fx["x_sha256"])
    n = int(dec["n"])
    counts = dec["counts"].reshape(-1, 2)
    assert counts.shape == (n, 2)
    assert dec["thr"].shape == (n,)
    # every row has near neighbours, none more than the other samples
    tot = counts.sum(axis=1)
    assert (tot > 0).all() and (tot <= n - 1).all()
    assert (counts >= 0).all()
