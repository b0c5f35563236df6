"""CPU checks of the data-family fixtures (tests/golden/make_families.py):
each regenerates to the committed input hash, and its oracle scores are
finite and carry a usable scale (the GPU parity test compares against them).
"""
import hashlib
import importlib.util
import os

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")
_spec = importlib.util.spec_from_file_location("mk_families",
                                               os.path.join(GOLD, "make_families.py"))
mk = importlib.util.module_from_spec(_spec)
_spec.loader.exec_module(mk)


@pytest.mark.parametrize("name", mk.CASES)
def test_family_fixture_regenerates(name):
    fx = np.load(os.path.join(GOLD, f"family_{name}.npz"), allow_pickle=False)
    X, y = mk.make(name)
    assert X.shape == (mk.N, mk.P) and X.dtype == np.float32
    assert hashlib.sha256(X.tobytes()).hexdigest() == str(fx["x_sha256"])
    assert int(np.sum(y)) == int(fx["y_sum"])
    for key in ("scores", "scores_star"):
        s = fx[key]
        assert s.shape == (mk.P,) and np.all(np.isfinite(s))
        assert np.max(np.abs(s)) > 0.0
