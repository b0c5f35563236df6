"""Exact MultiSURF thresholds for the rows a refined pair sits close to
(exact_thresholds in fs_select.hip and fs_cpu.cpp).

The mean of a row's quantised distances is corrected exactly, but the spread
comes from the quantised second moments, so a threshold is off by ~(band /
12) / sqrt(n - 1) integer units; a refined pair -- the reference's own
distance -- that falls between the two values was decided differently (one
row of 16384 on the uniform-noise family, tests/test_gpu_families.py).  The
rows whose refined pairs lie that close now get their threshold from exact
distances to every other sample (MultiSURF.py:174-196).

The thr_exact_all test hook (fs_test_hook) takes every row through that route, so the
decisions must then be the oracle's (oracle_multisurf_decisions) row by row,
on both backends and on 16-bit operands too; the default route must give
the oracle's decisions on the same data.
"""
import numpy as np
import pytest

from conftest import assert_parity
from oracle import oracle as O


def _data(kind, n, p, seed):
    rng = np.random.default_rng(seed)
    if kind == "classification":
        from sklearn.datasets import make_classification
        X, y = make_classification(n_samples=n, n_features=p, n_informative=10, n_redundant=20,
                                   random_state=seed)
    elif kind == "lognormal":
        X = np.exp(3.0 * rng.standard_normal((n, p)))
        y = rng.integers(0, 2, n)
    elif kind == "mixed":
        X = rng.standard_normal((n, p))
        X[:, : p // 4] = rng.integers(0, 4, (n, p // 4))       # discrete columns
        X[:, p // 4: p // 2] = np.round(X[:, p // 4: p // 2], 1)  # coarse grid
        y = rng.integers(0, 3, n)
    else:  # uniform noise, unrelated labels
        X = rng.uniform(size=(n, p))
        y = rng.integers(0, 2, n)
    return X.astype(np.float32), y


def _step(X, y, backend):
    from fastselect_amd import parallel
    x, yv, recip, isd = parallel.prepare_inputs(X, y, backend=backend)
    job = parallel.ShardedMultiSURF(x, yv, recip, isd, backend=backend, shard=False)
    try:
        s = job.step().cpu().numpy()
        counts = job.counts.cpu().numpy().reshape(-1, 2).astype(np.int64)
    finally:
        job.close()
    return s, counts


def _check(X, y, backend, hooks, all_rows):
    hooks("thr_exact_all", 1 if all_rows else 0)
    s, counts = _step(X, y, backend)
    _, ref_counts = O.multisurf_decisions(X, y)
    flipped = np.flatnonzero(np.any(counts != ref_counts, axis=1))
    assert flipped.size == 0, f"rows {flipped[:10].tolist()} decide differently from the reference"
    assert_parity(s, O.multisurf_scores(X, y), 1e-5, 10)


CASES = [("classification", 400, 300, 0), ("lognormal", 400, 200, 1), ("mixed", 360, 160, 2),
         ("uniform", 500, 120, 3)]


@pytest.mark.parametrize("kind,n,p,seed", CASES)
@pytest.mark.parametrize("all_rows", [True, False])
def test_cpu_backend_decisions(kind, n, p, seed, all_rows, hooks):
    X, y = _data(kind, n, p, seed)
    _check(X, y, "cpu", hooks, all_rows)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,p,seed", CASES)
@pytest.mark.parametrize("all_rows", [True, False])
def test_gpu_decisions(kind, n, p, seed, all_rows, hooks):
    X, y = _data(kind, n, p, seed)
    _check(X, y, "gpu", hooks, all_rows)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["uniform", "classification"])
def test_gpu_16bit_operands_exact_thresholds_everywhere(kind, hooks):
    """16-bit pass-1 operands (thresholds 256x coarser than on 32-bit ones):
    with every threshold exact, the refinement band alone must bring each
    decision to the reference's."""
    hooks("q16", 1)
    hooks("q16_guard_off", 1)
    X, y = _data(kind, 1200, 400, 5)
    _check(X, y, "gpu", hooks, True)
