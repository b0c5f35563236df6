"""Reference-order accumulation (``accumulation='reference'``,
fs_set_accumulation(FS_ACCUM_REFERENCE)) on the native CPU backend: the
reference's float32 per-sample sums and float32 sequential column sums
(MultiSURF.py:198-253, ReliefF.py:181-220; SURF / SURF* in the reference's
n_jobs=1 order, SURF.py:139-218), so the scores must equal the
oracle's (oracle/relief_oracle.c, the restatement of those lines) BIT FOR BIT
-- including the inputs where the reference's own float32 error exceeds
1e-5 of max |s| and the default mode can only be judged by the attributed
bar (VERDICT r4 missing #1).  tests/test_gpu_refacc.py runs the same cases
through the HIP kernels.
"""
import warnings

import numpy as np
import pytest

from fastselect_amd import SURF, MultiSURF, MultiSURFstar, ReliefF, SURFstar, TuRF, _lib
from test_random_parity import make_case, make_tail_case


def assert_bitexact(got, ref):
    got = np.asarray(got, dtype=np.float32)
    ref = np.asarray(ref, dtype=np.float32)
    assert got.shape == ref.shape
    bad = np.flatnonzero(got.view(np.uint32) != ref.view(np.uint32))
    assert bad.size == 0, (
        f"{bad.size} of {got.size} scores differ from the oracle; first {bad[:5]}: "
        f"{got[bad[:5]]} vs {ref[bad[:5]]}")


def verdict_case(kind, n, p, seed=7):
    """VERDICT r4 missing #1's inputs: signal-free labels over heavy-tailed
    columns, where the reference's float32 sums sit 1.1-2.3e-5 of max |s|
    from the float64 sums (and top-k moves with them for the outliers)."""
    rng = np.random.default_rng(seed)
    if kind == "exp4z":
        X = np.exp(4.0 * rng.standard_normal((n, p)))
    elif kind == "pareto1":
        X = rng.pareto(1.0, (n, p)) + 1.0
    elif kind == "outlier":
        X = rng.standard_normal((n, p))
        X[rng.integers(0, n, p), np.arange(p)] = 1e7
    else:
        raise ValueError(kind)
    y = rng.integers(0, 2, n)
    return X.astype(np.float32), y


def fit_ref(est_cls, X, y, **kw):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)
        return est_cls(accumulation="reference", **kw).fit(X, y).feature_importances_


@pytest.mark.parametrize("seed", range(0, 40, 3))
def test_sweep_bitexact_cpu(oracle, seed):
    X, y, dl, k = make_case(seed)
    assert_bitexact(fit_ref(MultiSURF, X, y, backend="cpu", discrete_limit=dl),
                    oracle.multisurf_scores(X, y, discrete_limit=dl))
    assert_bitexact(fit_ref(MultiSURFstar, X, y, backend="cpu", discrete_limit=dl),
                    oracle.multisurf_scores(X, y, use_star=True, discrete_limit=dl))
    if X.shape[0] > k:
        assert_bitexact(fit_ref(ReliefF, X, y, backend="cpu", discrete_limit=dl, n_neighbors=k),
                        oracle.relieff_scores(X, y, n_neighbors=k, discrete_limit=dl))
    assert_bitexact(fit_ref(SURF, X, y, backend="cpu", discrete_limit=dl),
                    oracle.surf_scores(X, y, discrete_limit=dl))
    assert_bitexact(fit_ref(SURFstar, X, y, backend="cpu", discrete_limit=dl),
                    oracle.surf_scores(X, y, use_star=True, discrete_limit=dl))


@pytest.mark.parametrize("seed", [0, 3, 7])
def test_tail_bitexact_cpu(oracle, seed):
    X, y, k = make_tail_case(seed)
    assert_bitexact(fit_ref(MultiSURF, X, y, backend="cpu"), oracle.multisurf_scores(X, y))
    assert_bitexact(fit_ref(MultiSURF, X, y, backend="cpu", use_star=True),
                    oracle.multisurf_scores(X, y, use_star=True))
    assert_bitexact(fit_ref(ReliefF, X, y, backend="cpu", n_neighbors=k),
                    oracle.relieff_scores(X, y, n_neighbors=k))
    for star in (False, True):
        assert_bitexact(fit_ref(SURF, X, y, backend="cpu", use_star=star),
                        oracle.surf_scores(X, y, use_star=star))


@pytest.mark.parametrize("kind", ["exp4z", "pareto1", "outlier"])
def test_verdict_cases_bitexact_cpu(oracle, kind):
    X, y = verdict_case(kind, 900, 240)
    for star in (False, True):
        ref = oracle.multisurf_scores(X, y, use_star=star)
        got = fit_ref(MultiSURF, X, y, backend="cpu", use_star=star)
        assert_bitexact(got, ref)
        assert np.array_equal(np.argsort(got)[::-1][:10], np.argsort(ref)[::-1][:10])
        ref = oracle.surf_scores(X, y, use_star=star)
        got = fit_ref(SURF, X, y, backend="cpu", use_star=star)
        assert_bitexact(got, ref)
        assert np.array_equal(np.argsort(got)[::-1][:10], np.argsort(ref)[::-1][:10])


def tie_order_case(seed, n_fill=60):
    """A focal sample whose three nearest hits share one key exactly (the
    grid column) while one feature's diffs to them are 1, 2^-53, 2^-53:
    summed in float64 as 1 + e + e they give 1, as e + e + 1 they give
    1 + 2^-52, and the three misses sum to 1 -- so the focal row's float32
    update is 0 or -2^-52 / 3 depending on the ORDER of the tied hits, which
    the reference takes from numba's quicksort of the whole row
    (ReliefF.py:157-207).  Far filler samples of both classes vary that
    quicksort's path.  Returns X, y and the focal row (score it alone through
    a one-row slice: the column sum of one row is its update)."""
    eps = 2.0 ** -53
    rng = np.random.default_rng(seed)
    rows = [(0.0, 0.0, 0), (0.0, 1.0, 0), (1.0, eps, 0), (1.0, eps, 0),
            (0.0, 1.0, 1), (0.25, 0.0, 1), (0.25, 0.0, 1)]
    rows += [(rng.uniform(0.5, 1.0), 0.5 + eps * rng.integers(2, 40), int(rng.integers(0, 2)))
             for _ in range(n_fill)]
    perm = rng.permutation(len(rows))
    X = np.array([rows[q][:2] for q in perm])
    y = np.array([rows[q][2] for q in perm])
    return X, y, int(np.flatnonzero(perm == 0)[0])


def relieff_row(backend, X, y, i, k=3, dl=2):
    """ReliefF reference-order score of focal row i alone (its float32
    update, / n)."""
    from fastselect_amd.ReliefF import relieff_inputs
    x32, y_enc, recip, isd, cp = relieff_inputs(X, y, dl, backend)
    with _lib.accumulation("reference"):
        s = _lib.relieff_score(backend, x32, y_enc, recip, isd, k, cp, rows=(i, i + 1))
    return (s / X.shape[0]).astype(np.float32)


def test_relieff_tied_neighbours_in_quicksort_order_cpu(oracle):
    """VERDICT r5 missing #3: neighbours at one key in numba's quicksort
    order, not index order.  Of these 40 seeds, the index order gives a
    different float32 update than the reference on 10 (measured before the
    replay was built); every one must now be the oracle's bit for bit."""
    for seed in range(40):
        X, y, i = tie_order_case(seed)
        assert_bitexact(relieff_row("cpu", X, y, i),
                        oracle.relieff_scores(X, y, n_neighbors=3, discrete_limit=2,
                                              i_range=(i, i + 1)))
    X, y, _ = tie_order_case(1)
    assert_bitexact(fit_ref(ReliefF, X, y, backend="cpu", n_neighbors=3, discrete_limit=2),
                    oracle.relieff_scores(X, y, n_neighbors=3, discrete_limit=2))


def test_relieff_tie_replay_only_where_order_matters_cpu(oracle, hooks):
    """Grid-valued continuous features tie neighbour keys on most rows, but
    their diffs add exactly in any order, so the replay is skipped for them
    (ref_order_matters): the result is the oracle's and the same as with the
    replay forced on every tied row (the rf_ref_replay hook)."""
    rng = np.random.default_rng(8)
    X = rng.integers(0, 12, (600, 40)) / 11.0
    y = rng.integers(0, 2, 600)
    ref = oracle.relieff_scores(X, y, n_neighbors=5, discrete_limit=2)
    assert_bitexact(fit_ref(ReliefF, X, y, backend="cpu", n_neighbors=5, discrete_limit=2), ref)
    hooks("rf_ref_replay", 1)
    assert_bitexact(fit_ref(ReliefF, X, y, backend="cpu", n_neighbors=5, discrete_limit=2), ref)


def test_relieff_classes_and_small_class_cpu(oracle):
    rng = np.random.default_rng(3)
    X = np.exp(2.0 * rng.standard_normal((400, 60)))
    X[:, :8] = rng.integers(0, 4, (400, 8))          # discrete columns
    y = rng.integers(0, 3, 400)
    y[:3] = 3                                        # a class smaller than k
    for k in (1, 5, 10):
        assert_bitexact(fit_ref(ReliefF, X, y, backend="cpu", n_neighbors=k),
                        oracle.relieff_scores(X, y, n_neighbors=k))


def test_rows_slice_is_the_oracle_slice_cpu(oracle):
    """fs_multisurf_score_rows in reference order: the float32 column sum of
    the slice's rows, i.e. the oracle restricted to i_range."""
    X, y = verdict_case("exp4z", 500, 90, seed=2)
    x, yv, recip, isd = (X, y.astype(np.float64), *_recip_disc(X))
    with _lib.accumulation("reference"):
        sums = _lib.multisurf_score("cpu", x, yv, recip, None, False, isd, rows=(128, 384))
    ref = oracle.multisurf_scores(X, y, i_range=(128, 384))
    assert_bitexact((sums / X.shape[0]).astype(np.float32), ref)


def test_surf_rows_slice_and_ex_call_cpu(oracle):
    """fs_surf_score_rows in reference order is the float32 column sum of the
    slice's rows (the oracle restricted to i_range); fs_surf_score_ex takes
    the mode as an argument and leaves the thread's mode alone."""
    import ctypes
    X, y = verdict_case("pareto1", 400, 70, seed=3)
    x = X.astype(np.float64)
    rng = x.max(0) - x.min(0)                                  # SURF.py:352-355
    rng[rng == 0] = 1.0
    recip = (1.0 / rng).astype(np.float32)
    isd = np.zeros(x.shape[1], np.uint8)
    yi = y.astype(np.int32)
    for star in (False, True):
        with _lib.accumulation("reference"):
            sums = _lib.surf_score("cpu", x, yi, recip, star, isd, rows=(128, 300))
        assert_bitexact((sums / X.shape[0]).astype(np.float32),
                        oracle.surf_scores(X, y, use_star=star, i_range=(128, 300)))
        out = np.zeros(x.shape[1], np.float32)
        L = _lib.lib()
        f32p = ctypes.POINTER(ctypes.c_float)
        _lib.check(L.fs_surf_score_ex(0, 0, x.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                      x.shape[0], x.shape[1],
                                      yi.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)),
                                      recip.ctypes.data_as(f32p), int(star),
                                      isd.ctypes.data_as(ctypes.POINTER(ctypes.c_uint8)), -1, 1,
                                      out.ctypes.data_as(f32p)))
        assert L.fs_get_accumulation() == 0
        assert_bitexact(out, oracle.surf_scores(X, y, use_star=star))
    with pytest.raises(ValueError, match="accumulation"):
        _lib.check(L.fs_surf_score_ex(0, 0, None, 0, 0, None, None, 0, None, -1, 7, None))


def _recip_disc(X):
    r = (X.max(0) - X.min(0)).astype(np.float32)
    r[r == 0] = 1
    return (1.0 / r).astype(np.float32), np.zeros(X.shape[1], np.uint8)


def turf_oracle(score, X, n_select, pct):
    """TuRF's elimination loop (TuRF.py:61-120) over oracle scores."""
    active = np.arange(X.shape[1])
    scores = score(X)
    first = scores.copy()
    while len(active) > n_select:
        drop = min(max(1, int(len(active) * pct)), len(active) - n_select)
        active = np.delete(active, np.argsort(scores)[:drop])
        scores = score(X[:, active])
    return first, np.sort(active[np.argsort(scores)[::-1]])


def test_turf_reference_mode_cpu(oracle):
    """TuRF re-scores column subsets through the resident plan, which keeps
    the mode it was created with (fs_plan_set_features): every round's
    scores are the oracle's, so the eliminations are too."""
    X, y = verdict_case("pareto1", 300, 60, seed=4)
    cases = ((MultiSURF(backend="cpu", accumulation="reference"),
              lambda Z: oracle.multisurf_scores(Z, y)),
             (ReliefF(backend="cpu", n_neighbors=5, accumulation="reference"),
              lambda Z: oracle.relieff_scores(Z, y, n_neighbors=5)),
             (SURFstar(backend="cpu", accumulation="reference"),
              lambda Z: oracle.surf_scores(Z, y, use_star=True)))
    for base, score in cases:
        t = TuRF(base, n_features_to_select=10, pct_remove=0.25).fit(X, y)
        first, top = turf_oracle(score, X, 10, 0.25)
        assert_bitexact(t.feature_importances_, first)
        assert np.array_equal(t.top_features_, top)


def test_plan_keeps_creation_mode_cpu(oracle):
    from fastselect_amd import parallel
    X, y = verdict_case("exp4z", 300, 50, seed=5)
    x, yv, recip, isd = parallel.prepare_inputs(X, y, backend="cpu")
    job = parallel.ShardedMultiSURF(x, yv, recip, isd, backend="cpu", shard=False,
                                    accumulation="reference")
    try:
        assert _lib.lib().fs_get_accumulation() == 0   # the context was left
        assert_bitexact(job.step().numpy(), oracle.multisurf_scores(X, y))
        job.set_features(np.arange(10, 40))
        assert_bitexact(job.step().numpy(), oracle.multisurf_scores(X[:, 10:40], y))
    finally:
        job.close()


def test_accumulation_errors():
    X, y = verdict_case("exp4z", 60, 8)
    with pytest.raises(ValueError, match="accumulation"):
        MultiSURF(backend="cpu", accumulation="f16").fit(X, y)
    with pytest.raises(ValueError, match="accumulation"):
        ReliefF(backend="cpu", accumulation=None).fit(X, y)
    with pytest.raises(ValueError, match="accumulation"):
        SURF(backend="cpu", accumulation="exact").fit(X, y)
    # the mode is per thread and restored by the context manager
    assert _lib.lib().fs_get_accumulation() == 0
    with _lib.accumulation("reference"):
        assert _lib.lib().fs_get_accumulation() == 1
    assert _lib.lib().fs_get_accumulation() == 0
    with pytest.raises(ValueError, match="one device"):
        from fastselect_amd import _base
        _base.check_accumulation_devices("reference", [0, 1])


def test_reference_over_ranks_is_gpu_only_cpu():
    """Reference order over world > 1 ranks is the GPU plans' masks / chains
    / chained column sums (fs_plan_ref_*); the CPU backend refuses it, and the
    fs_plan_ref_* calls refuse CPU plans."""
    from fastselect_amd import parallel
    X, y = verdict_case("exp4z", 200, 30, seed=2)
    x, yv, recip, isd = parallel.prepare_inputs(X, y, backend="cpu")
    with _lib.accumulation("reference"):
        with pytest.raises(RuntimeError, match="GPU backend"):
            _lib.Plan("cpu", x, yv, recip, isd, rank=0, world=2)
        plan = _lib.Plan("cpu", x, yv, recip, isd)
    try:
        with pytest.raises(RuntimeError, match="reference-order"):
            plan.ref_mask_words()
        with pytest.raises(RuntimeError, match="GPU backend"):
            plan.set_shard(1, 2)
    finally:
        plan.close()


def test_fast_mode_unchanged_cpu():
    """The default stays the fast path: same scores as before the option."""
    X, y = verdict_case("exp4z", 200, 40, seed=9)
    a = MultiSURF(backend="cpu").fit(X, y).feature_importances_
    b = MultiSURF(backend="cpu", accumulation="fast").fit(X, y).feature_importances_
    assert np.array_equal(a, b)
