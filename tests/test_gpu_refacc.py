"""Reference-order accumulation on the HIP path (fs_refacc.hip): scores
BIT-IDENTICAL to the oracle's float32 arithmetic on

  * the n = 16384 uniform-noise and lognormal families, whose reference
    float32 sums sit 2.6-2.9e-5 of max |s| from the float64 sums
    (tests/golden/family_*.npz, oracle vectors);
  * the heavy-tail sweep of tests/test_random_parity.py and the small sweep;
  * VERDICT r4's n = 2500, p = 600 signal-free cases (exp(4z), Pareto(1),
    one 1e7 outlier per column: MultiSURF*'s top-10 there is the reference's
    only when its float32 rounding is replayed);
  * the BASELINE configurations cfg2, cfg3 (2 and 3 classes) and cfg4 -- the
    north star, 20000 x 20000 -- against the full-size oracle fixtures;
  * SURF / SURF* in the reference's n_jobs=1 order (round 6, VERDICT r5
    next #1): the same sweeps and verdict cases, row panels, rows slices,
    ranks, TuRF, the cfg5 focal slices and the cfg5 whole fits.

The oracle runs live for the small cases (oracle/_build, C, the box's host
threads); the large ones use the committed fixtures with the sha256 of X.
"""
import hashlib
import importlib.util
import os
import warnings

import numpy as np
import pytest

from test_random_parity import make_case, make_tail_case
from test_refacc import assert_bitexact, verdict_case

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = os.path.join(HERE, "golden")


@pytest.fixture(scope="module")
def F():
    import fastselect_amd
    from fastselect_amd import _lib
    if _lib.device_count() < 1:
        pytest.fail("no HIP device visible")
    return fastselect_amd


def fit_ref(est, X, y):
    with warnings.catch_warnings():
        warnings.simplefilter("ignore", UserWarning)
        return est.fit(X, y).feature_importances_


def _families():
    spec = importlib.util.spec_from_file_location("mk_families",
                                                  os.path.join(GOLD, "make_families.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    return mk


@pytest.mark.parametrize("name", ["uniform_16k", "lognormal_16k", "mixed_16k"])
@pytest.mark.parametrize("star", [False, True])
def test_family_bitexact(F, name, star):
    fx = np.load(os.path.join(GOLD, f"family_{name}.npz"), allow_pickle=False)
    X, y = _families().make(name)
    assert hashlib.sha256(X.tobytes()).hexdigest() == str(fx["x_sha256"])
    s = fit_ref(F.MultiSURF(backend="gpu", use_star=star, accumulation="reference"), X, y)
    assert_bitexact(s, fx["scores_star" if star else "scores"])


@pytest.mark.parametrize("seed", range(10))
def test_tail_sweep_bitexact(F, oracle, seed):
    X, y, k = make_tail_case(seed)
    for star in (False, True):
        assert_bitexact(
            fit_ref(F.MultiSURF(backend="gpu", use_star=star, accumulation="reference"), X, y),
            oracle.multisurf_scores(X, y, use_star=star))
    assert_bitexact(
        fit_ref(F.ReliefF(backend="gpu", n_neighbors=k, accumulation="reference"), X, y),
        oracle.relieff_scores(X, y, n_neighbors=k))
    for star in (False, True):
        assert_bitexact(
            fit_ref(F.SURF(backend="gpu", use_star=star, accumulation="reference"), X, y),
            oracle.surf_scores(X, y, use_star=star))


@pytest.mark.parametrize("seed", range(0, 40, 2))
def test_small_sweep_bitexact(F, oracle, seed):
    X, y, dl, k = make_case(seed)
    for star in (False, True):
        assert_bitexact(
            fit_ref(F.MultiSURF(backend="gpu", use_star=star, discrete_limit=dl,
                                accumulation="reference"), X, y),
            oracle.multisurf_scores(X, y, use_star=star, discrete_limit=dl))
    if X.shape[0] > k:
        assert_bitexact(
            fit_ref(F.ReliefF(backend="gpu", n_neighbors=k, discrete_limit=dl,
                              accumulation="reference"), X, y),
            oracle.relieff_scores(X, y, n_neighbors=k, discrete_limit=dl))
    for star in (False, True):
        assert_bitexact(
            fit_ref(F.SURF(backend="gpu", use_star=star, discrete_limit=dl,
                           accumulation="reference"), X, y),
            oracle.surf_scores(X, y, use_star=star, discrete_limit=dl))


@pytest.mark.parametrize("kind", ["exp4z", "pareto1", "outlier"])
def test_verdict_cases_bitexact(F, oracle, kind):
    X, y = verdict_case(kind, 2500, 600)
    for star in (False, True):
        ref = oracle.multisurf_scores(X, y, use_star=star)
        got = fit_ref(F.MultiSURF(backend="gpu", use_star=star, accumulation="reference"), X, y)
        assert_bitexact(got, ref)
        assert np.array_equal(np.argsort(got)[::-1][:10], np.argsort(ref)[::-1][:10])
        ref = oracle.surf_scores(X, y, use_star=star)
        got = fit_ref(F.SURF(backend="gpu", use_star=star, accumulation="reference"), X, y)
        assert_bitexact(got, ref)
        assert np.array_equal(np.argsort(got)[::-1][:10], np.argsort(ref)[::-1][:10])


def test_surf_discrete_and_mixed_bitexact(F, oracle):
    """SURF's discrete features add 1 / 0 to the chains (SURF.py:153-154):
    discrete-only and mixed layouts, including a 128-feature block that
    holds both kinds."""
    rng = np.random.default_rng(17)
    X = np.exp(1.5 * rng.standard_normal((700, 300)))
    X[:, 100:140] = rng.integers(0, 4, (700, 40))
    X[:, 250:] = rng.integers(0, 3, (700, 50))
    y = rng.integers(0, 2, 700)
    for star in (False, True):
        assert_bitexact(
            fit_ref(F.SURF(backend="gpu", use_star=star, accumulation="reference"), X, y),
            oracle.surf_scores(X, y, use_star=star))
    Xd = rng.integers(0, 5, (500, 130)).astype(np.float64)
    for star in (False, True):
        assert_bitexact(
            fit_ref(F.SURF(backend="gpu", use_star=star, accumulation="reference"), Xd, y[:500]),
            oracle.surf_scores(Xd, y[:500], use_star=star))


def test_surf_panels_chain_the_column_sums(F, oracle, hooks):
    """A one-shot SURF scored in row panels continues one float32 column sum
    across the panels (each panel's plan seeded with the previous sums)."""
    hooks("row_panel", 256)
    X, y = verdict_case("exp4z", 1000, 90, seed=12)
    for star in (False, True):
        assert_bitexact(
            fit_ref(F.SURF(backend="gpu", use_star=star, accumulation="reference"), X, y),
            oracle.surf_scores(X, y, use_star=star))


def test_surf_rows_slice_is_the_oracle_slice(F, oracle):
    from fastselect_amd import _lib
    from fastselect_amd.SURF import surf_inputs
    X, y = verdict_case("outlier", 1500, 200, seed=5)
    x = X.astype(np.float64)
    isd, recip = surf_inputs(x, 10, "gpu")
    for star in (False, True):
        with _lib.accumulation("reference"):
            sums = _lib.surf_score("gpu", x, y.astype(np.int32), recip, star, isd,
                                   rows=(300, 1100))
        assert_bitexact((sums / X.shape[0]).astype(np.float32),
                        oracle.surf_scores(X, y, use_star=star, i_range=(300, 1100)))


def test_relieff_tied_neighbours_in_quicksort_order(F, oracle):
    """Neighbours at one key summed in numba's quicksort order
    (k_rf_ref_ties; VERDICT r5 missing #3): the crafted rows whose float32
    update depends on that order (tests/test_refacc.py tie_order_case; the
    index order misses 10 of these 40), then a whole fit."""
    from test_refacc import relieff_row, tie_order_case
    for seed in range(40):
        X, y, i = tie_order_case(seed)
        assert_bitexact(relieff_row("gpu", X, y, i),
                        oracle.relieff_scores(X, y, n_neighbors=3, discrete_limit=2,
                                              i_range=(i, i + 1)))
    for seed in (1, 12):
        X, y, _ = tie_order_case(seed, n_fill=3000)
        assert_bitexact(
            fit_ref(F.ReliefF(backend="gpu", n_neighbors=3, discrete_limit=2,
                              accumulation="reference"), X, y),
            oracle.relieff_scores(X, y, n_neighbors=3, discrete_limit=2))


def test_relieff_tie_replay_only_where_order_matters(F, oracle, hooks):
    """Rows whose tied neighbours' diffs add exactly in any order skip the
    quicksort replay (k_rf_ref_order_matters): grid-valued continuous data,
    ties on most rows, is the oracle's with the check and with the replay
    forced on every tied row (rf_ref_replay)."""
    rng = np.random.default_rng(8)
    X = rng.integers(0, 12, (3000, 64)) / 11.0
    y = rng.integers(0, 3, 3000)
    ref = oracle.relieff_scores(X, y, n_neighbors=5, discrete_limit=2)
    for replay in (0, 1):
        hooks("rf_ref_replay", replay)
        assert_bitexact(fit_ref(F.ReliefF(backend="gpu", n_neighbors=5, discrete_limit=2,
                                          accumulation="reference"), X, y), ref)


def test_relieff_panels_chain_the_column_sums(F, oracle, hooks):
    """A one-shot ReliefF scored in row panels (the row_panel test hook
    forces their height) continues one float32 column sum across the panels."""
    hooks("row_panel", 256)
    rng = np.random.default_rng(21)
    X = np.exp(2.0 * rng.standard_normal((1000, 80)))
    y = rng.integers(0, 3, 1000)
    assert_bitexact(
        fit_ref(F.ReliefF(backend="gpu", n_neighbors=7, accumulation="reference"), X, y),
        oracle.relieff_scores(X, y, n_neighbors=7))


def test_rows_slice_is_the_oracle_slice(F, oracle):
    from fastselect_amd import _lib
    from fastselect_amd.parallel import prepare_inputs
    X, y = verdict_case("exp4z", 1500, 300, seed=3)
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
    with _lib.accumulation("reference"):
        sums = _lib.multisurf_score("gpu", x, yv, recip, None, False, isd, rows=(300, 1100))
    assert_bitexact((sums / X.shape[0]).astype(np.float32),
                    oracle.multisurf_scores(X, y, i_range=(300, 1100)))


def _ref_rank_worker(rank, world, port, out_path, rows):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    X, y = verdict_case("pareto1", 1300, 200, seed=8)
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu", device=0)
    for star in (False, True):
        job = ShardedMultiSURF(x, yv, recip, isd, use_star=star, backend="gpu", device=0,
                               rows=rows, accumulation="reference")
        assert job.ref_chain and job.world == world
        np.save(f"{out_path}.{int(star)}.{rank}.npy", job.step().cpu().numpy())
        np.save(f"{out_path}.{int(star)}.{rank}.again.npy", job.step().cpu().numpy())
        job.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,rows", [(2, None), (3, None), (2, (170, 1111))])
def test_ranks_chain_the_column_sums_bitexact(F, oracle, tmp_path, world, rows):
    """Reference order over world ranks (two or three processes sharing
    cuda:0, gloo): each rank's pair-tile decisions as masks, their SUM
    all-reduce, every rank's chains for its block of focal rows, then the
    float32 column sums handed from rank to rank -- every rank ends with the
    oracle's scores bit for bit, step after step (fs_plan_ref_masks /
    fs_plan_ref_pass2 / fs_plan_ref_sums)."""
    import torch.multiprocessing as mp

    from test_gpu_dist import _port
    out = str(tmp_path / "ref")
    mp.spawn(_ref_rank_worker, args=(world, _port(), out, rows), nprocs=world, join=True)
    X, y = verdict_case("pareto1", 1300, 200, seed=8)
    for star in (False, True):
        if rows is None:
            ref = oracle.multisurf_scores(X, y, use_star=star)
        else:  # a focal slice: the sums over those samples, divided by n
            ref = oracle.multisurf_scores(X, y, use_star=star, i_range=rows)
        for r in range(world):
            for tag in ("", ".again"):
                assert_bitexact(np.load(f"{out}.{int(star)}.{r}{tag}.npy"), ref)


def test_forced_tile_shards_bitexact(F, oracle, hooks):
    """n beyond HBM: the one-shot call in V tile shards writes every shard's
    decisions into the masks before the chains run."""
    hooks("shards", 3)
    X, y = verdict_case("pareto1", 1300, 200, seed=8)
    for star in (False, True):
        assert_bitexact(
            fit_ref(F.MultiSURF(backend="gpu", use_star=star, accumulation="reference"), X, y),
            oracle.multisurf_scores(X, y, use_star=star))


def test_plan_narrow_then_wide_features_bitexact(F, oracle):
    """a reference-order plan created on a few features
    and re-targeted to all of them (fs_plan_set_features) keeps fixing every
    flagged row's threshold -- its batch counts are sized for any layout --
    and scores the wide layout as a fresh plan would, bit for bit."""
    import torch

    from fastselect_amd import _lib
    from fastselect_amd.parallel import prepare_inputs
    X, y = verdict_case("exp4z", 4500, 240, seed=13)
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
    dev = torch.device("cuda", 0)
    n, p = x.shape
    rs = torch.zeros(3 * n, dtype=torch.float64, device=dev)
    cnt = torch.zeros(2 * n, dtype=torch.float64, device=dev)
    with _lib.accumulation("reference"):
        plan = _lib.Plan("gpu", x, yv, recip, isd, feat_idx=np.arange(50))
    try:
        for fidx in (np.arange(50), None):
            if fidx is None:
                plan.set_features(None)
            sc = torch.zeros(plan.n_kept, dtype=torch.float64, device=dev)
            torch.cuda.synchronize()  # the plan runs on its own stream
            plan.pass1(rs.data_ptr())
            plan.select(rs.data_ptr(), cnt.data_ptr())
            plan.pass2(cnt.data_ptr(), sc.data_ptr())
            torch.cuda.synchronize()
            got = (sc.cpu().numpy() / n).astype(np.float32)
            Z = X if fidx is None else X[:, fidx]
            assert_bitexact(got, oracle.multisurf_scores(Z, y))
    finally:
        plan.close()


def test_turf_resident_bitexact(F, oracle):
    from test_refacc import turf_oracle
    X, y = verdict_case("exp4z", 1200, 120, seed=6)
    cases = ((F.MultiSURF(backend="gpu", accumulation="reference"),
              lambda Z: oracle.multisurf_scores(Z, y)),
             (F.ReliefF(backend="gpu", n_neighbors=5, accumulation="reference"),
              lambda Z: oracle.relieff_scores(Z, y, n_neighbors=5)),
             (F.SURFstar(backend="gpu", accumulation="reference"),
              lambda Z: oracle.surf_scores(Z, y, use_star=True)))
    for base, score in cases:
        t = F.TuRF(base, n_features_to_select=12, pct_remove=0.3).fit(X, y)
        first, top = turf_oracle(score, X, 12, 0.3)
        assert_bitexact(t.feature_importances_, first)
        assert np.array_equal(t.top_features_, top)


# ---- BASELINE configurations at full size --------------------------------------------
from test_gpu_baseline import _fixture, _inputs  # noqa: E402


@pytest.mark.parametrize("name,algo,kw", [
    ("cfg2_multisurf", "multisurf", {}),
    ("cfg3_relieff_k10", "relieff", {"n_neighbors": 10}),
    ("cfg3_relieff_k10_3class", "relieff", {"n_neighbors": 10}),
    ("cfg5_multisurfstar", "multisurf", {"use_star": True}),
    ("cfg5_surf", "surf", {}),
    ("cfg5_surfstar", "surf", {"use_star": True}),
    ("cfg4_multisurf", "multisurf", {}),
])
def test_fullsize_bitexact(F, name, algo, kw):
    """The reference's scores bit for bit at the BASELINE sizes, cfg4 (the
    north star, 20000 x 20000) and the cfg5 SURF / SURF* whole fits
    (10000 x 50000, float64 X) included."""
    fx = _fixture(name)
    X, y = _inputs(fx)
    cls = {"multisurf": F.MultiSURF, "relieff": F.ReliefF, "surf": F.SURF}[algo]
    est = cls(backend="gpu", accumulation="reference", n_features_to_select=10, **kw).fit(X, y)
    assert est.effective_backend_ == "gpu"
    assert_bitexact(est.feature_importances_, fx["scores"])


@pytest.mark.parametrize("name", ["cfg5_surfstar_slice", "cfg5_surf_slice"])
def test_cfg5_surf_slice_bitexact(F, name):
    """The cfg5 SURF / SURF* focal slices (384 samples of 10000 x 50000)
    through fs_surf_score_rows in reference order: the slice's float32
    column sum, / n, bit for bit."""
    from fastselect_amd import _lib
    from fastselect_amd.SURF import surf_inputs
    fx = _fixture(name)
    X, y = _inputs(fx)
    x = np.ascontiguousarray(X, dtype=np.float64)
    isd, recip = surf_inputs(x, 10, "gpu")
    lo, hi = (int(v) for v in fx["i_range"])
    with _lib.accumulation("reference"):
        sums = _lib.surf_score("gpu", x, np.asarray(y).astype(np.int32), recip,
                               bool(fx["use_star"]), isd, rows=(lo, hi))
    assert_bitexact((sums / x.shape[0]).astype(np.float32), fx["scores"])


@pytest.mark.parametrize("name,fast_bound", [("cfg2_multisurf", 0), ("cfg4_multisurf", 40)])
def test_decisions_row_by_row(F, name, fast_bound):
    """near / far decisions row by row against the
    oracle's (tests/golden/fullsize_<cfg>_multisurf_decisions.npz,
    oracle_multisurf_decisions on the full-size input).  Reference order
    (32-bit operands, every flagged row's threshold exact): every row
    identical.  The default path: cfg2 (32-bit operands, the flagged rows
    within the exact-threshold budget) identical too; cfg4 (16-bit operands;
    2070 rows flagged, above the budget, so their thresholds stay quantised)
    counted and bounded -- 22 measured (one near pair each), reported by
    bench.py as decisions_vs_reference."""
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    dec = np.load(os.path.join(GOLD, f"fullsize_{name}_decisions.npz"), allow_pickle=False)
    fx = _fixture(name)
    X, y = _inputs(fx)
    assert str(dec["x_sha256"]) == str(fx["x_sha256"])
    ref = dec["counts"].astype(np.int64).reshape(-1, 2)
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu")
    flipped = {}
    for mode in ("reference", "fast"):
        job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", shard=False, accumulation=mode)
        try:
            job.step()
            got = job.counts.cpu().numpy().reshape(-1, 2).astype(np.int64)
        finally:
            job.close()
        flipped[mode] = int(np.sum(np.any(got != ref, axis=1)))
    print(name, "rows decided differently from the reference:", flipped)
    assert flipped["reference"] == 0
    assert flipped["fast"] <= fast_bound


def _fullsize_rank_worker(rank, world, port, name, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    X, y = _inputs(_fixture(name))
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu", device=0)
    job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", device=0, accumulation="reference")
    np.save(f"{out_path}.{rank}.npy", job.step().cpu().numpy())
    job.close()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["cfg2_multisurf", "cfg4_multisurf"])
def test_fullsize_two_ranks_bitexact(F, tmp_path, name):
    """Reference order over two ranks at the BASELINE sizes (cfg4: the north
    star's 20000 x 20000, each rank half the pair tiles; two processes on
    cuda:0, gloo): the reference's scores bit for bit on both ranks."""
    import torch.multiprocessing as mp

    from test_gpu_dist import _port
    out = str(tmp_path / name)
    mp.spawn(_fullsize_rank_worker, args=(2, _port(), name, out), nprocs=2, join=True)
    fx = _fixture(name)
    for r in range(2):
        assert_bitexact(np.load(f"{out}.{r}.npy"), fx["scores"])


def _relieff_rank_worker(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastselect_amd import parallel
    X, y, k = make_tail_case(3)
    np.save(f"{out_path}.rf.{rank}.npy",
            parallel.relieff_scores(X, y, n_neighbors=k, backend="gpu", device=0,
                                    accumulation="reference"))
    X2, y2 = verdict_case("exp4z", 1100, 150, seed=4)
    np.save(f"{out_path}.ms.{rank}.npy",
            parallel.multisurf_scores(X2, y2, use_star=True, backend="gpu", device=0,
                                      accumulation="reference"))
    for star in (False, True):
        np.save(f"{out_path}.sf{int(star)}.{rank}.npy",
                parallel.surf_scores(X2, y2, use_star=star, backend="gpu", device=0,
                                     accumulation="reference"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_relieff_ranks_chain_the_column_sums_bitexact(F, oracle, tmp_path, world):
    """Row-sharded ReliefF in reference order over world ranks (processes
    sharing cuda:0, gloo): every rank's float32 temp rows at once
    (fs_plan_ref_temp), then the column sums passed rank to rank
    (fs_plan_ref_sums) -- the oracle's scores bit for bit on every rank; and
    parallel.multisurf_scores / surf_scores(accumulation='reference')
    likewise."""
    import torch.multiprocessing as mp

    from test_gpu_dist import _port
    out = str(tmp_path / "rf")
    mp.spawn(_relieff_rank_worker, args=(world, _port(), out), nprocs=world, join=True)
    X, y, k = make_tail_case(3)
    ref = oracle.relieff_scores(X, y, n_neighbors=k)
    X2, y2 = verdict_case("exp4z", 1100, 150, seed=4)
    ref2 = oracle.multisurf_scores(X2, y2, use_star=True)
    ref3 = [oracle.surf_scores(X2, y2, use_star=star) for star in (False, True)]
    for r in range(world):
        assert_bitexact(np.load(f"{out}.rf.{r}.npy"), ref)
        assert_bitexact(np.load(f"{out}.ms.{r}.npy"), ref2)
        for star in (0, 1):
            assert_bitexact(np.load(f"{out}.sf{star}.{r}.npy"), ref3[star])
