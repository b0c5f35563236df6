"""GPU parity tests: the HIP path (backend='gpu', through the C ABI) against
the C oracle (oracle/relief_oracle.c) and against the committed fixtures.

Bar (north_star / SURVEY.md §8d): scores within 1e-5 scale-relative
(max_f |s_f - ref_f| <= 1e-5 * max_f |ref_f|) and identical top-k index sets.
Every test here needs a visible HIP device and fails (does not skip) without
one, so a run can never pass on a CPU fallback.
"""
import os

import numpy as np
import pytest
from conftest import assert_parity, scale_rel_err
from sklearn.datasets import make_classification

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-5


@pytest.fixture(scope="module", autouse=True)
def require_gpu():
    from fastselect_amd import _lib
    assert _lib.device_count() >= 1, "no HIP device visible: GPU tests cannot run"
    assert os.path.dirname(_lib.LIB_PATH).endswith("fastselect_amd")


def _fit(est_cls, X, y, **kw):
    est = est_cls(backend="gpu", n_features_to_select=kw.pop("n_features_to_select", 1), **kw)
    est.fit(X, y)
    assert est.effective_backend_ == "gpu"
    return est.feature_importances_


def test_golden_oracle_vectors():
    from fastselect_amd import SURF, MultiSURF, ReliefF
    g = np.load(os.path.join(GOLD, "oracle_vectors.npz"))
    for name in ("a", "b", "c"):
        X, y = g[f"{name}_X"], g[f"{name}_y"]
        assert_parity(_fit(MultiSURF, X, y), g[f"{name}_multisurf"], TOL, k=5)
        assert_parity(_fit(MultiSURF, X, y, use_star=True), g[f"{name}_multisurfstar"], TOL, k=5)
        assert_parity(_fit(SURF, X, y), g[f"{name}_surf"], TOL, k=5)
        assert_parity(_fit(SURF, X, y, use_star=True), g[f"{name}_surfstar"], TOL, k=5)
        for k in (1, 3, 10):
            assert_parity(_fit(ReliefF, X, y, n_neighbors=k), g[f"{name}_relieff_k{k}"], TOL, k=5)


def test_reference_kats_on_gpu():
    """The reference tests' known answers, on the GPU backend."""
    from fastselect_amd import SURF, MultiSURF, ReliefF
    fx = np.load(os.path.join(GOLD, "reference_fixtures.npz"))
    m = MultiSURF(n_features_to_select=1, backend="gpu", discrete_limit=4).fit(fx["ms_x"], fx["ms_y"])
    assert set(m.top_features_) == {0}
    np.testing.assert_allclose(m.feature_importances_[3], 0.0, atol=1e-7)
    r = ReliefF(n_neighbors=1, n_features_to_select=2, discrete_limit=4, backend="gpu").fit(
        fx["rs_x"], fx["rs_y"])
    s = r.feature_importances_
    assert s[0] > s[1] and s[2] > s[1] and set(r.top_features_) == {0, 2}
    np.testing.assert_allclose(s[3], 0.0)
    f = SURF(n_features_to_select=2, backend="gpu", discrete_limit=3).fit(fx["rs_x"], fx["rs_y"])
    s = f.feature_importances_
    assert s[0] > s[1] and s[2] > s[1] and set(f.top_features_) == {0, 2}
    np.testing.assert_allclose(s[3], 0.0, atol=1e-7)
    for est in (MultiSURF(backend="gpu", n_features_to_select=4),
                SURF(backend="gpu"), ReliefF(backend="gpu", n_neighbors=2)):
        x = fx["ms_x"] if isinstance(est, MultiSURF) else fx["rs_x"]
        est.fit(x, np.zeros(x.shape[0]))
        assert np.all(est.feature_importances_ <= 1e-7)


@pytest.mark.parametrize("star", [False, True])
def test_cfg1_multisurf(oracle, star):
    """BASELINE cfg1 (README dataset, n=500 p=1000) vs the oracle; the
    non-star top-15 also equals the reference's recorded top-15."""
    import json

    from fastselect_amd import MultiSURF
    X, y = make_classification(n_samples=500, n_features=1000, n_informative=20,
                               n_redundant=100, random_state=42)
    s = _fit(MultiSURF, X, y, use_star=star, n_features_to_select=15)
    ref = oracle.multisurf_scores(X, y, use_star=star)
    assert_parity(s, ref, TOL, k=15)
    if not star:
        with open(os.path.join(GOLD, "cfg1_reference.json")) as f:
            assert sorted(np.argsort(s)[::-1][:15].tolist()) == json.load(f)["top15"]


@pytest.mark.parametrize("n,p,ncls,seed", [(129, 70, 2, 0), (257, 300, 3, 1), (1000, 2000, 2, 2),
                                          (384, 5000, 2, 3), (2500, 3000, 2, 4)])
def test_multisurf_sizes(oracle, n, p, ncls, seed):
    from fastselect_amd import MultiSURF
    X, y = make_classification(n_samples=n, n_features=p, n_informative=20,
                               n_redundant=min(50, p // 4), n_classes=ncls, random_state=seed)
    for star in (False, True):
        assert_parity(_fit(MultiSURF, X, y, use_star=star), oracle.multisurf_scores(X, y, use_star=star),
                      TOL, k=10)


@pytest.mark.parametrize("n,p,nd,seed", [(1024, 64, 0, 1), (700, 600, 0, 2), (900, 800, 0, 7),
                                          (600, 1400, 30, 8), (640, 300, 300, 5), (800, 576, 0, 9),
                                          (700, 520, 20, 10)])
def test_multisurf_sparse_pass2_layouts(oracle, n, p, nd, seed):
    """Layouts of the sparse pass 2 (k_score_sparse2): a single 64-feature
    block with n a multiple of 128 (the last row's B reads run into xs's
    slack), a 256-feature tail, a tail over 256 features (one partial
    512-feature block), discrete columns in the last block, all discrete, a
    64-feature tail (one F = 4 block), continuous and discrete."""
    from fastselect_amd import MultiSURF
    X, y = make_classification(n_samples=n, n_features=p, n_informative=min(10, p // 2),
                               n_redundant=min(20, p // 4), random_state=seed)
    if nd:
        X[:, :nd] = np.round(X[:, :nd])
    assert_parity(_fit(MultiSURF, X, y), oracle.multisurf_scores(X, y), TOL, k=10)


@pytest.mark.parametrize("n,p,seed", [(300, 400, 0), (700, 1500, 1), (700, 1500, 11)])
def test_surf_sizes(oracle, n, p, seed):
    """SURF's float32 sequential mean makes it sensitive to 1-ulp distance
    differences; seeds 1 and 11 (perturbed) once exposed that."""
    from fastselect_amd import SURF
    X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=30,
                               random_state=seed)
    X = X + np.random.default_rng(seed).standard_normal(X.shape) * 1e-9
    for star in (False, True):
        assert_parity(_fit(SURF, X, y, use_star=star), oracle.surf_scores(X, y, use_star=star),
                      TOL, k=10)


@pytest.mark.parametrize("n,p,ncls,k,seed", [(500, 300, 2, 10, 0), (600, 200, 5, 3, 1),
                                            (300, 100, 3, 40, 2), (900, 150, 12, 5, 3)])
def test_relieff_sizes(oracle, n, p, ncls, k, seed):
    """12 classes: k_rf_select's 8-bit first digit (10-bit up to 8 classes)."""
    from fastselect_amd import ReliefF
    X, y = make_classification(n_samples=n, n_features=p, n_informative=10, n_redundant=10,
                               n_classes=ncls, n_clusters_per_class=1, random_state=seed)
    assert_parity(_fit(ReliefF, X, y, n_neighbors=k), oracle.relieff_scores(X, y, n_neighbors=k),
                  TOL, k=10)


@pytest.mark.parametrize("kind", ["discrete", "mixed", "duplicates"])
@pytest.mark.parametrize("k", [1, 3, 10])
def test_relieff_boundary_ties_follow_numba_quicksort(oracle, kind, k):
    """Neighbours tied at exactly the k-th distance are taken in numba's
    quicksort order (k_rf_ties replays it on the device)."""
    from fastselect_amd import ReliefF
    rng = np.random.default_rng(k)
    n = 400
    if kind == "discrete":
        X = rng.integers(0, 3, size=(n, 12)).astype(float)
    elif kind == "mixed":
        X = np.column_stack([rng.integers(0, 3, size=(n, 8)),
                             np.round(rng.standard_normal((n, 3)), 1)])
    else:
        X = rng.standard_normal((n, 20))
        X[200:260] = X[0:60]
    y = rng.integers(0, 3, n)
    dl = 3 if kind != "duplicates" else 10
    s = _fit(ReliefF, X, y, n_neighbors=k, discrete_limit=dl)
    assert_parity(s, oracle.relieff_scores(X, y, n_neighbors=k, discrete_limit=dl), TOL)


def test_relieff_small_and_big_buckets_in_one_row(oracle):
    """k_rf_select: one class's k-th key settled by the small-bucket gather
    while another class, whose members all sit at one distance (> 64 keys in
    the bucket), still needs radix passes; the settled class must keep its
    key (a further pass once re-bucketed it: TuRF over ReliefF then varied
    from run to run)."""
    from fastselect_amd import ReliefF
    rng = np.random.default_rng(12)
    n, p = 600, 40
    X = rng.standard_normal((n, p))
    y = np.zeros(n, dtype=int)
    y[200:400] = 1
    y[400:] = 2
    X[200:400] = X[200]                     # class 1: 200 identical rows
    X[400:] = np.round(X[400:], 1)          # class 2: coarse grid (ties)
    for k in (3, 10):
        s = _fit(ReliefF, X, y, n_neighbors=k)
        assert_parity(s, oracle.relieff_scores(X, y, n_neighbors=k), TOL)
        np.testing.assert_array_equal(_fit(ReliefF, X, y, n_neighbors=k), s)


def test_relieff_unstaged_rows(oracle):
    """n past what k_rf_select stages in LDS (5 bytes per sample + the
    histograms > 160 KB: n > ~31000): the row is read from HBM on every
    sweep (k_rf_select<false>, 256 threads per row)."""
    from fastselect_amd import ReliefF
    X, y = make_classification(n_samples=33000, n_features=24, n_informative=8, n_redundant=4,
                               random_state=13)
    s = _fit(ReliefF, X, y, n_neighbors=5)
    assert_parity(s, oracle.relieff_scores(X, y, n_neighbors=5), TOL, k=5)


@pytest.mark.parametrize("n", [2500, 33000])
def test_relieff_exact_keys_lds_and_global(n, hooks):
    """k_rf_select's in-kernel exact keys: candidate rows gathered into LDS
    in batches (default; one row per batch with the rf_xlds hook at 4*pc) or summed
    straight from HBM (rf_xlds = 0), and the
    exact k-th key comes from the row's candidate list (default) or from a
    second selection over the whole row (rf_fcap = 0, the route of rows with
    over 256 candidates): the keys are the same float32 numbers and the
    selections agree, so the scores are bit-identical.  Mixed data (a
    discrete block), 1100 continuous columns (not a multiple of the unrolled
    column step); n=33000 takes the unstaged kernel."""
    from fastselect_amd import ReliefF
    rng = np.random.default_rng(5)
    p = 1200 if n < 10000 else 80
    X, y = make_classification(n_samples=n, n_features=p, n_informative=12, n_redundant=20,
                               n_classes=3, random_state=17)
    X[:, -100 if n < 10000 else -10:] = rng.integers(0, 4, size=(n, 100 if n < 10000 else 10))
    out = {}
    pc = 1100 if n < 10000 else 70
    from fastselect_amd import _lib
    for mode, hk in (("default", {}), ("hbm", {"rf_xlds": 0}),
                     ("batch1", {"rf_xlds": 4 * pc}),
                     ("general", {"rf_fcap": 0})):
        with _lib.test_hooks(**hk):
            out[mode] = _fit(ReliefF, X, y, n_neighbors=7)
    for mode in ("hbm", "batch1", "general"):
        assert np.array_equal(out["default"], out[mode]), mode


def test_relieff_ties_large_rows(oracle):
    """Tie replay on rows long enough for many 64-wide partition rounds and
    deep recursion (all-discrete data: ties in every row), CPU == GPU == oracle."""
    from fastselect_amd import ReliefF
    rng = np.random.default_rng(5)
    X = rng.integers(0, 4, size=(3000, 15)).astype(float)
    y = rng.integers(0, 2, 3000)
    s = _fit(ReliefF, X, y, n_neighbors=10, discrete_limit=4)
    assert_parity(s, oracle.relieff_scores(X, y, n_neighbors=10, discrete_limit=4), TOL)


def test_relieff_ties_multiwave_matches_single_wave(hooks):
    """k_rf_ties_mw (whole-workgroup partitions of the ranges of >= 2048
    samples, then 16 waves taking the smaller ranges from a shared queue)
    against the one-wave replay (ties_1w test hook) and against workgroup
    partitions down to 16 samples (ties_coop=16): every row of
    all-discrete data is a tie row; the orders, so the scores, must be
    bit-identical.  Mixed data (exact keys from k_rf_exact_rows) too."""
    from fastselect_amd import ReliefF
    rng = np.random.default_rng(12)
    X = rng.integers(0, 3, size=(4000, 40)).astype(float)
    X2 = X.copy()
    X2[:, :3] = np.round(rng.standard_normal((4000, 3)), 1)
    y = rng.integers(0, 3, 4000)
    for data in (X, X2):
        out = []
        from fastselect_amd import _lib
        for hk in ({}, {"ties_1w": 1}, {"ties_coop": 16}):
            with _lib.test_hooks(**hk):
                out.append(_fit(ReliefF, data, y, n_neighbors=10))
        assert np.array_equal(out[0], out[1])
        assert np.array_equal(out[0], out[2])


def test_relieff_collection_overflow(oracle):
    """Rows where most keys tie at the k-th key (90% of the samples are one
    point): the per-wave hit lists of k_rf_select's collection overflow and
    its pass 2 sweeps the row again; numba's quicksort order then decides
    (k_rf_ties).  GPU == oracle."""
    from fastselect_amd import ReliefF
    rng = np.random.default_rng(9)
    X = rng.standard_normal((2400, 5))
    X[rng.random(2400) < 0.9] = X[0]
    y = rng.integers(0, 2, 2400)
    s = _fit(ReliefF, X, y, n_neighbors=10)
    assert_parity(s, oracle.relieff_scores(X, y, n_neighbors=10), TOL)


def test_relieff_large_n_boundary(oracle):
    """n large enough that k-th-neighbour keys crowd within float32 ulps:
    the exact-key band must make every selection the reference's."""
    from fastselect_amd import ReliefF
    X, y = make_classification(n_samples=4000, n_features=400, n_informative=20,
                               n_redundant=50, n_classes=3, n_clusters_per_class=1,
                               random_state=42)
    s = _fit(ReliefF, X, y, n_neighbors=10)
    assert_parity(s, oracle.relieff_scores(X, y, n_neighbors=10), TOL, k=10)


def test_gpu_matches_cpu_backend():
    """Same integer distances and weights on both product backends: scores
    differ only by floating-point accumulation order."""
    from fastselect_amd import SURF, MultiSURF, ReliefF
    X, y = make_classification(n_samples=400, n_features=600, n_informative=15, random_state=9)
    X[:, 3] = np.round(X[:, 3])
    for cls, kw in ((MultiSURF, {}), (MultiSURF, {"use_star": True}), (SURF, {}),
                    (SURF, {"use_star": True}), (ReliefF, {"n_neighbors": 7})):
        g = cls(backend="gpu", **kw).fit(X, y).feature_importances_
        c = cls(backend="cpu", **kw).fit(X, y).feature_importances_
        assert scale_rel_err(g, c) < 1e-6, (cls.__name__, kw)


def test_determinism():
    from fastselect_amd import MultiSURF
    X, y = make_classification(n_samples=700, n_features=900, random_state=4)
    a = MultiSURF(backend="gpu", use_star=True).fit(X, y).feature_importances_
    b = MultiSURF(backend="gpu", use_star=True).fit(X, y).feature_importances_
    np.testing.assert_array_equal(a, b)


def test_edge_cases(oracle):
    from fastselect_amd import SURF, MultiSURF, ReliefF
    rng = np.random.default_rng(11)
    # n = 2, one feature
    X = np.array([[0.0], [1.0]])
    y = np.array([0, 1])
    assert_parity(_fit(MultiSURF, X, y), oracle.multisurf_scores(X, y), TOL)
    assert_parity(_fit(SURF, X, y), oracle.surf_scores(X, y), TOL)
    # all-discrete data with duplicate rows (exact distance ties)
    X = rng.integers(0, 3, size=(150, 12)).astype(float)
    X[50:60] = X[0]
    y = rng.integers(0, 2, 150)
    assert_parity(_fit(MultiSURF, X, y), oracle.multisurf_scores(X, y), TOL)
    assert_parity(_fit(SURF, X, y, use_star=True), oracle.surf_scores(X, y, use_star=True), TOL)
    # mixed: many-level discrete, constant, continuous; discrete_limit large
    X = np.column_stack([rng.integers(0, 9, 200), np.full(200, 7.0), rng.standard_normal((200, 5))])
    y = rng.integers(0, 3, 200)
    assert_parity(_fit(MultiSURF, X, y, discrete_limit=9), oracle.multisurf_scores(X, y, discrete_limit=9), TOL)
    # k larger than a class
    X, y = make_classification(n_samples=120, n_features=30, weights=[0.9], random_state=1)
    with pytest.warns(UserWarning):
        s = _fit(ReliefF, X, y, n_neighbors=20)
    assert_parity(s, oracle.relieff_scores(X, y, n_neighbors=20), TOL)


@pytest.mark.parametrize("n,pc,pd", [(400, 150, 70), (333, 64, 200), (260, 300, 10)])
def test_mixed_feature_blocks(oracle, n, pc, pd):
    """Continuous and discrete columns in every pass-2 block layout: a
    128-feature block wholly continuous, wholly discrete, half-and-half, and
    a trailing single 64-feature half (continuous-first permutation padded to
    64 per kind)."""
    from fastselect_amd import SURF, MultiSURF, ReliefF
    rng = np.random.default_rng(n + pc)
    Xc, y = make_classification(n_samples=n, n_features=pc, n_informative=min(10, pc),
                                n_redundant=0, random_state=pc)
    Xd = rng.integers(0, 4, size=(n, pd)).astype(float)
    Xd[:, 0] = (y + rng.integers(0, 2, n)) % 3   # an informative discrete column
    X = np.empty((n, pc + pd))
    perm = rng.permutation(pc + pd)               # interleave the two kinds
    X[:, perm[:pc]] = Xc
    X[:, perm[pc:]] = Xd
    for star in (False, True):
        assert_parity(_fit(MultiSURF, X, y, use_star=star),
                      oracle.multisurf_scores(X, y, use_star=star), TOL, k=10)
        assert_parity(_fit(SURF, X, y, use_star=star), oracle.surf_scores(X, y, use_star=star),
                      TOL, k=10)
    assert_parity(_fit(ReliefF, X, y, n_neighbors=5), oracle.relieff_scores(X, y, n_neighbors=5),
                  TOL, k=10)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_column_stats_gpu_matches_numpy(dtype):
    """GPU column statistics (fs_column_stats) == numpy min / max / np.unique
    counts, for caps on both sides of every column's level count, shapes
    that are not multiples of the kernels' blocks, and the LDS hash set at
    its largest supported cap."""
    from test_abi import _np_stats, column_stats_cases

    from fastselect_amd import _lib
    x = column_stats_cases().astype(dtype)
    big = np.random.default_rng(1).integers(0, 5000, size=(9000, 3)).astype(dtype)
    for data in (x, big, x[:1], x[:, :1]):
        for cap in (0, 2, 10, 11, 50, 8191):
            mn, mx, nd = _lib.column_stats("gpu", data, cap)
            emn, emx, end = _np_stats(data, cap)
            np.testing.assert_array_equal(mn, emn)
            np.testing.assert_array_equal(mx, emx)
            np.testing.assert_array_equal(nd, end)
    with pytest.raises(RuntimeError):
        _lib.column_stats("gpu", x, 8192)


def test_feat_idx_subset(oracle):
    from fastselect_amd import _lib
    X, y = make_classification(n_samples=260, n_features=90, random_state=3)
    x = X.astype(np.float32)
    r = (x.max(0) - x.min(0)).astype(np.float32)
    recip = (1 / r).astype(np.float32)
    fidx = np.array([5, 80, 3, 44, 44, 0], dtype=np.int64)
    g = _lib.multisurf_score("gpu", x, y, recip, fidx, False, np.zeros(90, bool))
    ref = oracle.multisurf_scores(X, y, feat_idx=fidx)
    assert_parity(g, ref, TOL)


def test_sharded_plans_sum_to_single():
    """Tile sharding on one GPU: world=3 plans' exchanged partials, summed,
    reproduce the world=1 result (the RCCL all-reduce is a sum)."""
    import torch

    from fastselect_amd import _lib
    X, y = make_classification(n_samples=700, n_features=300, random_state=8)
    x = X.astype(np.float32)
    r = (x.max(0) - x.min(0)).astype(np.float32)
    recip = (1 / r).astype(np.float32)
    isd = np.zeros(300, bool)
    n, p = x.shape

    def run(world):
        plans = [_lib.Plan("gpu", x, y, recip, isd, use_star=True, rank=rk, world=world)
                 for rk in range(world)]
        rs = [torch.zeros(3 * n, dtype=torch.float64, device="cuda") for _ in plans]
        for pl, b in zip(plans, rs):
            pl.pass1(b.data_ptr())
        rsum = sum(rs)
        cn = [torch.zeros(2 * n, dtype=torch.float64, device="cuda") for _ in plans]
        for pl, b in zip(plans, cn):
            pl.select(rsum.data_ptr(), b.data_ptr())
        csum = sum(cn)
        sc = [torch.zeros(p, dtype=torch.float64, device="cuda") for _ in plans]
        for pl, b in zip(plans, sc):
            pl.pass2(csum.data_ptr(), b.data_ptr())
        torch.cuda.synchronize()
        return (sum(sc) / n).float().cpu().numpy()

    one = run(1)
    three = run(3)
    assert scale_rel_err(three, one) < 1e-6
    ref = _lib.multisurf_score("gpu", x, y, recip, None, True, isd)
    assert scale_rel_err(one, ref) < 1e-6


def test_large_p_flush_path(oracle):
    """p >> 256 exercises the packed high-word carry of the pass-1 integer
    accumulators; distances must stay exact (GPU == CPU backend)."""
    from fastselect_amd import MultiSURF
    X, y = make_classification(n_samples=256, n_features=20000, n_informative=20,
                               n_redundant=50, random_state=6)
    g = MultiSURF(backend="gpu").fit(X, y).feature_importances_
    c = MultiSURF(backend="cpu").fit(X, y).feature_importances_
    assert scale_rel_err(g, c) < 1e-6
    assert_parity(g, oracle.multisurf_scores(X, y), TOL, k=10)


@pytest.mark.parametrize("name", ["MultiSURF", "ReliefF", "SURF"])
def test_sklearn_api_compliance_gpu(name):
    """The 47 scikit-learn estimator checks with every fit on the GPU."""
    from sklearn.utils.estimator_checks import check_estimator

    import fastselect_amd
    check_estimator(getattr(fastselect_amd, name)(backend="gpu"))


def test_plan_set_features_matches_fresh_scoring(oracle):
    """A resident plan re-targeted to feature subsets (fs_plan_set_features)
    scores each subset as a fresh call with that feat_idx, and as the oracle."""
    import torch

    from fastselect_amd import _lib
    X, y = make_classification(n_samples=500, n_features=300, random_state=12)
    X[:, 7] = np.round(X[:, 7])
    x = X.astype(np.float32)
    r = (x.max(0) - x.min(0)).astype(np.float32)
    recip = (1 / r).astype(np.float32)
    isd = oracle.is_discrete_mask(x, 10)
    assert isd[7] and isd.sum() == 1
    n = x.shape[0]
    plan = _lib.Plan("gpu", x, y, recip, isd, use_star=True)
    rng = np.random.default_rng(0)
    for size in (300, 250, 130, 64, 3):
        fidx = np.sort(rng.choice(300, size, replace=False)) if size < 300 else None
        plan.set_features(fidx)
        rs = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
        cn = torch.zeros(2 * n, dtype=torch.float64, device="cuda")
        sc = torch.zeros(plan.n_kept, dtype=torch.float64, device="cuda")
        plan.pass1(rs.data_ptr())
        plan.select(rs.data_ptr(), cn.data_ptr())
        plan.pass2(cn.data_ptr(), sc.data_ptr())
        got = (sc / n).float().cpu().numpy()
        fresh = _lib.multisurf_score("gpu", x, y, recip, fidx, True, isd)
        assert scale_rel_err(got, fresh) < 1e-6
        ref = oracle.multisurf_scores(X, y, use_star=True, feat_idx=fidx, discrete_limit=10)
        assert_parity(got, ref, TOL)
    plan.close()


def test_turf_resident_gpu_equals_refits():
    from fastselect_amd import TuRF, MultiSURF

    class Refit(MultiSURF):
        _resident_scorer = None

    X, y = make_classification(n_samples=400, n_features=200, n_informative=10, random_state=2)
    kw = dict(n_features_to_select=10, pct_remove=0.25)
    fast = TuRF(MultiSURF(backend="gpu"), **kw).fit(X, y)
    slow = TuRF(Refit(backend="gpu"), **kw).fit(X, y)
    np.testing.assert_array_equal(fast.top_features_, slow.top_features_)
    np.testing.assert_allclose(fast.feature_importances_, slow.feature_importances_, atol=1e-7)


@pytest.mark.parametrize("name", ["ReliefF", "SURF", "SURFstar"])
def test_turf_resident_rows_gpu_equals_refits(name):
    """TuRF over resident ReliefF / SURF plans (fs_plan_set_features +
    fs_plan_score on the device) equals refitting on X[:, active]."""
    import fastselect_amd as fa
    cls = {"ReliefF": fa.ReliefF, "SURF": fa.SURF, "SURFstar": fa.SURFstar}[name]
    kw_est = {"n_neighbors": 6} if name == "ReliefF" else {}

    class Refit(cls):
        _resident_scorer = None

    X, y = make_classification(n_samples=700, n_features=300, n_informative=10, n_classes=3,
                               random_state=8)
    X[:, 4] = np.round(X[:, 4])
    kw = dict(n_features_to_select=10, pct_remove=0.3)
    fast = fa.TuRF(cls(backend="gpu", **kw_est), **kw).fit(X, y)
    slow = fa.TuRF(Refit(backend="gpu", **kw_est), **kw).fit(X, y)
    np.testing.assert_array_equal(fast.top_features_, slow.top_features_)
    np.testing.assert_allclose(fast.feature_importances_, slow.feature_importances_, atol=1e-7)


def _two_rank_worker(rank, world, port, out_path, star=False):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastselect_amd.parallel import multisurf_scores
    X, y = make_classification(n_samples=900, n_features=400, random_state=7)
    s = multisurf_scores(X, y, use_star=star, backend="gpu", device=0)
    np.save(f"{out_path}.{rank}.npy", s)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("star", [False, True])
def test_two_ranks_share_one_gpu(tmp_path, star):
    """The multi-process path with GPU plans: two ranks (both on cuda:0,
    gloo collectives on device tensors) each compute half the pair tiles;
    every rank ends with the single-process scores.  MultiSURF*: each rank
    also adds the star split's column terms of its half of the columns."""
    import socket

    import torch.multiprocessing as mp

    from fastselect_amd import MultiSURF
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = str(tmp_path / "scores")
    mp.spawn(_two_rank_worker, args=(2, port, out, star), nprocs=2, join=True)
    a, b = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    np.testing.assert_array_equal(a, b)
    X, y = make_classification(n_samples=900, n_features=400, random_state=7)
    ref = MultiSURF(backend="gpu", use_star=star).fit(X, y).feature_importances_
    assert scale_rel_err(a, ref) < 1e-6


@pytest.mark.parametrize("algo,star", [("multisurf", False), ("multisurf", True), ("surf", False),
                                       ("surf", True)])
def test_sparse_pass2_matches_dense(algo, star, hooks):
    """k_weights_sparse + k_score_sparse (non-zero pair weights only) against
    the dense k_weights + k_score on the same data (the sparse test hook forces either),
    with mixed continuous/discrete blocks so both the asm loop and the generic
    loop run; and both against the oracle."""
    from fastselect_amd import SURF, MultiSURF
    from oracle import oracle as O
    rng = np.random.default_rng(7)
    X, y = make_classification(n_samples=700, n_features=600, n_informative=15,
                               n_redundant=30, random_state=3)
    X[:, 500:] = rng.integers(0, 3, size=(700, 100))  # discrete tail: a mixed 256-block
    est = MultiSURF if algo == "multisurf" else SURF
    out = {}
    for mode in ("0", "1"):
        hooks("sparse", int(mode))
        out[mode] = _fit(est, X, y, use_star=star)
    ref = (O.multisurf_scores if algo == "multisurf" else O.surf_scores)(X, y, use_star=star)
    assert scale_rel_err(out["1"], out["0"]) <= 1e-6
    assert_parity(out["1"], ref, TOL, k=10)


def test_exact_pairs_row_reads_match_gather(hooks):
    """k_exact_pairs_rows (float4 reads of whole rows, all-continuous
    float32 data in input order) against the column-indexed gather
    (the exact_gather test hook forces it): the 16-bit pass 1 (q16 hook) refines
    hundreds of pairs here; 1500 features is not a multiple of 256.
    Both refine the same pairs, so the scores agree to f64 summation order."""
    from fastselect_amd.parallel import ShardedMultiSURF
    X, y = make_classification(n_samples=1200, n_features=1500, n_informative=20,
                               n_redundant=40, random_state=11)
    x = X.astype(np.float32)
    recip = (1 / (x.max(0) - x.min(0))).astype(np.float32)
    hooks("q16", 1)
    out = {}
    for mode in ("rows", "gather"):
        if mode == "gather":
            hooks("exact_gather", 1)
        job = ShardedMultiSURF(x, y, recip, np.zeros(x.shape[1], bool), backend="gpu", device=0)
        out[mode] = job.step().cpu().numpy()
        refined = job.info()[2]
        job.close()
        assert refined > 200
    assert scale_rel_err(out["rows"], out["gather"]) <= 1e-7


def test_device_cache_reuse_gives_same_scores(oracle):
    """Plans take their device buffers from the block cache, with the stale
    contents of the previous fit: a fit on other data in between must not
    change a result, and both must match the oracle."""
    from fastselect_amd import MultiSURF, _lib
    X1, y1 = make_classification(n_samples=700, n_features=900, random_state=21)
    X2, y2 = make_classification(n_samples=700, n_features=900, random_state=22)
    _lib.release_device_cache()
    a = MultiSURF(backend="gpu").fit(X1, y1).feature_importances_
    b = MultiSURF(backend="gpu").fit(X2, y2).feature_importances_
    c = MultiSURF(backend="gpu").fit(X1, y1).feature_importances_
    np.testing.assert_array_equal(a, c)
    assert_parity(a, oracle.multisurf_scores(X1, y1), TOL, k=10)
    assert_parity(b, oracle.multisurf_scores(X2, y2), TOL, k=10)
    _lib.release_device_cache()


def test_staged_x_matches_uploads():
    """fs_stage_x: column statistics and scoring calls on the same host
    array read the staged device copy; results are bit-identical to the
    uploading path (MultiSURF float32 and SURF float64)."""
    from fastselect_amd import _lib
    X, y = make_classification(n_samples=500, n_features=700, random_state=31)
    x32 = np.ascontiguousarray(X, dtype=np.float32)
    recip = (1 / (x32.max(0) - x32.min(0))).astype(np.float32)
    isd = np.zeros(700, bool)
    fidx = np.arange(700, dtype=np.int64)
    plain_cs = _lib.column_stats("gpu", x32, 10)
    plain_ms = _lib.multisurf_score("gpu", x32, y, recip, fidx, False, isd)
    plain_sf = _lib.surf_score("gpu", X, y, recip, True, isd)
    with _lib.staged_x("gpu", x32):
        st_cs = _lib.column_stats("gpu", x32, 10)
        st_ms = _lib.multisurf_score("gpu", x32, y, recip, fidx, False, isd)
    with _lib.staged_x("gpu", X):
        st_sf = _lib.surf_score("gpu", X, y, recip, True, isd)
    for a, b in zip(plain_cs, st_cs):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal(plain_ms, st_ms)
    np.testing.assert_array_equal(plain_sf, st_sf)


def test_plan_outlives_its_staged_x():
    """A plan reads the library's staged copy in place and holds a
    reference to it: fs_unstage_x while the plan lives defers the free to
    the plan's end, so later steps still score the same X (bit-identical to
    a plan that uploaded X itself).  A copy cast by fs_stage_x_cast carries
    its column extrema: the column statistics give x32.min(0) / x32.max(0)
    exactly."""
    from fastselect_amd import _lib
    from fastselect_amd.parallel import ShardedMultiSURF
    X, y = make_classification(n_samples=700, n_features=600, random_state=32)
    x32 = np.ascontiguousarray(X, dtype=np.float32)
    recip = (1 / (x32.max(0) - x32.min(0))).astype(np.float32)
    isd = np.zeros(600, bool)
    plain = ShardedMultiSURF(x32, y, recip, isd, backend="gpu", shard=False)
    try:
        ref = plain.step().cpu().numpy()
    finally:
        plain.close()
    with _lib.staged_x("gpu", x32):
        job = ShardedMultiSURF(x32, y, recip, isd, backend="gpu", shard=False)
    try:
        # the staged block has ended: the plan's reference keeps the copy
        np.testing.assert_array_equal(job.step().cpu().numpy(), ref)
        np.testing.assert_array_equal(job.step().cpu().numpy(), ref)
    finally:
        job.close()
    xc, finite, h = _lib.stage_x_cast(X, -1, 0)
    assert finite and h
    with _lib.unstaged(h):
        mn, mx, _ = _lib.column_stats("gpu", xc, 10)
    np.testing.assert_array_equal(mn, x32.min(0))
    np.testing.assert_array_equal(mx, x32.max(0))


def test_concurrent_fits_on_one_array():
    """Fits of the same host array in several threads each stage and free
    their own device copy (staged X is per thread): results equal the
    sequential fits."""
    import threading
    from fastselect_amd import MultiSURF, SURF
    X, y = make_classification(n_samples=600, n_features=800, random_state=41)
    X = np.ascontiguousarray(X)
    ref_m = MultiSURF(backend="gpu").fit(X, y).feature_importances_
    ref_s = SURF(backend="gpu").fit(X, y).feature_importances_
    out, errs = {}, []

    def work(k):
        try:
            est = MultiSURF(backend="gpu") if k % 2 == 0 else SURF(backend="gpu")
            out[k] = est.fit(X, y).feature_importances_
        except Exception as e:  # noqa: BLE001
            errs.append(e)
    th = [threading.Thread(target=work, args=(k,)) for k in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errs
    for k, v in out.items():
        np.testing.assert_array_equal(v, ref_m if k % 2 == 0 else ref_s)


def test_sparse_weighted_pairs_count():
    """fs_plan_weighted_pairs: MultiSURF weighs the pairs near one of their two
    samples (~40% here); the count is exact against a numpy restatement."""
    from fastselect_amd.parallel import ShardedMultiSURF
    X, y = make_classification(n_samples=600, n_features=300, n_informative=10,
                               n_redundant=20, random_state=5)
    X = X.astype(np.float32)
    recip = (1 / (X.max(0) - X.min(0))).astype(np.float32)
    job = ShardedMultiSURF(X, y, recip, np.zeros(300, bool), use_star=False, backend="gpu",
                           device=0)
    job.step()
    nz = job.weighted_pairs()
    job.close()
    Xs = (X - X.min(0)) * recip
    D = np.abs(Xs[:, None, :].astype(np.float64) - Xs[None, :, :]).sum(-1)
    n = len(X)
    off = ~np.eye(n, dtype=bool)
    mu = D.sum(1) / (n - 1)
    sd = np.sqrt(np.maximum((D ** 2).sum(1) / (n - 1) - mu ** 2, 0))
    near = (D < (mu - sd / 2)[:, None]) & off
    want = int(np.triu(near | near.T, 1).sum())
    assert 0.2 * n * (n - 1) / 2 < nz < 0.7 * n * (n - 1) / 2
    assert abs(nz - want) <= max(3, want // 2000)
