"""CPU-side parity: the product's native CPU backend (same pipeline as the HIP
path: integer distances, mean correction, ambiguous-pair refinement, pair
weights) against the oracle, and the sharded multi-rank path over gloo.

Bar: 1e-5 scale-relative and identical top-k.
"""
import os
import socket
import warnings

import numpy as np
import pytest
from conftest import assert_parity, scale_rel_err
from sklearn.datasets import make_classification

from fastselect_amd import SURF, MultiSURF, ReliefF, _lib

GOLD = os.path.join(os.path.dirname(__file__), "golden")
TOL = 1e-5


def test_golden_vectors_cpu_backend():
    g = np.load(os.path.join(GOLD, "oracle_vectors.npz"))
    for name in ("a", "b", "c"):
        X, y = g[f"{name}_X"], g[f"{name}_y"]
        assert_parity(MultiSURF(backend="cpu").fit(X, y).feature_importances_,
                      g[f"{name}_multisurf"], TOL, k=5)
        assert_parity(MultiSURF(backend="cpu", use_star=True).fit(X, y).feature_importances_,
                      g[f"{name}_multisurfstar"], TOL, k=5)
        assert_parity(SURF(backend="cpu").fit(X, y).feature_importances_,
                      g[f"{name}_surf"], TOL, k=5)
        assert_parity(SURF(backend="cpu", use_star=True).fit(X, y).feature_importances_,
                      g[f"{name}_surfstar"], TOL, k=5)
        for k in (1, 3, 10):
            assert_parity(ReliefF(backend="cpu", n_neighbors=k).fit(X, y).feature_importances_,
                          g[f"{name}_relieff_k{k}"], TOL, k=5)


@pytest.mark.parametrize("seed", [1, 11])
def test_surf_mean_sensitivity(oracle, seed):
    """SURF's float32 sequential row mean: 1-ulp distance errors used to flip
    near/far decisions on these inputs."""
    X, y = make_classification(n_samples=700, n_features=1500, n_informative=20,
                               n_redundant=30, random_state=seed)
    X = X + np.random.default_rng(seed).standard_normal(X.shape) * 1e-9
    assert_parity(SURF(backend="cpu").fit(X, y).feature_importances_, oracle.surf_scores(X, y),
                  TOL, k=10)


def test_multisurf_threshold_flip_case(oracle):
    """n=384, p=5000: one pair sits 7e-7 from its row threshold; quantised
    distances alone flip it (6e-4 score error).  Refinement must fix it."""
    X, y = make_classification(n_samples=384, n_features=5000, n_informative=20,
                               n_redundant=50, random_state=3)
    assert_parity(MultiSURF(backend="cpu").fit(X, y).feature_importances_,
                  oracle.multisurf_scores(X, y), TOL, k=10)


def test_relieff_small_class_self_hit(oracle):
    """A class with fewer than k other members: the reference also counts the
    focal sample itself as a (zero-diff) hit (ReliefF.py:144-168)."""
    X, y = make_classification(n_samples=120, n_features=30, weights=[0.9], random_state=1)
    for k in (10, 12, 20, 119):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", UserWarning)
            s = ReliefF(backend="cpu", n_neighbors=k).fit(X, y).feature_importances_
        assert_parity(s, oracle.relieff_scores(X, y, n_neighbors=k), TOL)


def _sharded_cpu(x, y, recip, isd, world, use_star):
    n, p = x.shape
    plans = [_lib.Plan("cpu", x, y, recip, isd, use_star=use_star, rank=r, world=world)
             for r in range(world)]
    rs = [np.zeros(3 * n) for _ in plans]
    for pl, b in zip(plans, rs):
        pl.pass1(b.ctypes.data)
    rsum = np.sum(rs, axis=0)
    cn = [np.zeros(2 * n) for _ in plans]
    for pl, b in zip(plans, cn):
        pl.select(rsum.ctypes.data, b.ctypes.data)
    csum = np.sum(cn, axis=0)
    sc = [np.zeros(p) for _ in plans]
    for pl, b in zip(plans, sc):
        pl.pass2(csum.ctypes.data, b.ctypes.data)
    return (np.sum(sc, axis=0) / n).astype(np.float32)


@pytest.mark.parametrize("world", [2, 3, 5])
def test_tile_sharding_sums_to_single(world):
    X, y = make_classification(n_samples=450, n_features=40, random_state=world)
    x = X.astype(np.float32)
    r = (x.max(0) - x.min(0)).astype(np.float32)
    recip = (1 / r).astype(np.float32)
    isd = np.zeros(40, bool)
    for star in (False, True):
        one = _lib.multisurf_score("cpu", x, y, recip, None, star, isd)
        many = _sharded_cpu(x, y, recip, isd, world, star)
        assert scale_rel_err(many, one) < 1e-6


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_worker(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastselect_amd.parallel import multisurf_scores
    X, y = make_classification(n_samples=300, n_features=50, random_state=0)
    s = multisurf_scores(X, y, use_star=True, backend="cpu")
    np.save(f"{out_path}.{rank}.npy", s)
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_matches_single(tmp_path):
    """The N>1 path end to end: two processes, gloo all-reduces of the three
    exchange vectors (the RCCL path on GPUs), equal to one process."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "scores")
    mp.spawn(_gloo_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    a, b = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    np.testing.assert_array_equal(a, b)
    X, y = make_classification(n_samples=300, n_features=50, random_state=0)
    ref = MultiSURF(backend="cpu", use_star=True).fit(X, y).feature_importances_
    assert scale_rel_err(a, ref) < 1e-6


@pytest.mark.parametrize("kind", ["discrete", "mixed", "duplicates"])
@pytest.mark.parametrize("k", [1, 3, 10])
def test_relieff_boundary_ties_follow_numba_quicksort(oracle, kind, k):
    """Neighbours tied at exactly the k-th distance: the reference takes them
    in numba-quicksort order (ReliefF.py:157); SURVEY.md §8f row 3."""
    rng = np.random.default_rng(k)
    n = 400
    if kind == "discrete":      # integer distances: ties in almost every row
        X = rng.integers(0, 3, size=(n, 12)).astype(float)
    elif kind == "mixed":       # a few coarse continuous columns + discrete
        X = np.column_stack([rng.integers(0, 3, size=(n, 8)),
                             np.round(rng.standard_normal((n, 3)), 1)])
    else:                       # exact duplicate samples
        X = rng.standard_normal((n, 20))
        X[200:260] = X[0:60]
    y = rng.integers(0, 3, n)
    dl = 3 if kind != "duplicates" else 10
    s = ReliefF(backend="cpu", n_neighbors=k, discrete_limit=dl).fit(X, y).feature_importances_
    assert_parity(s, oracle.relieff_scores(X, y, n_neighbors=k, discrete_limit=dl), TOL)


def _gather_worker(rank, world, port, out_path, dtype):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastselect_amd.parallel import gather_rows
    x = np.random.default_rng(4).normal(size=(301, 17)).astype(dtype)
    buf = gather_rows(x, None)           # host tensors: the gloo rehearsal of the RCCL gather
    np.save(f"{out_path}.{rank}.npy", buf.numpy()[:301])
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,dtype", [(2, "float32"), (3, "float32"), (2, "float64")])
def test_gather_rows_assembles_x(tmp_path, world, dtype):
    """Multi-GPU data path: each rank contributes only its row_chunk and the
    all-gather assembles all of X on every rank (gloo here, RCCL on GPUs);
    float64 rows for SURF and ReliefF's row-sharded jobs."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "x")
    mp.spawn(_gather_worker, args=(world, _free_port(), out, dtype), nprocs=world, join=True)
    x = np.random.default_rng(4).normal(size=(301, 17)).astype(dtype)
    for r in range(world):
        got = np.load(f"{out}.{r}.npy")
        assert got.dtype == np.dtype(dtype)
        np.testing.assert_array_equal(got, x)


def test_row_chunks_cover_every_row_once():
    from fastselect_amd.parallel import row_chunk
    for n in (1, 7, 128, 1000, 20000):
        for world in (1, 2, 3, 8):
            seen = np.zeros(n, int)
            for r in range(world):
                lo, hi, rows = row_chunk(n, r, world)
                assert 0 <= lo <= hi <= n and hi - lo <= rows
                seen[lo:hi] += 1
            assert (seen == 1).all()


@pytest.mark.parametrize("shards", [2, 3])
def test_tile_shards_match_one_shard_cpu(shards):
    """fs_plan_set_shard: a job scored in V tile shards (three rounds, each
    shard's distances recomputed per round; the GPU backend's mode for n
    beyond HBM) equals the one-shard job."""
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    X, y = make_classification(n_samples=700, n_features=60, n_informative=8, n_redundant=10,
                               random_state=11)
    x, yv, recip, isd = prepare_inputs(X, y, backend="cpu")
    out = []
    for v in (1, shards):
        job = ShardedMultiSURF(x, yv, recip, isd, backend="cpu", shard=False, shards=v)
        assert job.shards == v
        out.append(job.step().numpy())
        job.close()
    assert scale_rel_err(out[1], out[0]) < 1e-6
    assert set(np.argsort(out[1])[::-1][:10]) == set(np.argsort(out[0])[::-1][:10])


def _shard_worker(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    X, y = make_classification(n_samples=500, n_features=40, random_state=2)
    x, yv, recip, isd = prepare_inputs(X, y, backend="cpu")
    job = ShardedMultiSURF(x, yv, recip, isd, backend="cpu", shards=2)
    np.save(f"{out_path}.{rank}.npy", job.step().numpy())
    job.close()
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_world2_with_two_tile_shards_each(tmp_path):
    """Ranks x shards: rank r takes shards r + 2 v of 4; equal to one process."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "s")
    mp.spawn(_shard_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    a, b = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    np.testing.assert_array_equal(a, b)
    X, y = make_classification(n_samples=500, n_features=40, random_state=2)
    ref = MultiSURF(backend="cpu").fit(X, y).feature_importances_
    assert scale_rel_err(a, ref) < 1e-6


def _uneven_shard_worker(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    X, y = make_classification(n_samples=500, n_features=40, random_state=2)
    x, yv, recip, isd = prepare_inputs(X, y, backend="cpu")
    # each rank sizes its shard count from its own memory: here they disagree
    job = ShardedMultiSURF(x, yv, recip, isd, backend="cpu", shards=1 + 2 * rank)
    np.save(f"{out_path}.{rank}.npy", job.step().numpy())
    np.save(f"{out_path}.{rank}.v.npy", np.array(job.shards))
    job.close()
    dist.barrier()
    dist.destroy_process_group()


def test_gloo_ranks_agree_on_the_shard_count(tmp_path):
    """ranks that size their tile-shard count differently
    (shards=1 and 3 here; free memory on GPUs) must still deal the tiles
    by one ownership map -- the MAX over ranks -- or tiles are scored twice or
    never.  Equal to one process."""
    import torch.multiprocessing as mp
    out = str(tmp_path / "u")
    mp.spawn(_uneven_shard_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    assert int(np.load(out + ".0.v.npy")) == int(np.load(out + ".1.v.npy")) == 3
    a, b = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    np.testing.assert_array_equal(a, b)
    X, y = make_classification(n_samples=500, n_features=40, random_state=2)
    ref = MultiSURF(backend="cpu").fit(X, y).feature_importances_
    assert scale_rel_err(a, ref) < 1e-6


def test_cpu_backend_duplicated_columns(oracle):
    """Coherent column rounding (4 base columns x 1000 copies) on the CPU
    backend, whose refinement band is calibrated on sampled pairs as the
    GPU's is (fs_cpu.cpp calibrated_band)."""
    rng = np.random.default_rng(31)
    base = rng.standard_normal((800, 4)).astype(np.float32)
    X = np.repeat(base, 1000, axis=1)
    y = (base[:, 0] - base[:, 2] > 0).astype(int)
    for star in (False, True):
        s = MultiSURF(backend="cpu", use_star=star).fit(X, y).feature_importances_
        assert scale_rel_err(s, oracle.multisurf_scores(X, y, use_star=star)) < 1e-5
