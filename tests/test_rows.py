"""Row-sharded ReliefF / SURF (SURVEY.md §8e "same row sharding"):
``fs_relieff_score_rows`` / ``fs_surf_score_rows`` score a slice of the focal
samples; the slices of a partition of [0, n) sum to the one-shot result, and
``fastselect_amd.parallel.{relieff,surf}_scores`` combine them with one
all-reduce (gloo here, RCCL on GPUs).

Checked against the one-shot call (same engine: float64 summation order
only) and against the oracle (1e-5 scale-relative), per slice against the
oracle's own focal-range scores (``i_range``), on CPU and on the GPU.
"""
import os
import socket

import numpy as np
import pytest
from conftest import assert_parity, scale_rel_err
from sklearn.datasets import make_classification

from fastselect_amd import SURF, ReliefF, _lib
from fastselect_amd.parallel import shard_rows
from fastselect_amd.ReliefF import relieff_inputs
from fastselect_amd.SURF import surf_inputs

TOL = 1e-5


def _data(n=300, p=40, classes=3, seed=0):
    X, y = make_classification(n_samples=n, n_features=p, n_informative=8, n_redundant=4,
                               n_classes=classes, random_state=seed)
    X[:, 3] = np.round(X[:, 3])          # a discrete column
    X[:, 5] = 1.5                        # a constant column
    return X, y


def _partitions(n):
    return [[(0, n)], [(0, 128), (128, n)], [(0, 7), (7, 200), (200, n)],
            [shard_rows(n, r, 3) for r in range(3)], [(0, 0), (0, n), (n, n)]]


def _relieff_sums(backend, X, y, k, rows):
    x32, ye, recip, isd, pr = relieff_inputs(X, y, 10, "cpu")
    return _lib.relieff_score(backend, x32, ye, recip, isd, k, pr, rows=rows)


def _surf_sums(backend, X, y, star, rows):
    isd, recip = surf_inputs(X, 10, "cpu")
    return _lib.surf_score(backend, X, y.astype(np.int32), recip, star, isd, rows=rows)


def _check_partitions(backend, oracle):
    X, y = _data()
    n = X.shape[0]
    for k in (1, 5):
        one = ReliefF(backend=backend, n_neighbors=k).fit(X, y).feature_importances_
        ref = oracle.relieff_scores(X, y, n_neighbors=k)
        for part in _partitions(n):
            s = sum(_relieff_sums(backend, X, y, k, r) for r in part) / n
            assert scale_rel_err(s, one) < 2e-7
            assert_parity(s, ref, TOL, k=5)
        # one slice against the oracle's focal range
        lo, hi = 37, 211
        sl = _relieff_sums(backend, X, y, k, (lo, hi)) / n
        o = oracle.relieff_scores(X, y, n_neighbors=k, i_range=(lo, hi))
        assert np.abs(sl - o).max() <= TOL * np.abs(ref).max()
    for star in (False, True):
        one = SURF(backend=backend, use_star=star).fit(X, y).feature_importances_
        ref = oracle.surf_scores(X, y, use_star=star)
        for part in _partitions(n):
            s = sum(_surf_sums(backend, X, y, star, r) for r in part) / n
            assert scale_rel_err(s, one) < 2e-7
            assert_parity(s, ref, TOL, k=5)


def test_rows_partition_cpu(oracle):
    _check_partitions("cpu", oracle)


def test_rows_invalid_range():
    X, y = _data(n=50, p=20)
    for rows in [(-1, 10), (10, 5), (0, 51)]:
        with pytest.raises(ValueError):
            _relieff_sums("cpu", X, y, 3, rows)
        with pytest.raises(ValueError):
            _surf_sums("cpu", X, y, False, rows)


def test_shard_rows_cover_blocks():
    for n in (2, 127, 128, 129, 1000, 20000):
        for world in (1, 2, 3, 8):
            rs = [shard_rows(n, r, world) for r in range(world)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            for (a, b), (c, d) in zip(rs, rs[1:]):
                assert b == c and a <= b
            for a, _ in rs:
                assert a % 128 == 0 or a == n


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rows_worker(rank, world, port, out_path, backend):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastselect_amd.parallel import relieff_scores, surf_scores
    X, y = _data()
    r = relieff_scores(X, y, n_neighbors=4, backend=backend)
    s = surf_scores(X, y, use_star=True, backend=backend)
    np.save(f"{out_path}.{rank}.npy", np.stack([r, s]))
    dist.barrier()
    dist.destroy_process_group()


def _check_world2(tmp_path, backend):
    import torch.multiprocessing as mp
    out = str(tmp_path / "rows")
    mp.spawn(_rows_worker, args=(2, _free_port(), out, backend), nprocs=2, join=True)
    a, b = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    np.testing.assert_array_equal(a, b)
    X, y = _data()
    r = ReliefF(backend=backend, n_neighbors=4).fit(X, y).feature_importances_
    s = SURF(backend=backend, use_star=True).fit(X, y).feature_importances_
    assert scale_rel_err(a[0], r) < 1e-6
    assert scale_rel_err(a[1], s) < 1e-6


def test_gloo_world2_rows_cpu(tmp_path):
    _check_world2(tmp_path, "cpu")


@pytest.mark.gpu
def test_rows_partition_gpu(oracle):
    _check_partitions("gpu", oracle)


@pytest.mark.gpu
def test_two_ranks_rows_one_gpu(tmp_path):
    _check_world2(tmp_path, "gpu")


@pytest.mark.gpu
def test_rows_partition_gpu_large():
    """cfg3-shaped ReliefF (k=10) and a SURF* case at a few thousand samples:
    the 8-way block partition sums to the one-shot scores."""
    X, y = make_classification(n_samples=3000, n_features=600, n_informative=20,
                               n_redundant=30, random_state=42)
    n = X.shape[0]
    one = ReliefF(backend="gpu", n_neighbors=10).fit(X, y).feature_importances_
    s = sum(_relieff_sums("gpu", X, y, 10, shard_rows(n, r, 8)) for r in range(8)) / n
    assert scale_rel_err(s, one) < 2e-7
    assert set(np.argsort(s)[::-1][:10]) == set(np.argsort(one)[::-1][:10])
    one = SURF(backend="gpu", use_star=True).fit(X, y).feature_importances_
    s = sum(_surf_sums("gpu", X, y, True, shard_rows(n, r, 8)) for r in range(8)) / n
    assert scale_rel_err(s, one) < 2e-7
