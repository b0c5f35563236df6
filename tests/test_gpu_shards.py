"""Tile shards on one GPU (fs_plan_set_shard): the mode for n beyond HBM.

A MultiSURF job whose distance tiles do not fit the device runs in V shards,
the device holding one shard's tiles at a time and recomputing them in each
of the three rounds (MultiSURF.py:174-214 streams distance rows the same
way).  Forced here at sizes the oracle checks (the shards test hook / shards=V) and
compared with the one-shard job and the oracle; the automatic choice
(fs_multisurf_shards) is checked at sizes that do and do not fit 288 GB.
"""
import numpy as np
import pytest
from sklearn.datasets import make_classification

from conftest import assert_parity, scale_rel_err

pytestmark = pytest.mark.gpu
TOL = 1e-5


def _inputs(n=1500, p=400, seed=21):
    from fastselect_amd.parallel import prepare_inputs
    X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=30,
                               random_state=seed)
    return X, y, prepare_inputs(X, y, backend="gpu")


@pytest.mark.parametrize("shards", [2, 5])
def test_one_shot_in_shards_matches_oracle(oracle, shards, hooks):
    from fastselect_amd import _lib
    X, y, (x, yv, recip, isd) = _inputs()
    one = _lib.multisurf_score("gpu", x, yv, recip, None, False, isd)
    hooks("shards", shards)
    many = _lib.multisurf_score("gpu", x, yv, recip, None, False, isd)
    assert scale_rel_err(many, one) < 1e-6
    assert_parity(many, oracle.multisurf_scores(X, y), TOL, k=10)


def test_sharded_job_in_tile_shards():
    from fastselect_amd import _lib
    from fastselect_amd.parallel import ShardedMultiSURF
    X, y, (x, yv, recip, isd) = _inputs(n=2100, p=300, seed=4)
    for star in (False, True):
        ref = _lib.multisurf_score("gpu", x, yv, recip, None, star, isd)
        job = ShardedMultiSURF(x, yv, recip, isd, use_star=star, backend="gpu", shard=False,
                               shards=3)
        s = job.step().cpu().numpy()
        s2 = job.step().cpu().numpy()  # a second step re-targets the shards again
        job.close()
        np.testing.assert_array_equal(s, s2)
        assert scale_rel_err(s, ref) < 1e-6
        assert set(np.argsort(s)[::-1][:10]) == set(np.argsort(ref)[::-1][:10])


def test_shard_count_follows_device_memory(hooks):
    from fastselect_amd import _lib
    hooks("shards", 0)
    assert _lib.multisurf_shards(20000, 20000) == 1          # cfg4: 3.2 GB of tiles
    assert _lib.multisurf_shards(400000, 20000) > 1          # ~1.3 TB of tiles
    assert _lib.multisurf_shards(400000, 20000, world=8) < _lib.multisurf_shards(400000, 20000)
