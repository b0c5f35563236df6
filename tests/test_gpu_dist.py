"""RCCL (torch.distributed 'nccl' backend) on the GPU box.

The box has one MI355X, so the collective path runs at world 1: the process
group is up, every exchange point of ShardedMultiSURF.step() (rowstats,
counts, scores) goes through dist.all_reduce over RCCL, and the result must
equal the single-device C-ABI call bit for bit (an all-reduce over one rank
is the identity).  N > 1 is covered by the gloo tests (tests/test_bench.py,
test_parity_cpu.py, test_rows.py) and the driver's multi-GPU bench.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_nccl_world1_step_matches_one_shot():
    import torch
    import torch.distributed as dist
    from sklearn.datasets import make_classification

    from fastselect_amd import _lib
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        assert dist.get_backend() == "nccl"
        X, y = make_classification(n_samples=1500, n_features=700, n_informative=20,
                                   n_redundant=40, random_state=5)
        x, yv, recip, isd = prepare_inputs(X, y, backend="gpu", device=0)
        job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", device=0)
        assert job.dist is not None and job.world == 1
        s = job.step().cpu().numpy()
        job.close()
        ref = _lib.multisurf_score("gpu", x, yv, recip, None, False, isd)
        np.testing.assert_array_equal(s, ref)
        # the one-call RCCL all-reduce helper of the row-sharded algorithms
        from fastselect_amd import parallel
        v = np.arange(7, dtype=np.float64)
        np.testing.assert_array_equal(parallel._allreduce_sums(v, "gpu", 0), v)
    finally:
        dist.destroy_process_group()


def test_nccl_gathered_x_matches_uploaded_x():
    """The multi-GPU data path at world 1: X assembled on the device by the
    RCCL all-gather (gather_rows) and registered for the column statistics
    and the plan (fs_stage_x_device) gives bit-identical scores to the plain
    upload."""
    import torch
    import torch.distributed as dist
    from sklearn.datasets import make_classification

    from fastselect_amd import _lib
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs, resident_x

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        X, y = make_classification(n_samples=1000, n_features=300, n_informative=20,
                                   n_redundant=40, random_state=9)
        x = np.ascontiguousarray(X, dtype=np.float32)
        with resident_x(x, "gpu", 0, gather=True):
            xi, yv, recip, isd = prepare_inputs(x, y, backend="gpu", device=0)
            job = ShardedMultiSURF(xi, yv, recip, isd, backend="gpu", device=0)
            s = job.step().cpu().numpy()
            job.close()
        ref = _lib.multisurf_score("gpu", x, yv, recip, None, False, isd)
        np.testing.assert_array_equal(s, ref)
    finally:
        dist.destroy_process_group()


def test_nccl_gathered_rows_relieff_surf():
    """ReliefF and SURF's row-sharded jobs through the multi-GPU data path at
    world 1: X's float64 rows all-gathered over RCCL
    and registered for the column statistics, SURF's plan reading them and
    ReliefF's float32 copy cast on the device -- bit-identical scores to the
    per-rank upload (gather=False)."""
    import torch
    import torch.distributed as dist
    from sklearn.datasets import make_classification

    from fastselect_amd import parallel

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        X, y = make_classification(n_samples=1300, n_features=240, n_informative=15,
                                   n_redundant=30, n_classes=3, random_state=5)
        X[:, :6] = np.round(X[:, :6])          # discrete columns too
        for fn, kw in ((parallel.relieff_scores, {"n_neighbors": 6}),
                       (parallel.surf_scores, {"use_star": True})):
            a = fn(X, y, backend="gpu", device=0, gather=True, **kw)
            b = fn(X, y, backend="gpu", device=0, gather=False, **kw)
            np.testing.assert_array_equal(a, b)
    finally:
        dist.destroy_process_group()


def test_column_stats_run_on_the_ranks_device():
    """prepare_inputs(device=d) computes the column statistics on GPU d
    (they used to default to GPU 0 on every rank)."""
    import torch
    from fastselect_amd.parallel import prepare_inputs
    d = torch.cuda.device_count() - 1
    X = np.random.default_rng(0).normal(size=(300, 50))
    x, _, recip, isd = prepare_inputs(X, np.arange(300) % 2, backend="gpu", device=d)
    rng = (x.max(0) - x.min(0)).astype(np.float32)
    np.testing.assert_array_equal(recip, (1.0 / rng).astype(np.float32))
    assert not isd.any()


def test_pinned_float32_cast_equals_numpy():
    """_base.to_float32 with a GPU visible casts into pinned host memory
    (fs_host_alloc); the values are numpy's cast, and blocks are reused."""
    from fastselect_amd import _base
    rng = np.random.default_rng(8)
    x = rng.normal(size=(3000, 2000)) * 10.0 ** rng.integers(-20, 20, size=(3000, 2000))
    for _ in range(3):
        got = _base.to_float32(x)
        assert got.flags.c_contiguous and got.dtype == np.float32
        np.testing.assert_array_equal(got, x.astype(np.float32))
        del got


def _uniform_family():
    import importlib.util
    here = os.path.dirname(os.path.abspath(__file__))
    spec = importlib.util.spec_from_file_location("mk_families",
                                                  os.path.join(here, "golden", "make_families.py"))
    mk = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mk)
    return mk.make("uniform_16k")


def test_nccl_world1_decision_check_reruns():
    """The 16-bit decision check on the RCCL path: on
    signal-free data the all-reduced risk trips it, the plan moves to 32-bit
    operands and the step runs again -- the result is the one-shot fit's."""
    import torch
    import torch.distributed as dist

    import fastselect_amd as F
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs

    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ["MASTER_PORT"] = str(_port())
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    try:
        X, y = _uniform_family()
        x, yv, recip, isd = prepare_inputs(X, y, backend="gpu", device=0)
        job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", device=0)
        assert job.dist is not None
        s = job.step().cpu().numpy()
        risk, switched = job.last_guard
        job.close()
    finally:
        dist.destroy_process_group()
    assert risk > 5e-6 and switched
    one = F.MultiSURF(backend="gpu", n_features_to_select=10).fit(X, y).feature_importances_
    np.testing.assert_array_equal(s, one)


def _guard_rank_worker(rank, world, port, out_path):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    X, y = _uniform_family()
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu", device=0)
    job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", device=0)
    s = job.step().cpu().numpy()
    np.save(f"{out_path}.{rank}.npy", s)
    np.save(f"{out_path}.{rank}.guard.npy", np.array(job.last_guard, dtype=np.float64))
    job.close()
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_decide_the_rerun_together(tmp_path):
    """World 2 (two ranks sharing cuda:0, gloo): each rank holds half the
    tiles, both see the same all-reduced risk and re-run on 32-bit operands
    together; both end with the one-shot fit's scores."""
    import torch.multiprocessing as mp

    import fastselect_amd as F
    out = str(tmp_path / "guard")
    mp.spawn(_guard_rank_worker, args=(2, _port(), out), nprocs=2, join=True)
    a, b = np.load(out + ".0.npy"), np.load(out + ".1.npy")
    ga, gb = np.load(out + ".0.guard.npy"), np.load(out + ".1.guard.npy")
    np.testing.assert_array_equal(ga, gb)
    assert ga[0] > 5e-6 and ga[1] == 1.0
    np.testing.assert_array_equal(a, b)
    X, y = _uniform_family()
    one = F.MultiSURF(backend="gpu", n_features_to_select=10).fit(X, y).feature_importances_
    assert np.max(np.abs(a - one)) <= 1e-6 * np.max(np.abs(one))


def test_job_on_a_caller_stream_matches_one_shot():
    """ShardedMultiSURF on a caller's non-default stream runs its plan and
    buffers there (with torch's default stream it makes a stream of its own):
    the scores are the one-shot call's either way, and the result is ready on
    the caller's stream."""
    import torch
    from sklearn.datasets import make_classification

    from fastselect_amd import _lib
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs

    X, y = make_classification(n_samples=1200, n_features=300, n_informative=20,
                               n_redundant=30, random_state=11)
    x, yv, recip, isd = prepare_inputs(X, y, backend="gpu", device=0)
    ref = _lib.multisurf_score("gpu", x, yv, recip, None, False, isd)
    torch.cuda.set_device(0)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", device=0, shard=False)
        assert job.stream == s
        got = job.step().cpu().numpy()
        job.close()
    np.testing.assert_array_equal(got, ref)
    job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", device=0, shard=False)
    assert job.stream.cuda_stream != 0
    got = job.step().cpu().numpy()
    job.close()
    np.testing.assert_array_equal(got, ref)
