"""bench.py's multi-rank launcher (``--gpus N`` without torch.distributed.run).

The GPU box has one MI355X, so the N > 1 path is rehearsed here on host
threads: ``--backend cpu`` runs the same sharded MultiSURF job (pair tiles
dealt over the ranks, three SUM all-reduces) over gloo.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def test_rank_envs_follow_torchrun_convention():
    envs = bench.rank_envs(3, 29511, base={"PATH": "/bin"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2"]
    for e in envs:
        assert e["WORLD_SIZE"] == "3" and e["LOCAL_WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29511"
        assert e["PATH"] == "/bin"


def _run(gpus, extra=()):
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "2"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--backend", "cpu",
           "--samples", "300", "--features", "160", "--steps", "2", "--warmup", "1",
           "--no-cpu-baseline", "--no-fit", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    return json.loads(lines[0])


def test_bench_gpus2_launches_two_ranks_cpu_rehearsal():
    one = _run(1)
    two = _run(2)
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["steps"] == 2 and two["value"] > 0
    assert "x2" in two["config"]["parallelism"] and "gloo" in two["config"]["parallelism"]
    assert one["roofline"] is None  # no GPU kernels timed in a CPU rehearsal


def test_bench_refuses_world_mismatch():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--backend", "cpu", "--samples", "300", "--features", "160"],
                       capture_output=True, text=True, env=env, timeout=300, cwd=ROOT)
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in r.stderr


def test_sharded_cpu_world2_matches_one_shot(tmp_path):
    """Two gloo ranks (as the bench launches them) give the one-shot scores."""
    script = tmp_path / "w2.py"
    script.write_text(f"""
import os, sys, numpy as np
sys.path.insert(0, {ROOT!r})
import torch.distributed as dist
from sklearn.datasets import make_classification
from fastselect_amd import _lib
from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
dist.init_process_group("gloo")
X, y = make_classification(n_samples=260, n_features=90, n_informative=10, random_state=3)
x, yv, recip, isd = prepare_inputs(X, y)
job = ShardedMultiSURF(x, yv, recip, isd, backend="cpu")
s = job.step().numpy()
ref = _lib.multisurf_score("cpu", x, yv, recip, None, False, isd)
assert np.abs(s - ref).max() <= 1e-6 * np.abs(ref).max(), np.abs(s - ref).max()
job.close()
dist.destroy_process_group()
""")
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE")}
    env["OMP_NUM_THREADS"] = "2"
    procs = [subprocess.Popen([sys.executable, str(script)], env=e, stdout=subprocess.PIPE,
                              stderr=subprocess.PIPE, text=True)
             for e in bench.rank_envs(2, _free_port(), base=env)]
    for p in procs:
        out, err = p.communicate(timeout=300)
        assert p.returncode == 0, err[-3000:]


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]
