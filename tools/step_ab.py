"""Same-process A/B of a MultiSURF step under test hooks: each variant's
resident step timed over --steps (after --warmup), variants alternated
--rounds times so clock drift hits them alike.

    python tools/step_ab.py --config cfg2 --variants "base;ksplit=1;ksplit=2"
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg2")
    ap.add_argument("--variants", default="base")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--nostar", action="store_true", help="the config's algorithm without star")
    a = ap.parse_args()
    import numpy as np
    import torch

    import bench
    from fastselect_amd import _lib
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    cfg = dict(bench.CONFIGS[a.config])
    if a.nostar:
        cfg["star"] = False
    X, y = bench.make_data(cfg["n"], cfg["p"], 42, cfg["red"])
    surf = cfg["algo"] == "surf"
    if surf:  # a resident SURF row plan (bench.py's cfg5s step)
        from fastselect_amd.SURF import surf_inputs
        xin = np.ascontiguousarray(X, dtype=np.float64)
        sisd, srecip = surf_inputs(xin, 10, "gpu")
        sums = torch.zeros(cfg["p"], dtype=torch.float64, device="cuda")
    else:
        x, yv, recip, isd = prepare_inputs(X.astype(np.float32), y, backend="gpu")
    variants = []
    for v in a.variants.split(";"):
        hooks = []
        if v != "base":
            for kv in v.split(","):
                k, val = kv.split("=")
                hooks.append((k, int(val)))
        variants.append((v, hooks))
    res = {v: [] for v, _ in variants}
    for _ in range(a.rounds):
        for v, hooks in variants:
            _lib.set_test_hook("reset", 0)
            for k, val in hooks:
                _lib.set_test_hook(k, val)
            if surf:
                job = _lib.RowsPlan("gpu", "surf", xin, np.asarray(y).astype(np.int32), srecip,
                                    sisd, use_star=cfg["star"])
                step = lambda: job.score(sums.data_ptr())  # noqa: E731
            else:
                job = ShardedMultiSURF(x, yv, recip, isd, use_star=cfg["star"], backend="gpu",
                                       shard=False)
                step = job.step
            for _ in range(a.warmup):
                step()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(a.steps):
                step()
            torch.cuda.synchronize()
            res[v].append((time.perf_counter() - t) / a.steps * 1e3)
            job.close()
    _lib.set_test_hook("reset", 0)
    for v, _ in variants:
        print(f"{a.config} {v:24s} " + " ".join(f"{t:8.3f}" for t in res[v]) +
              f"   min {min(res[v]):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
