"""Share of the unordered pairs that are near one of their two samples at a
BASELINE config (MultiSURF: D < mu - sigma/2; SURF: D < the row mean) -- the
pairs a near-only sparse pass 2 would evaluate.  Uses the non-star
algorithms, whose non-zero pair weights are exactly those pairs
(fs_plan_weighted_pairs, sparse pass 2 forced).

    python tools/near_density.py --config cfg5m
"""
import argparse
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", default="cfg5m")
    a = ap.parse_args()
    import torch

    import bench
    from fastselect_amd import _lib
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    cfg = bench.CONFIGS[a.config]
    n, p = cfg["n"], cfg["p"]
    X, y = bench.make_data(n, p, 42, cfg["red"])
    pairs = n * (n - 1) / 2
    _lib.set_test_hook("sparse", 1)
    x, yv, recip, isd = prepare_inputs(X.astype(np.float32), y, backend="gpu")
    job = ShardedMultiSURF(x, yv, recip, isd, use_star=False, backend="gpu", shard=False)
    job.step()
    torch.cuda.synchronize()
    print(f"{a.config} MultiSURF near pairs: {job.plan.weighted_pairs() / pairs:.3f} of {pairs:.3e}",
          flush=True)
    job.close()
    from fastselect_amd.SURF import surf_inputs
    xin = np.ascontiguousarray(X, dtype=np.float64)
    sisd, srecip = surf_inputs(xin, 10, "gpu")
    plan = _lib.RowsPlan("gpu", "surf", xin, np.asarray(y).astype(np.int32), srecip, sisd,
                         use_star=False)
    sums = torch.zeros(p, dtype=torch.float64, device="cuda")
    plan.score(sums.data_ptr())
    torch.cuda.synchronize()
    print(f"{a.config} SURF near pairs: {plan.weighted_pairs() / pairs:.3f}", flush=True)
    plan.close()
    _lib.set_test_hook("reset", 0)


if __name__ == "__main__":
    main()
