"""Time one rank's share of a world-N MultiSURF step on one GPU (what each
rank of an N-GPU run executes, minus the collectives).

    python tools/shard_profile.py --world 8 [--samples 20000 --features 20000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--samples", type=int, default=20000)
    ap.add_argument("--features", type=int, default=20000)
    ap.add_argument("--steps", type=int, default=3)
    args = ap.parse_args()
    import torch
    from sklearn.datasets import make_classification

    from fastselect_amd import _lib
    X, y = make_classification(n_samples=args.samples, n_features=args.features,
                               n_informative=20, n_redundant=100, random_state=42)
    x = X.astype(np.float32)
    r = (x.max(0) - x.min(0)).astype(np.float32)
    r[r == 0] = 1
    recip = (1 / r).astype(np.float32)
    isd = np.zeros(args.features, bool)
    n = args.samples
    stream = torch.cuda.current_stream().cuda_stream
    # The exchanged vectors (row moments, neighbour counts) of the whole job,
    # from a world-1 plan, stand in for the all-reduces: the rank's sparse
    # pass 2 then sees the real pair weights.
    rs_all = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
    cn_all = torch.zeros(2 * n, dtype=torch.float64, device="cuda")
    sc = torch.zeros(args.features, dtype=torch.float64, device="cuda")
    full = _lib.Plan("gpu", x, y, recip, isd, stream=stream)
    full.pass1(rs_all.data_ptr())
    full.select(rs_all.data_ptr(), cn_all.data_ptr())
    torch.cuda.synchronize()
    full.close()
    plan = _lib.Plan("gpu", x, y, recip, isd, rank=args.rank, world=args.world, stream=stream)
    rs = torch.zeros(3 * n, dtype=torch.float64, device="cuda")
    cn = torch.zeros(2 * n, dtype=torch.float64, device="cuda")

    def step():
        plan.pass1(rs.data_ptr())
        plan.select(rs_all.data_ptr(), cn.data_ptr())
        plan.pass2(cn_all.data_ptr(), sc.data_ptr())

    step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / args.steps
    tiles, _, refined = plan.info()
    print(json.dumps({"world": args.world, "rank": args.rank, "tiles": tiles, "step_ms": dt * 1e3,
                      "k_dist_ms": plan.kernel_ms(0), "k_score_ms": plan.kernel_ms(1),
                      "refined": refined, "weighted_pairs": plan.weighted_pairs()}))


if __name__ == "__main__":
    main()
