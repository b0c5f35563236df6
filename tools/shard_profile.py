"""Time one rank's share of a world-N MultiSURF step on one GPU (what each
rank of an N-GPU run executes, minus the collectives), and add a model of
the step's three SUM all-reduces (rowstats 3n, counts 2n, scores p float64)
so the projected per-rank step covers the whole exchange: ring all-reduce
2 (N-1) / N * bytes / link_bw + 2 (N-1) * hop_latency, with conservative
xGMI figures (50 GB/s effective per ring direction -- a third of the
153 GB/s link -- and 10 us per ring step; measured RCCL small-message
latency on MI300-class nodes is below that).  Not measured: this box has one
GPU.

    python tools/shard_profile.py --world 8 [--samples 20000 --features 20000]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


LINK_BW = 50e9   # bytes/s per ring direction (conservative xGMI figure)
HOP_S = 10e-6    # seconds per ring step (conservative RCCL latency)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rank", type=int, default=0)
    ap.add_argument("--samples", type=int, default=20000)
    ap.add_argument("--features", type=int, default=20000)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--world1", action="store_true", help="also time the whole job (world 1)")
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
    N = args.world
    ar_bytes = [3 * n * 8, 2 * n * 8, args.features * 8]
    ar_ms = sum(2 * (N - 1) / N * b / LINK_BW + 2 * (N - 1) * HOP_S for b in ar_bytes) * 1e3 \
        if N > 1 else 0.0
    print(json.dumps({"world": args.world, "rank": args.rank, "tiles": tiles, "step_ms": dt * 1e3,
                      "k_dist_ms": plan.kernel_ms(0), "k_score_ms": plan.kernel_ms(1),
                      "refined": refined, "weighted_pairs": plan.weighted_pairs(),
                      "allreduce_model_ms": ar_ms, "step_with_allreduce_ms": dt * 1e3 + ar_ms,
                      "allreduce_model": f"ring, {LINK_BW / 1e9:.0f} GB/s, {HOP_S * 1e6:.0f} us "
                                         f"per step, bytes {ar_bytes}"}))


if __name__ == "__main__":
    main()
