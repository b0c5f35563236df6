"""Pair-weight density per 128 x 128 tile at cfg4 (would
scoring the densest tiles dense pay?).  Dense pass 2 (k_score) costs ~1/1.7
of the sparse loop per evaluated pair, so a tile is cheaper dense above ~58%
of its pairs weighted.  After one MultiSURF step the plan's row statistics
give every row's threshold (mu - sigma / 2 with the exact mean correction,
in real distance units: / SC); the distances of sampled row blocks against
all samples come from torch (float32 L1 over the scaled features, within
~1e-6 of the reference's, which moves a handful of pairs only); a pair
(i, j) carries a weight when D_ij < thr_i or D_ij < thr_j.

    python tools/tile_density.py [n p row_blocks]
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    p = int(sys.argv[2]) if len(sys.argv) > 2 else 20000
    nblk = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    import torch
    from sklearn.datasets import make_classification
    from fastselect_amd import parallel
    X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=100,
                               random_state=42)
    X = X.astype(np.float32)
    x, yv, recip, isd = parallel.prepare_inputs(X, y, backend="gpu")
    job = parallel.ShardedMultiSURF(x, yv, recip, isd, backend="gpu", shard=False)
    job.step()
    rs = job.rowstats.cpu().numpy().reshape(-1, 3).astype(np.float64)
    sc = job.plan.calibration()["SC"]
    job.close()
    mu = (rs[:, 0] - rs[:, 2]) / (n - 1)
    var = np.maximum(rs[:, 1] / (n - 1) - (rs[:, 0] / (n - 1)) ** 2, 0.0)
    thr = torch.tensor((mu - 0.5 * np.sqrt(var)) / sc, device="cuda", dtype=torch.float64)
    xs = torch.tensor(X, device="cuda") * torch.tensor(recip, device="cuda")
    T = 128
    nb = (n + T - 1) // T
    rng = np.random.default_rng(0)
    blocks = sorted(rng.choice(nb, size=min(nblk, nb), replace=False).tolist())
    dens = []
    for bi in blocks:
        i0, i1 = bi * T, min(n, bi * T + T)
        D = torch.zeros(i1 - i0, n, device="cuda", dtype=torch.float64)
        for f0 in range(0, p, 2048):
            D += torch.cdist(xs[i0:i1, f0:f0 + 2048], xs[:, f0:f0 + 2048], p=1).double()
        near = (D < thr[i0:i1, None]) | (D < thr[None, :])
        idx = torch.arange(i0, i1, device="cuda")[:, None]
        near &= idx != torch.arange(n, device="cuda")[None, :]
        for bj in range(nb):
            j0, j1 = bj * T, min(n, bj * T + T)
            m = near[:, j0:j1]
            pairs = (i1 - i0) * (j1 - j0) - ((i1 - i0) if bi == bj else 0)
            dens.append(float(m.sum().item()) / max(pairs, 1))
    d = np.array(dens)
    hist, edges = np.histogram(d, bins=20, range=(0.0, 1.0))
    print(json.dumps({"n": n, "p": p, "row_blocks": blocks, "tiles": int(d.size),
                      "mean": float(d.mean()), "std": float(d.std()), "min": float(d.min()),
                      "max": float(d.max()), "frac_tiles_above_0.58": float((d > 0.58).mean()),
                      "hist_5pct_bins": hist.tolist()}))


if __name__ == "__main__":
    main()
