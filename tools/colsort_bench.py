"""Mean-correction kernels alone (k_colsort and friends) on a cfg4-shaped
column set: n = 20000 samples, p columns of make_classification data, a few
MultiSURF steps through ShardedMultiSURF (the side-stream kernels run beside
k_dist as in bench.py).  For rocprofv3 kernel traces / PMC passes.

    python tools/colsort_bench.py [n p steps family]
"""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    p = int(sys.argv[2]) if len(sys.argv) > 2 else 2048
    steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    fam = sys.argv[4] if len(sys.argv) > 4 else "gauss"
    from fastselect_amd import parallel
    rng = np.random.default_rng(1)
    if fam == "gauss":
        from sklearn.datasets import make_classification
        X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=100,
                                   random_state=42)
        X = X.astype(np.float32)
    else:  # lognormal: every column crowded
        X = np.exp(3.0 * rng.standard_normal((n, p), dtype=np.float32)).astype(np.float32)
        y = rng.integers(0, 2, n)
    x, yv, recip, isd = parallel.prepare_inputs(X, y, backend="gpu")
    job = parallel.ShardedMultiSURF(x, yv, recip, isd, backend="gpu", shard=False)
    import torch
    for _ in range(steps):
        job.step()
    torch.cuda.synchronize()
    print("done", job.plan.calibration()["q16"])
    job.close()


if __name__ == "__main__":
    main()
