"""Reference-order chains in isolation, for kernel traces and PMC passes:
MultiSURF (k_ms_chains) at cfg4's shape scaled down and SURF* (k_surf_chains)
at cfg5's, one resident plan each, `--reps` scoring passes.

    python tools/chains_probe.py [--n 8192] [--p 8192] [--reps 3] [--algo ms,surf]
"""
import argparse
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=8192)
    ap.add_argument("--p", type=int, default=8192)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--algo", default="ms,surf")
    a = ap.parse_args()
    import torch
    from sklearn.datasets import make_classification

    from fastselect_amd import _lib
    from fastselect_amd.SURF import surf_inputs
    from fastselect_amd.parallel import ShardedMultiSURF, prepare_inputs
    X, y = make_classification(n_samples=a.n, n_features=a.p, n_informative=20,
                               n_redundant=min(100, a.p // 4), random_state=42)
    for algo in a.algo.split(","):
        if algo == "ms":
            x, yv, recip, isd = prepare_inputs(X.astype(np.float32), y, backend="gpu")
            job = ShardedMultiSURF(x, yv, recip, isd, backend="gpu", shard=False,
                                   accumulation="reference")
            job.step()
            torch.cuda.synchronize()
            t = time.perf_counter()
            for _ in range(a.reps):
                job.step()
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t) / a.reps * 1e3
            print(f"multisurf reference n={a.n} p={a.p}: {ms:.2f} ms/step, chains "
                  f"{job.kernel_ms(1):.2f} ms", flush=True)
            job.close()
        else:
            x = np.ascontiguousarray(X, dtype=np.float64)
            isd, recip = surf_inputs(x, 10, "gpu")
            with _lib.accumulation("reference"):
                plan = _lib.RowsPlan("gpu", "surf", x, y.astype(np.int32), recip, isd,
                                     use_star=True)
            sums = torch.zeros(a.p, dtype=torch.float64, device="cuda")
            plan.score(sums.data_ptr())
            t = time.perf_counter()
            for _ in range(a.reps):
                plan.score(sums.data_ptr())
            ms = (time.perf_counter() - t) / a.reps * 1e3
            print(f"surf* reference n={a.n} p={a.p}: {ms:.2f} ms/score, masks + chains "
                  f"{plan.kernel_ms(1):.2f} ms", flush=True)
            plan.close()


if __name__ == "__main__":
    main()
