"""Time every BASELINE.json config through the product entry points.

    python tools/bench_configs.py [--only cfg2,cfg3,...] [--repeat 2]

Per config: the one-shot C-ABI call (device alloc + H2D + all kernels + D2H,
the same call an estimator's fit makes), the estimator's whole fit() and,
for the MultiSURF configs, the kernel-only step of a resident plan.  Prints one JSON line per config.
Data: make_classification(n_informative=20, n_redundant=R, random_state=42)
as in SURVEY.md §8d.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

CONFIGS = {
    "cfg1": dict(algo="multisurf", n=500, p=1000, R=100),
    "cfg2": dict(algo="multisurf", n=5000, p=5000, R=100),
    "cfg3": dict(algo="relieff", n=20000, p=2000, R=50, k=10),
    "cfg3c": dict(algo="relieff", n=20000, p=2000, R=50, k=10, classes=3),
    "cfg4": dict(algo="multisurf", n=20000, p=20000, R=100),
    "cfg5s": dict(algo="surf", n=10000, p=50000, R=100, star=True),
    "cfg5m": dict(algo="multisurf", n=10000, p=50000, R=100, star=True),
    # SURF (no star) on cfg5's data: the sparse pass-2 choice for plain SURF
    "cfg5surf": dict(algo="surf", n=10000, p=50000, R=100, star=False),
    # TuRF over MultiSURF on cfg2's data: device-resident re-targeting vs refits
    "turf2": dict(algo="turf", n=5000, p=5000, R=100),
    # TuRF over ReliefF (k=10) on cfg3's data
    "turf3": dict(algo="turf", base="ReliefF", n=20000, p=2000, R=50, k=10),
}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default=",".join(CONFIGS))
    ap.add_argument("--repeat", type=int, default=2)
    args = ap.parse_args()
    from sklearn.datasets import make_classification

    from fastselect_amd import _lib
    for name in args.only.split(","):
        c = CONFIGS[name]
        t0 = time.perf_counter()
        X, y = make_classification(n_samples=c["n"], n_features=c["p"], n_informative=20,
                                   n_redundant=c["R"], n_classes=c.get("classes", 2),
                                   random_state=42)
        t_data = time.perf_counter() - t0
        n, p = X.shape
        x32 = X.astype(np.float32)
        r = (x32.max(0) - x32.min(0)).astype(np.float32)
        r[r == 0] = 1
        recip = (1 / r).astype(np.float32)
        isd = np.zeros(p, bool)
        star = c.get("star", False)
        if c["algo"] == "turf":
            import fastselect_amd as F

            cls = getattr(F, c.get("base", "MultiSURF"))
            ekw = {"n_neighbors": c["k"]} if "k" in c else {}

            class Refit(cls):
                _resident_scorer = None

            out = {"config": name, **c, "data_s": t_data}
            for label, base in (("resident", cls), ("refit", Refit)):
                t0 = time.perf_counter()
                tf = F.TuRF(base(backend="gpu", **ekw), n_features_to_select=10,
                            pct_remove=0.1).fit(X, y)
                out[f"{label}_s"] = time.perf_counter() - t0
                out[f"{label}_top"] = tf.top_features_.tolist()
            print(json.dumps(out), flush=True)
            continue
        times = []
        for _ in range(args.repeat):
            t0 = time.perf_counter()
            if c["algo"] == "multisurf":
                _lib.multisurf_score("gpu", x32, y, recip, None, star, isd)
            elif c["algo"] == "surf":
                _lib.surf_score("gpu", X, y.astype(np.int32), recip, star, isd)
            else:
                classes, y_enc = np.unique(y, return_inverse=True)
                prior = (np.bincount(y_enc) / n).astype(np.float32)
                _lib.relieff_score("gpu", x32, y_enc.astype(np.int32), recip, isd, c["k"], prior)
            times.append(time.perf_counter() - t0)
        out = {"config": name, **c, "oneshot_s": min(times), "feature_scores_per_s": n * p / min(times),
               "data_s": t_data}
        # estimator fit(): validation, column statistics, scoring, ranking
        import fastselect_amd as F
        est = {"multisurf": lambda: F.MultiSURF(backend="gpu", use_star=star, n_features_to_select=10),
               "surf": lambda: F.SURF(backend="gpu", use_star=star, n_features_to_select=10),
               "relieff": lambda: F.ReliefF(backend="gpu", n_neighbors=c.get("k", 10),
                                            n_features_to_select=10)}[c["algo"]]
        Xin = x32 if c["algo"] == "multisurf" else X
        t0 = time.perf_counter()
        est().fit(Xin, y)
        out["fit_s"] = time.perf_counter() - t0
        if c["algo"] == "multisurf":
            import torch

            from fastselect_amd.parallel import ShardedMultiSURF
            job = ShardedMultiSURF(x32, y, recip, isd, use_star=star)
            job.step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.repeat):
                job.step()
            torch.cuda.synchronize()
            out["step_s"] = (time.perf_counter() - t0) / args.repeat
            out["k_dist_ms"], out["k_score_ms"] = job.kernel_ms(0), job.kernel_ms(1)
            job.close()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
