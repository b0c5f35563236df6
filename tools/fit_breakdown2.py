"""fit() at cfg4 from the float64 make_classification output (bench.py's
fit_ms), phase by phase: the float32 cast, validation, the staged upload,
column statistics, the plan (FS_TRACE phases on stderr), ranking."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from sklearn.datasets import make_classification

    import fastselect_amd as F
    from fastselect_amd import _base, _lib
    X, y = make_classification(n_samples=20000, n_features=20000, n_informative=20,
                               n_redundant=100, random_state=42)
    est = F.MultiSURF(backend="gpu", n_features_to_select=10)
    est.fit(X, y)  # warm-up (device block cache)
    for rep in range(2):
        t = {}
        t0 = time.perf_counter()
        x32 = _base.to_float32(X)
        t["cast"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        xv, yv = _base.validate_xy(est, x32, y, np.float32)
        t["validate_xy(f32)"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        with _lib.staged_x("gpu", xv):
            t["stage"] = time.perf_counter() - t0
            t0 = time.perf_counter()
            isd, mn, mx = _base.column_preprocess(xv, 10, "gpu")
            t["column_stats"] = time.perf_counter() - t0
            r = (mx - mn).astype(np.float32)
            r[r == 0] = 1
            recip = (1 / r).astype(np.float32)
            t0 = time.perf_counter()
            s = _lib.multisurf_score("gpu", xv, yv, recip, np.arange(xv.shape[1]), False, isd)
            t["score"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        _base.top_features(s, 10)
        t["rank"] = time.perf_counter() - t0
        t0 = time.perf_counter()
        est.fit(X, y)
        t["fit(float64 X)"] = time.perf_counter() - t0
        print(rep, " ".join(f"{k} {v * 1e3:.1f} ms" for k, v in t.items()), flush=True)


if __name__ == "__main__":
    main()
