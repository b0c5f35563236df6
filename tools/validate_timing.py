"""Timing of validate_xy's pieces at cfg4 (float64 X -> float32)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from sklearn.datasets import make_classification
    from sklearn.utils.validation import validate_data

    import fastselect_amd as F
    from fastselect_amd import _base, _lib
    X, y = make_classification(n_samples=20000, n_features=20000, n_informative=20,
                               n_redundant=100, random_state=42)
    est = F.MultiSURF(backend="gpu")
    for rep in range(3):
        t0 = time.perf_counter()
        xc = _base.to_float32(X, -1)
        t1 = time.perf_counter()
        xv, yv = validate_data(est, xc, y, y_numeric=True, dtype=np.float32, ensure_2d=True,
                               ensure_all_finite=False)
        t2 = time.perf_counter()
        xv = np.ascontiguousarray(xv)
        ok = _lib.all_finite(xv, -1)
        t3 = time.perf_counter()
        print(f"inline   cast {1e3*(t1-t0):.1f} validate {1e3*(t2-t1):.1f} finite {1e3*(t3-t2):.1f} same={xv is xc}", flush=True)
        del xc, xv
    for rep in range(3):
        t0 = time.perf_counter()
        xv, yv = _base.validate_xy(est, X, y, np.float32, -1)
        t1 = time.perf_counter()
        print(f"validate_xy {1e3*(t1-t0):.1f}", flush=True)
        del xv
    for rep in range(3):
        t0 = time.perf_counter()
        xc = _base.to_float32(X, -1)
        t1 = time.perf_counter()
        print(f"to_float32 alone {1e3*(t1-t0):.1f}", flush=True)
        del xc


if __name__ == "__main__":
    main()
