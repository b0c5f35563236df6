"""Where a MultiSURF.fit() at cfg4 spends its time (host validation, column
statistics, scoring call), with FS_TRACE phases from the native library."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from sklearn.datasets import make_classification
    from sklearn.utils.validation import check_array

    import fastselect_amd as F
    from fastselect_amd import _base, _lib
    X, y = make_classification(n_samples=20000, n_features=20000, n_informative=20,
                               n_redundant=100, random_state=42)
    x = X.astype(np.float32)
    F.MultiSURF(backend="gpu").fit(x[:500, :500], y[:500])  # warm-up
    t0 = time.perf_counter()
    F.MultiSURF(backend="gpu").fit(x, y)
    print(f"fit total            {time.perf_counter() - t0:8.3f} s")
    t0 = time.perf_counter()
    check_array(x, dtype=np.float32)
    print(f"check_array          {time.perf_counter() - t0:8.3f} s")
    t0 = time.perf_counter()
    isd, mn, mx = _base.column_preprocess(x, 10, "gpu")
    print(f"column_preprocess    {time.perf_counter() - t0:8.3f} s")
    r = (mx - mn).astype(np.float32)
    r[r == 0] = 1
    recip = (1 / r).astype(np.float32)
    t0 = time.perf_counter()
    _lib.multisurf_score("gpu", x, y, recip, np.arange(x.shape[1]), False, isd)
    print(f"multisurf_score      {time.perf_counter() - t0:8.3f} s")


if __name__ == "__main__":
    main()
