"""Median fit() time of MultiSURF(backend='gpu') on cfg4 from float64 and
from float32 X (5 runs after 1 warm-up each), one JSON line.  Imports the
fastselect_amd package of the current directory."""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.getcwd())


def main():
    from sklearn.datasets import make_classification

    from fastselect_amd import MultiSURF
    X, y = make_classification(n_samples=20000, n_features=20000, n_informative=20,
                               n_redundant=100, random_state=42)
    out = {}
    for name, x in (("f64", X), ("f32", X.astype(np.float32))):
        ts = []
        for r in range(6):
            t0 = time.perf_counter()
            MultiSURF(n_features_to_select=10, backend="gpu").fit(x, y)
            ts.append((time.perf_counter() - t0) * 1e3)
        out[name] = round(float(np.median(ts[1:])), 1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
