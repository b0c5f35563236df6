"""Prints the 16-bit decision check (fs_multisurf_last_guard) of a GPU
MultiSURF fit at cfg4 (BASELINE configs[3]) and cfg2: the risk must stay
below the 5e-6 re-run bound on make_classification data."""
import json
import time

import numpy as np
from sklearn.datasets import make_classification

import fastselect_amd as F
from fastselect_amd import _lib

for n, p in ((20000, 20000), (5000, 5000)):
    X, y = make_classification(n_samples=n, n_features=p, n_informative=20, n_redundant=100,
                               random_state=42)
    X = X.astype(np.float32)
    t = time.time()
    F.MultiSURF(backend="gpu", n_features_to_select=10).fit(X, y)
    risk, rerun = _lib.multisurf_last_guard()
    print(json.dumps({"n": n, "p": p, "risk": risk, "rerun": rerun, "fit_s": time.time() - t}), flush=True)
