import time, numpy as np, sys
sys.path.insert(0, '.')
from sklearn.datasets import make_classification
import fastselect_amd as F
from fastselect_amd import _base
from fastselect_amd.ReliefF import relieff_inputs
X, y = make_classification(n_samples=20000, n_features=2000, n_informative=20, n_redundant=50, random_state=42)
F.ReliefF(n_neighbors=10, backend="gpu").fit(X, y)
t = time.perf_counter(); F.ReliefF(n_neighbors=10, backend="gpu").fit(X, y); print("fit", time.perf_counter() - t)
est = F.ReliefF(n_neighbors=10, backend="gpu")
t = time.perf_counter(); xv, yv = _base.validate_xy(est, X, y, np.float64); print("validate", time.perf_counter() - t)
t = time.perf_counter(); out = relieff_inputs(xv, yv, 10, "gpu"); print("relieff_inputs", time.perf_counter() - t)
t = time.perf_counter(); x32 = np.ascontiguousarray(xv, dtype=np.float32); print("cast", time.perf_counter() - t)
t = time.perf_counter(); _base.column_preprocess(xv, 10, "gpu"); print("colstats", time.perf_counter() - t)
