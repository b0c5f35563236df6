"""ReliefF on discrete (SNP-like, values 0/1/2) and mixed data: tie rows
(every row, on all-discrete data) and where the step's time goes, from the
native library's FS_TRACE lines.  Usage: FS_TRACE=1 python3 tools/rf_discrete_time.py [n] [p]"""
import sys
import time

import numpy as np

sys.path.insert(0, ".")
import fastselect_amd as F  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
p = int(sys.argv[2]) if len(sys.argv) > 2 else 2000
rng = np.random.default_rng(0)
X = rng.integers(0, 3, size=(n, p)).astype(np.float64)
y = rng.integers(0, 2, n)
X[:, :20] = (X[:, :20] + y[:, None]) % 3  # a few informative SNPs
for rep in range(2):
    t = time.perf_counter()
    est = F.ReliefF(n_neighbors=10, backend="gpu").fit(X, y)
    print(f"discrete n={n} p={p} fit {time.perf_counter() - t:.3f} s", flush=True)
print("top-10", sorted(np.argsort(est.feature_importances_)[::-1][:10].tolist()))
